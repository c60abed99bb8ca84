"""Attention kernel times at the step's shape with attention dropout on (0.1, the hub config)
and off: how much of each kernel is the counter-hash dropout mask."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "noise-robust-speech-embedding_amd"))
import torch
from nrse_amd import kernels as K, _lib
_lib.init_device(0)
B, T, H = 32, 399, 16
dev = "cuda"
def rnd(*s, scale=1.0):
    return ((torch.rand(*s, device=dev) * 2 - 1) * scale).to(torch.bfloat16)
qkv = rnd(B * T, 3 * H * 64)
gate = torch.rand(B, H, T, device=dev) + 0.5
bias = None
bvec = torch.randn(H, 2 * T - 1, device=dev)
ctx = torch.empty(B * T, H * 64, device=dev, dtype=torch.bfloat16)
lse = torch.empty(B, H, T, device=dev)
dctx = rnd(B * T, H * 64, scale=0.1)
delta = torch.empty(B, H, T, device=dev)
dqkv = torch.empty_like(qkv)
dgate = torch.empty(B, H, T, device=dev)
diag = torch.zeros(H, 2 * T - 1, device=dev)
def timeit(fn, iters=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3
for p in (0.0, 0.1):
    tf = timeit(lambda: K.attn_fwd(qkv, gate, bias, ctx, lse, B, T, H, p, 123, bias_vec=bvec))
    tb = timeit(lambda: K.attn_bwd(qkv, gate, bias, ctx, dctx, lse, delta, dqkv, dgate, diag, B, T, H, p, 123, bias_vec=bvec))
    print(f"dropout {p}: fwd {tf:.1f} us, bwd (q + kv) {tb:.1f} us", flush=True)
