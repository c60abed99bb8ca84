"""Micro-benchmark of the attention kernels at the WavLM-Large step shape (B=32, T=399, H=16)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "noise-robust-speech-embedding_amd"))
import torch
from nrse_amd import kernels as K, _lib

_lib.init_device(0)
dev = "cuda"
B, T, H = 32, 399, 16
qkv = (torch.randn(B * T, 3 * H * 64, device=dev) * 0.5).bfloat16()
gate = torch.rand(B, H, T, device=dev) + 1
bias = None
bvec = torch.randn(H, 2 * T - 1, device=dev)
ctx = torch.empty(B * T, H * 64, device=dev, dtype=torch.bfloat16)
lse = torch.empty(B, H, T, device=dev)
dctx = torch.randn_like(ctx)
dqkv = torch.empty_like(qkv)
dgate = torch.empty(B, H, T, device=dev)
diag = torch.zeros(H, 2 * T - 1, device=dev)
delta = torch.empty(B, H, T, device=dev)


def timeit(fn, iters=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / iters

for p in (0.0, 0.1):
    tf = timeit(lambda: K.attn_fwd(qkv, gate, bias, ctx, lse, B, T, H, p, 1, bias_vec=bvec))
    tb = timeit(lambda: K.attn_bwd(qkv, gate, bias, ctx, dctx, lse, delta, dqkv, dgate, diag, B, T, H, p, 1, bias_vec=bvec))
    tbn = timeit(lambda: K.attn_bwd(qkv, gate, bias, ctx, dctx, lse, delta, dqkv, dgate, None, B, T, H, p, 1, bias_vec=bvec))
    fl = 4.0 * B * H * T * T * 64
    print(f"p={p}: fwd {tf*1e3:.1f}us ({fl/tf/1e9:.0f} TF) | bwd {tb*1e3:.1f}us ({2.5*fl/tb/1e9:.0f} TF) | bwd no-diag {tbn*1e3:.1f}us", flush=True)

# the step's form: the forward records the dropout keep bits, the backward reads them
mask = torch.empty(K.attn_mask_elems(B, T, H), device=dev, dtype=torch.int16)
p = 0.1
tf = timeit(lambda: K.attn_fwd(qkv, gate, bias, ctx, lse, B, T, H, p, 1, bias_vec=bvec, drop_mask=mask))
tb = timeit(lambda: K.attn_bwd(qkv, gate, bias, ctx, dctx, lse, delta, dqkv, dgate, diag, B, T, H, p, 1, bias_vec=bvec,
                               drop_mask=mask))
fl = 4.0 * B * H * T * T * 64
print(f"p={p} recorded mask: fwd {tf*1e3:.1f}us ({fl/tf/1e9:.0f} TF) | bwd {tb*1e3:.1f}us ({2.5*fl/tb/1e9:.0f} TF)", flush=True)
# the mask computed ahead by its own kernel (alone here; in the step it runs beside the GEMMs) and
# read by the forward
tm = timeit(lambda: K.attn_dropout_mask(mask, B, T, H, p, 1))
tf2 = timeit(lambda: K.attn_fwd(qkv, gate, bias, ctx, lse, B, T, H, p, 1, bias_vec=bvec, drop_mask=mask, mask_in=True))
print(f"p={p} precomputed mask: mask kernel {tm*1e3:.1f}us | fwd {tf2*1e3:.1f}us ({fl/tf2/1e9:.0f} TF)", flush=True)
# the split-weight (bf16sw) step's form: the recorded mask plus the fp8 copy of ctx (ctx8)
ctx8 = torch.empty(B * T, H * 64, device=dev, dtype=K.FP8)
tf8 = timeit(lambda: K.attn_fwd(qkv, gate, bias, ctx, lse, B, T, H, p, 1, bias_vec=bvec, drop_mask=mask, ctx8=ctx8))
print(f"p={p} recorded mask + ctx8: fwd {tf8*1e3:.1f}us ({fl/tf8/1e9:.0f} TF)", flush=True)
