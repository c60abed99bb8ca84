"""Runs single hot kernels back to back on the step's WavLM-Large shapes (B=32, T=399, H=16,
bf16) for counter collection (tools/pmc_sq.sh): the forward GEMM shapes, the slab wgrad, and the
attention forward / backward."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "noise-robust-speech-embedding_amd"))
import torch
from nrse_amd import kernels as K, _lib

_lib.init_device(0)
reps = int(os.environ.get("REPS", "10"))
what = sys.argv[1] if len(sys.argv) > 1 else "all"
M = 12768
dev = "cuda"


def rnd(*s, scale=1.0):
    return ((torch.rand(*s, device=dev) * 2 - 1) * scale).to(torch.bfloat16)


if what in ("all", "gemm"):
    for N, Kd in ((3072, 1024), (1024, 1024), (4096, 1024), (1024, 4096)):
        a, w = rnd(M, Kd), rnd(N, Kd)
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        for _ in range(reps):
            K.linear_fwd(a, w, c)
    dy, x = rnd(M, 3072, scale=0.1), rnd(M, 1024)
    dw = torch.zeros(3072, 1024, device=dev)
    for _ in range(reps):
        K.linear_wgrad(dy, x, dw)
if what in ("all", "attn"):
    B, T, H = 32, 399, 16
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
    for _ in range(reps):
        K.attn_fwd(qkv, gate, bias, ctx, lse, B, T, H, 0.1, 123, bias_vec=bvec)
        K.attn_bwd(qkv, gate, bias, ctx, dctx, lse, delta, dqkv, dgate, diag, B, T, H, 0.1, 123, bias_vec=bvec)
torch.cuda.synchronize()
print("done", what)
