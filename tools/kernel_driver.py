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
    # the step's form: the forward records the dropout keep bits, the backward reads them
    mask = torch.empty(K.attn_mask_elems(B, T, H), device=dev, dtype=torch.int16)
    for _ in range(reps):
        K.attn_fwd(qkv, gate, bias, ctx, lse, B, T, H, 0.1, 123, bias_vec=bvec, drop_mask=mask)
        K.attn_bwd(qkv, gate, bias, ctx, dctx, lse, delta, dqkv, dgate, diag, B, T, H, 0.1, 123, bias_vec=bvec,
                   drop_mask=mask)
if what == "conv0":
    # conv0 (1 -> 512, k10 s5) + LN + GELU forward, and its backward with dy = the col2im fold
    # of conv1's dgrad [32 x 12799, 3 x 512] (bf16), as in the step
    L0, T0, T1 = 128000, 25599, 12799
    wav = torch.randn(32, L0, device=dev) * 0.1
    w0 = torch.randn(512, 10, device=dev) * 0.3
    g0 = torch.ones(512, device=dev); b0 = torch.zeros(512, device=dev)
    o0 = torch.empty(32 * T0, 512, device=dev, dtype=torch.bfloat16)
    m0 = torch.empty(32 * T0, device=dev); r0 = torch.empty(32 * T0, device=dev)
    col = rnd(32 * T1, 3 * 512)
    dw0 = torch.zeros(512, 10, device=dev); dg0 = torch.zeros(512, device=dev); db0 = torch.zeros(512, device=dev)
    for _ in range(reps):
        K.conv0_fwd(wav, w0, g0, b0, o0, m0, r0, T0, 10, 5, 1e-5)
        K.conv0_bwd(wav, w0, g0, b0, m0, r0, col, dw0, dg0, db0, T0, 10, 5, (3, 2, T1))
torch.cuda.synchronize()
print("done", what)
