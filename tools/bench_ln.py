"""LayerNorm backward in isolation at the step's shapes: the encoder layer form (12768 x 1024,
f32 dy / x / residual, fused bf16 dropout-cast + column sums) and the conv layer-1 form (32 x
12799 rows x 512, bf16 x, dy by col2im of a [32 x 6399, 3 x 512] bf16 dgrad output, GELU).
Prints us and effective GB/s (algorithmic bytes)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "noise-robust-speech-embedding_amd"))
import torch
from nrse_amd import _lib, kernels as K

_lib.init_device(0)
dev = "cuda"


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


rows, C = 12768, 1024
x = torch.randn(rows, C, device=dev); dy = torch.randn(rows, C, device=dev); r = torch.randn(rows, C, device=dev)
g = torch.ones(C, device=dev); b = torch.zeros(C, device=dev)
mean = torch.zeros(rows, device=dev); rstd = torch.ones(rows, device=dev)
dx = torch.empty(rows, C, device=dev); dv = torch.empty(rows, C, device=dev, dtype=torch.bfloat16)
dg = torch.zeros(C, device=dev); db = torch.zeros(C, device=dev); cs = torch.zeros(C, device=dev)
us = timeit(lambda: K.ln_bwd(dy, x, g, mean, rstd, dx, resid=r, dgamma=dg, dbeta=db, dv=dv, dv_colsum=cs, dv_p=0.1,
                             dv_seed=1))
byt = rows * C * (4 * 3 + 4 + 2)
print(f"encoder LN bwd 12768x1024 (+fused dv): {us:.1f} us  {byt / us / 1e3:.0f} GB/s", flush=True)
yb = torch.empty(rows, C, device=dev, dtype=torch.bfloat16)
us = timeit(lambda: K.ln_fwd(x, g, b, yb, mean, rstd, 1e-5))
byt = rows * C * (4 + 2)
print(f"encoder LN fwd 12768x1024 f32 -> bf16: {us:.1f} us  {byt / us / 1e3:.0f} GB/s", flush=True)
B, Tin, Tout, Cin, k, s = 32, 12799, 6399, 512, 3, 2
xc = torch.randn(B * Tin, Cin, device=dev).to(torch.bfloat16)
G = torch.randn(B * Tout, k * Cin, device=dev).to(torch.bfloat16)
gc = torch.ones(Cin, device=dev); bc = torch.zeros(Cin, device=dev)
mc = torch.zeros(B * Tin, device=dev); rc = torch.ones(B * Tin, device=dev)
dpre = torch.empty(B * Tin, Cin, device=dev, dtype=torch.bfloat16)
dgc = torch.zeros(Cin, device=dev); dbc = torch.zeros(Cin, device=dev)
us = timeit(lambda: K.ln_bwd(G, xc, gc, mc, rc, dpre, beta=bc, gelu=True, dgamma=dgc, dbeta=dbc, mode=_lib.DY_COL2IM,
                             col=(k, s, Tout, Tin), rows=B * Tin), iters=10)
byt = B * Tin * Cin * 2 * 2 + B * Tout * k * Cin * 2
print(f"conv1 LN+GELU bwd col2im 409568x512: {us:.1f} us  {byt / us / 1e3:.0f} GB/s", flush=True)
if os.environ.get("LN_VARIANTS"):
    us = timeit(lambda: K.ln_bwd(G, xc, gc, mc, rc, dpre, beta=bc, gelu=False, dgamma=dgc, dbeta=dbc,
                                 mode=_lib.DY_COL2IM, col=(k, s, Tout, Tin), rows=B * Tin), iters=10)
    print(f"  variant no GELU: {us:.1f} us", flush=True)
    dyd = torch.randn(B * Tin, Cin, device=dev).to(torch.bfloat16)
    us = timeit(lambda: K.ln_bwd(dyd, xc, gc, mc, rc, dpre, beta=bc, gelu=True, dgamma=dgc, dbeta=dbc), iters=10)
    print(f"  variant direct dy (bf16), GELU: {us:.1f} us", flush=True)
    us = timeit(lambda: K.ln_bwd(dyd, xc, gc, mc, rc, dpre), iters=10)
    print(f"  variant direct dy, no GELU, no dgamma: {us:.1f} us", flush=True)
# conv0 (1 -> 512, k10 s5) + LN + GELU backward, dy = col2im of conv1's dgrad [32 x 12799, 3 x 512]
L0, T0 = 128000, 25599
wav = torch.randn(32, L0, device=dev) * 0.1
w0 = torch.randn(512, 10, device=dev) * 0.3
g0 = torch.ones(512, device=dev); b0 = torch.zeros(512, device=dev)
o0 = torch.empty(32 * T0, 512, device=dev, dtype=torch.bfloat16)
m0 = torch.empty(32 * T0, device=dev); r0 = torch.empty(32 * T0, device=dev)
us = timeit(lambda: K.conv0_fwd(wav, w0, g0, b0, o0, m0, r0, T0, 10, 5, 1e-5), iters=10)
print(f"conv0 fwd 819168x512 (bf16 out): {us:.1f} us  {32 * T0 * 512 * 2 / us / 1e3:.0f} GB/s", flush=True)
o3 = torch.empty(3, 32 * T0, 512, device=dev, dtype=torch.bfloat16)
us = timeit(lambda: K.conv0_fwd(wav, w0, g0, b0, o3, m0, r0, T0, 10, 5, 1e-5, split3=True), iters=10)
print(f"conv0 fwd 819168x512 (bf16x3 out): {us:.1f} us  {3 * 32 * T0 * 512 * 2 / us / 1e3:.0f} GB/s", flush=True)
del o3
col0 = torch.randn(32 * Tin, 3 * 512, device=dev).to(torch.bfloat16)
dw0 = torch.zeros(512, 10, device=dev); dg0 = torch.zeros(512, device=dev); db0 = torch.zeros(512, device=dev)
us = timeit(lambda: K.conv0_bwd(wav, w0, g0, b0, m0, r0, col0, dw0, dg0, db0, T0, 10, 5, (3, 2, Tin)), iters=10)
print(f"conv0 bwd col2im 819168x512: {us:.1f} us  {32 * Tin * 3 * 512 * 2 / us / 1e3:.0f} GB/s (col read)", flush=True)
# conv-stack LN + GELU forward, bf16 in / out (conv1: 409568 x 512)
yc = torch.empty(B * Tin, Cin, device=dev, dtype=torch.bfloat16)
us = timeit(lambda: K.ln_fwd(xc, gc, bc, yc, mc, rc, 1e-5, gelu=True), iters=10)
print(f"conv1 LN+GELU fwd 409568x512 bf16: {us:.1f} us  {B * Tin * Cin * 4 / us / 1e3:.0f} GB/s", flush=True)
