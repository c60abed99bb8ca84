"""Grouped pos-conv (WavLM-Large: H = 1024, 16 groups x 64 channels, 128 taps, B = 32, T = 399)
forward as the step issues it: the sliding-window kernel (csrc/posconv.hip) vs the generic
LDS-DMA GEMM (NRSE_GEMM_GEN=2 path). Prints us and TFLOP/s (algorithmic 2*B*T*H*64*128)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "noise-robust-speech-embedding_amd"))
import torch
from nrse_amd import _lib, kernels as K

_lib.init_device(0)
dev = "cuda"
B, T, H, G, pk = 32, 399, 1024, 16, 128
cpg = H // G
hpad = (torch.randn(B, T + pk, H, device=dev) * 0.5).to(torch.bfloat16)
wf = (torch.randn(G, cpg, pk * cpg, device=dev) * 0.02).to(torch.bfloat16)
bias = torch.zeros(H, device=dev)
resid = torch.randn(B * T, H, device=dev)
out = torch.empty(B * T, H, device=dev)
pre = torch.empty(B * T, H, device=dev, dtype=torch.bfloat16)


def call():
    K.gemm(K.Operand(hpad, True, H, chunk_shift=6, ld_chunk=H, z1=(T + pk) * H, z2=cpg),
           K.Operand(wf, True, pk * cpg, z2=cpg * pk * cpg), out, T, cpg, pk * cpg, ldc=H, batch=B * G, zdiv=G,
           c_z1=T * H, c_z2=cpg, bias=bias, bias_z2=cpg, flags=_lib.EPI_GELU | _lib.EPI_DROP_AFTER, aux=pre,
           ldaux=H, aux_z1=T * H, aux_z2=cpg, resid=resid, ldr=H, r_z1=T * H, r_z2=cpg, dropout_p=0.1, seed=3)


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


flops = 2.0 * B * T * H * cpg * pk
for gen, name in ((0, "sliding-window posconv"), (2, "generic LDS-DMA GEMM")):
    prev = K.gemm_select(gen)
    us = timeit(call)
    K.gemm_select(prev)
    print(f"{name}: {us:.1f} us  {flops / us / 1e6:.0f} TFLOP/s", flush=True)

# weight gradient as encoder_backward issues it (f32 atomics into a zeroed dWf; the zeroing is
# part of the timed call for both kernels)
lead = pk // 2 - 1
dypad = (torch.randn(B, T + pk, H, device=dev) * 0.5).to(torch.bfloat16)
dWf = torch.zeros(G, cpg, pk * cpg, device=dev)


def wcall():
    dWf.zero_()
    K.gemm(K.Operand(dypad, False, H, offset=lead * H, seg_stride=(T + pk) * H, z1=cpg),
           K.Operand(hpad, False, H, chunk_shift=6, ld_chunk=H, seg_stride=(T + pk) * H, z1=cpg),
           dWf, cpg, pk * cpg, T, ldc=pk * cpg, nseg=4, splits=8, batch=G, c_z1=cpg * pk * cpg,
           flags=_lib.EPI_ATOMIC)


for gen, name in ((0, "wgrad sliding-window"), (2, "wgrad generic 128x128")):
    prev = K.gemm_select(gen)
    us = timeit(wcall)
    K.gemm_select(prev)
    print(f"{name}: {us:.1f} us  {flops / us / 1e6:.0f} TFLOP/s", flush=True)
