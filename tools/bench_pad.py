"""The pos-conv padding kernels in isolation at the step's shapes (B = 32, T = 399, C = 1024, pad 64
each side): SpecAugment + pad + bf16 cast (forward), GELU' + pad (backward), and a parity check of
both against torch. Prints us and effective GB/s (algorithmic bytes)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "noise-robust-speech-embedding_amd"))
import torch
import torch.nn.functional as F
from nrse_amd import _lib, kernels as K

_lib.init_device(0)
dev = "cuda"
B, T, C, pf, pb = 32, 399, 1024, 64, 64
Tp = T + pf + pb


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


h = torch.randn(B, T, C, device=dev)
mask = (torch.rand(B, T, device=dev) < 0.1).to(torch.uint8)
embed = torch.randn(C, device=dev)
dst = torch.empty(B, Tp, C, device=dev, dtype=torch.bfloat16)
hm = h.clone()
K.specaug_pad(hm, mask, embed, dst, B, T, C, pf, pb)
ref = torch.where(mask.bool()[..., None], embed, h)
assert torch.equal(hm, ref)
assert torch.equal(dst, F.pad(ref, (0, 0, pf, pb)).to(torch.bfloat16))
us = timeit(lambda: K.specaug_pad(hm, mask, embed, dst, B, T, C, pf, pb))
print(f"specaug_pad {B}x{T}x{C} -> {Tp} bf16: {us:.1f} us  {B * T * C * 8 / us / 1e3 + B * Tp * C * 2 / us / 1e3:.0f} GB/s", flush=True)
dy = torch.randn(B, T, C, device=dev)
pre = torch.randn(B, T, C, device=dev).to(torch.bfloat16)
out = torch.empty(B, Tp, C, device=dev, dtype=torch.bfloat16)
K.gelu_bwd_pad(dy, pre, out, B, T, C, pf, pb)
x = pre.double().requires_grad_(True)
F.gelu(x).backward(dy.double())
err = (out[:, pf:pf + T].double() - x.grad).norm() / x.grad.norm()
assert err < 5e-3 and not out[:, :pf].any() and not out[:, pf + T:].any(), err
us = timeit(lambda: K.gelu_bwd_pad(dy, pre, out, B, T, C, pf, pb))
print(f"gelu_bwd_pad {B}x{T}x{C} -> {Tp} bf16: {us:.1f} us  {(B * T * C * 6 + B * Tp * C * 2) / us / 1e3:.0f} GB/s", flush=True)
