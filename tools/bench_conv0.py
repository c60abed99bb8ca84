"""conv0 (1 -> 512, k 10, s 5) + LayerNorm + GELU forward in isolation at the step's shape
(B = 32 x 8 s): the bf16 output (the bf16 step), the bf16 output + the two fp8 correction planes
with the saturation counter (the bf16sw step, ABI 7 / 10), the three-plane split-bf16 output; and
the conv LayerNorm's fp8-plane form at conv layer 1 (32 x 12799 rows x 512). us, median of 5."""
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "noise-robust-speech-embedding_amd"))
import torch
from nrse_amd import _lib, kernels as K

_lib.init_device(0)
dev = "cuda"


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


B, L, C, k, st = 32, 128000, 512, 10, 5
T0 = (L - k) // st + 1
wav = torch.randn(B, L, device=dev)
w = torch.randn(C, k, device=dev) * 0.3
g = torch.ones(C, device=dev); b = torch.zeros(C, device=dev)
mean = torch.empty(B * T0, device=dev); rstd = torch.empty(B * T0, device=dev)
out = torch.empty(B * T0, C, device=dev, dtype=torch.bfloat16)
out3 = torch.empty(3, B * T0, C, device=dev, dtype=torch.bfloat16)
y8 = torch.empty(2, B * T0, C, device=dev, dtype=K.FP8)
sat = torch.zeros(1, device=dev, dtype=torch.int32)
res = {}
for rnd in range(5):
    res.setdefault("bf16", []).append(timeit(lambda: K.conv0_fwd(wav, w, g, b, out, mean, rstd, T0, k, st, 1e-5)))
    res.setdefault("bf16+fp8 planes", []).append(
        timeit(lambda: K.conv0_fwd(wav, w, g, b, out, mean, rstd, T0, k, st, 1e-5, y8=y8, y8_exp=11, sat=sat)))
    res.setdefault("split3", []).append(
        timeit(lambda: K.conv0_fwd(wav, w, g, b, out3, mean, rstd, T0, k, st, 1e-5, split3=True)))
print("conv0 fwd: " + "  ".join(f"{n} {statistics.median(v):.1f}us" for n, v in res.items()), flush=True)
