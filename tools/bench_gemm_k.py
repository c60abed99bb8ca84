"""Per-tile fixed cost of the 256x256 GEMM: time vs K at M=12768 (N=1024: 200 tiles = one round
on 256 CUs; N=2048: 400 tiles = two rounds), plain bf16 store."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "noise-robust-speech-embedding_amd"))
import torch
from nrse_amd import kernels as K, _lib

_lib.init_device(0)


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


M = 12768
for N in (1024, 2048):
    line = f"N={N}:"
    for Kd in (64, 256, 1024, 2048, 4096):
        a = torch.randn(M, Kd, device="cuda").to(torch.bfloat16); w = torch.randn(N, Kd, device="cuda").to(torch.bfloat16)
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        t = timeit(lambda: K.linear_fwd(a, w, c))
        line += f" K{Kd} {t:.1f}us"
    print(line, flush=True)
