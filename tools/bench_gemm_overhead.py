"""Per-tile fixed cost of the 256x256 GEMM generations: time per wave of tiles vs K-tiles at
exactly one (N=1024, M=16384: 256 tiles) and four (N=4096: 1024 tiles) tiles per CU."""
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
    return s.elapsed_time(e) / iters


M = 16384
for N in (1024, 4096):
    waves = (M // 256) * (N // 256) // 256
    for Kd in (128, 256, 512, 1024, 2048):
        a = (torch.rand(M, Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = (torch.rand(N, Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        line = f"N={N} K={Kd:5d} ({Kd // 64:3d} K-tiles, {waves} tiles/CU):"
        for g in (3, 4):
            K.gemm_select(g)
            t = timeit(lambda: K.linear_fwd(a, w, c))
            line += f"  g{g} {t * 1e3 / waves:6.1f} us/tile"
        K.gemm_select(0)
        print(line, flush=True)
