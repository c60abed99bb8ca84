"""How much of the 256x256 kernel's gap is wave quantization: TF/s vs M at fixed N, K
(tiles = ceil(M/256) * N/256 on 256 CUs)."""
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


for N, Kd in ((1024, 1024), (4096, 1024), (1024, 4096)):
    for M in (8192, 12768, 16384, 24576, 32768):
        a = (torch.rand(M, Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = (torch.rand(N, Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        fl = 2.0 * M * N * Kd
        t = timeit(lambda: K.linear_fwd(a, w, c))
        tt = timeit(lambda: torch.matmul(a, w.t()))
        tiles = -(-M // 256) * (N // 256)
        print(f"N={N} K={Kd} M={M:6d} tiles={tiles:5d} waves={tiles/256:5.2f}: g3 {fl/t/1e9:6.0f} TF  torch {fl/tt/1e9:6.0f} TF  "
              f"per-tile {t*1e3/-(-tiles//256):6.1f} us/wave", flush=True)
