"""Micro-benchmark of nrse_gemm at the WavLM-Large step shapes: kernel generations 2 (128x128)
and 3 (256x256) vs torch.matmul (hipBLASLt), random bf16 operands."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "noise-robust-speech-embedding_amd"))
import torch
from nrse_amd import kernels as K, _lib

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
    return s.elapsed_time(e) / iters


gens = [int(g) for g in os.environ.get("GENS", "2,3").split(",")]
shapes = [("qkv", 12768, 3072, 1024), ("out", 12768, 1024, 1024), ("ffn1", 12768, 4096, 1024),
          ("ffn2", 12768, 1024, 4096), ("conv", 12799 * 32, 512, 1536)]
for name, M, N, Kd in shapes:
    a = torch.randn(M, Kd, device=dev).to(torch.bfloat16); w = torch.randn(N, Kd, device=dev).to(torch.bfloat16)
    c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
    dx = torch.empty(M, Kd, device=dev, dtype=torch.bfloat16)
    dw = torch.zeros(N, Kd, device=dev)
    fl = 2.0 * M * N * Kd
    line = f"{name:5s} {M}x{N}x{Kd}:"
    t = timeit(lambda: torch.matmul(a, w.t()))
    line += f" torch {fl / t / 1e9:.0f}TF |"
    for g in gens:
        K.gemm_select(g)
        t1 = timeit(lambda: K.linear_fwd(a, w, c))
        t3 = timeit(lambda: K.linear_dgrad(dy, w, dx))
        t4 = timeit(lambda: K.linear_wgrad(dy, a, dw))
        line += f" g{g}: fwd {fl / t1 / 1e9:.0f} dgrad {fl / t3 / 1e9:.0f} wgrad {fl / t4 / 1e9:.0f} |"
    K.gemm_select(0)
    for slab in (False, True):
        K._SLAB_WGRAD = slab
        t5 = timeit(lambda: K.linear_wgrad(dy, a, dw))
        line += f" auto wgrad({'slab' if slab else 'atomic'}) {fl / t5 / 1e9:.0f} |"
    K._SLAB_WGRAD = True
    print(line, flush=True)
