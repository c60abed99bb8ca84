"""Micro-benchmark of nrse_gemm at the WavLM-Large step shapes vs torch.matmul (hipBLASLt)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "noise-robust-speech-embedding_amd"))
import torch
from nrse_amd import kernels as K, _lib

_lib.init_device(0)
dev = "cuda"

def timeit(fn, iters=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / iters

shapes = [("qkv", 12768, 3072, 1024), ("out", 12768, 1024, 1024), ("ffn1", 12768, 4096, 1024), ("ffn2", 12768, 1024, 4096)]
for dt in [torch.bfloat16]:
    for name, M, N, Kd in shapes:
        a = torch.randn(M, Kd, device=dev).to(dt); w = torch.randn(N, Kd, device=dev).to(dt)
        c = torch.empty(M, N, device=dev, dtype=dt)
        fl = 2.0 * M * N * Kd
        t1 = timeit(lambda: K.linear_fwd(a, w, c))
        t2 = timeit(lambda: torch.matmul(a, w.t()))
        dy = torch.randn(M, N, device=dev).to(dt)
        dx = torch.empty(M, Kd, device=dev, dtype=dt)
        t3 = timeit(lambda: K.linear_dgrad(dy, w, dx))
        dw = torch.zeros(N, Kd, device=dev)
        t4 = timeit(lambda: K.linear_wgrad(dy, a, dw, splits=max(1, 256 // ((N // 128) * (Kd // 128)))))
        print(f"{name:5s} {M}x{N}x{Kd}: fwd {t1:.3f}ms {fl/t1/1e9:.0f}TF | torch {t2:.3f}ms {fl/t2/1e9:.0f}TF | dgrad {t3:.3f}ms {fl/t3/1e9:.0f}TF | wgrad {t4:.3f}ms {fl/t4/1e9:.0f}TF", flush=True)
# f32 path
a = torch.randn(4096, 1024, device=dev); w = torch.randn(1024, 1024, device=dev); c = torch.empty(4096, 1024, device=dev)
t = timeit(lambda: K.linear_fwd(a, w, c)); print(f"f32 4096x1024x1024 {t:.3f}ms {2*4096*1024*1024/t/1e9:.0f}TF")
