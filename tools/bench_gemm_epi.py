"""Price the fused GEMM epilogues at the step's shapes: same GEMM, plain bf16 store vs the
epilogue the step uses (bias+GELU+aux, bias+resid+dropout f32, GELU' dgrad)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "noise-robust-speech-embedding_amd"))
import torch
from nrse_amd import kernels as K, _lib

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


M = 12768
for name, N, Kd in [("qkv", 3072, 1024), ("out", 1024, 1024), ("ffn1", 4096, 1024), ("ffn2", 1024, 4096)]:
    a = torch.randn(M, Kd, device=dev).to(torch.bfloat16); w = torch.randn(N, Kd, device=dev).to(torch.bfloat16)
    b = torch.randn(N, device=dev)
    fl = 2.0 * M * N * Kd
    cb = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    cf = torch.empty(M, N, device=dev)
    aux = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    res = torch.randn(M, N, device=dev)
    t0 = timeit(lambda: K.linear_fwd(a, w, cb))
    t1 = timeit(lambda: K.linear_fwd(a, w, cb, bias=b))
    t2 = timeit(lambda: K.linear_fwd(a, w, cb, bias=b, flags=_lib.EPI_GELU, aux=aux, ldaux=N))
    t3 = timeit(lambda: K.linear_fwd(a, w, cf, bias=b, resid=res, ldr=N, dropout_p=0.1, seed=5))
    t4 = timeit(lambda: K.linear_fwd(a, w, cf))
    print(f"{name} {M}x{N}x{Kd}: plain-bf16 {t0:.0f}us ({fl/t0/1e6:.0f}TF) +bias {t1:.0f} +gelu+aux {t2:.0f} "
          f"f32 {t4:.0f} f32+bias+resid+drop {t3:.0f}", flush=True)
