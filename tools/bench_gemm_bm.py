"""Isolated nrse_gemm rates at the WavLM-Large step shapes (M = 12768), forward (y = x W^T + b)
and dgrad (dx = dy W), 256-column kernel at tile rows 256 and 224, against torch (hipBLASLt) on
the same random bf16 operands; interleaved rounds in one process (median of 5)."""
import os, sys, statistics
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


M = int(os.environ.get("M", 12768))
rows = [int(r) for r in os.environ.get("ROWS", "256,224").split(",")]
rows_default = K.gemm_tile_rows(256)   # the process's setting, restored after each shape
for name, N, Kd in (("qkv", 3072, 1024), ("out", 1024, 1024), ("ffn1", 4096, 1024), ("ffn2", 1024, 4096)):
    x = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, Kd, device=dev) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, device=dev)
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
    dx = torch.empty(M, Kd, device=dev, dtype=torch.bfloat16)
    fl = 2.0 * M * N * Kd
    res = {}
    for rnd in range(5):
        res.setdefault("torch_fwd", []).append(timeit(lambda: torch.mm(x, w.t())))
        res.setdefault("torch_dgrad", []).append(timeit(lambda: torch.mm(dy, w)))
        for r in rows:
            K.gemm_tile_rows(r)
            res.setdefault(f"bm{r}_fwd", []).append(timeit(lambda: K.linear_fwd(x, w, y, bias=b)))
            res.setdefault(f"bm{r}_dgrad", []).append(timeit(lambda: K.linear_dgrad(dy, w, dx)))
        K.gemm_tile_rows(rows_default)
    print(f"{name} {M}x{N}x{Kd}: " + " ".join(f"{k} {fl / statistics.median(v) / 1e9:.0f}TF"
                                              for k, v in res.items()), flush=True)
