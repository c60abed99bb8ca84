"""Isolated backward GEMM rates at the WavLM-Large step shapes (M = 12768 tokens): dgrad
(dx = dy W, bf16 out) and wgrad (dW += dy^T x, f32 accumulate: the slab split-K of
kernels.linear_wgrad), ours against torch (hipBLASLt) on the same operands, median of 5."""
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
for name, N, Kd in (("qkv", 3072, 1024), ("out", 1024, 1024), ("ffn1", 4096, 1024), ("ffn2", 1024, 4096)):
    x = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, Kd, device=dev) * 0.05).to(torch.bfloat16)
    dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
    dx = torch.empty(M, Kd, device=dev, dtype=torch.bfloat16)
    dw = torch.zeros(N, Kd, device=dev)
    fl = 2.0 * M * N * Kd
    res = {}
    for rnd in range(5):
        res.setdefault("torch_dgrad", []).append(timeit(lambda: torch.mm(dy, w)))
        res.setdefault("ours_dgrad", []).append(timeit(lambda: K.linear_dgrad(dy, w, dx)))
        res.setdefault("torch_wgrad_bf16", []).append(timeit(lambda: torch.mm(dy.t(), x)))
        try:
            res.setdefault("torch_wgrad_f32", []).append(timeit(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32)))
        except Exception:
            res.pop("torch_wgrad_f32", None)
        res.setdefault("ours_wgrad", []).append(timeit(lambda: K.linear_wgrad(dy, x, dw)))
    print(f"{name} M={M} N={N} K={Kd}: " + " ".join(f"{k} {fl / statistics.median(v) / 1e9:.0f}TF"
                                                     for k, v in res.items()), flush=True)
