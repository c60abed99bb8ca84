"""Isolated forward GEMM rates at the WavLM-Large step shapes (M = 12768) with the step's
epilogues (bias; bias + GELU + bf16 pre-activation; bias + dropout + f32 residual), for the kernel
generations in GENS (default: the normal dispatch, i.e. the 256x256 kernel), against torch
(hipBLASLt, plain product) for scale; interleaved rounds in one process (median of 5)."""
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
gens = [int(g) for g in os.environ.get("GENS", "0").split(",")]
SHAPES = (("qkv", 3072, 1024, "bias"), ("out", 1024, 1024, "resid"), ("ffn1", 4096, 1024, "gelu"),
          ("ffn2", 1024, 4096, "resid"), ("ffn1t", 4096, 1024, "gelu_noaux"), ("fproj", 1024, 512, "bias_drop"))
only = os.environ.get("SHAPES")
for name, N, Kd, epi in SHAPES:
    if only and name not in only.split(","):
        continue
    x = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, Kd, device=dev) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, device=dev)
    r = torch.randn(M, N, device=dev)
    pre = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    fl = 2.0 * M * N * Kd

    def run():
        if epi == "bias":
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            return lambda: K.linear_fwd(x, w, y, bias=b), y
        if epi == "gelu":
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            return lambda: K.linear_fwd(x, w, y, bias=b, flags=_lib.EPI_GELU, aux=pre, ldaux=N), y
        if epi == "gelu_noaux":  # the target view's FFN-up (no tape)
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            return lambda: K.linear_fwd(x, w, y, bias=b, flags=_lib.EPI_GELU), y
        if epi == "bias_drop":  # the feature projection (f32 out)
            y = torch.empty(M, N, device=dev)
            return lambda: K.linear_fwd(x, w, y, bias=b, dropout_p=0.1, seed=5), y
        y = torch.empty(M, N, device=dev)
        return lambda: K.linear_fwd(x, w, y, bias=b, flags=_lib.EPI_RESID, resid=r, ldr=N, dropout_p=0.1,
                                    seed=5), y

    res, outs = {}, {}
    for rnd in range(5):
        res.setdefault("torch", []).append(timeit(lambda: torch.mm(x, w.t())))
        for g in gens:
            K.gemm_select(g)
            fn, y = run()
            res.setdefault(f"gen{g}", []).append(timeit(fn))
            if rnd == 0:
                fn(); torch.cuda.synchronize(); outs[g] = y.float()
        K.gemm_select(0)
    agree = ""
    if len(outs) > 1:
        a, c = outs[gens[0]], outs[gens[-1]]
        agree = f" rel(gen{gens[-1]} vs gen{gens[0]}) {((a - c).norm() / a.norm()).item():.2e}"
    print(f"{name}[{epi}] {M}x{N}x{Kd}: " + " ".join(f"{k} {fl / statistics.median(v) / 1e9:.0f}TF"
                                                      for k, v in res.items()) + agree, flush=True)
