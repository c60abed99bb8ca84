"""Isolated forward GEMMs of the split-weight mode at the WavLM-Large layer shapes (M = 12768):
plain bf16 (the bf16 step), the bf16 lo-plane form (two bf16 K segments) and the fp8 correction
form (one bf16 segment + one fp8 segment on the MX-scaled MFMA), each with the step's epilogue and
without one; interleaved rounds in one process (median of 5), times in us."""
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
    return s.elapsed_time(e) / iters * 1e3


M = int(os.environ.get("M", 12768))
SHAPES = (("qkv", 3072, 1024, "bias"), ("ffn1", 4096, 1024, "gelu"), ("ffn2", 1024, 4096, "resid"),
          ("out", 1024, 1024, "resid"))
for name, N, Kd, epi in SHAPES:
    x = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
    w32 = torch.randn(N, Kd, device=dev) * 0.03
    w2 = torch.empty(2, N, Kd, device=dev, dtype=torch.bfloat16)
    K.split_bf16(w32, w2[0], w2[1])
    w8 = torch.empty(N, Kd, device=dev, dtype=K.FP8)
    K.split_lo8(w32, w8, 19)
    x8 = torch.empty(M, Kd, device=dev, dtype=K.FP8)
    K.cast_fp8(x, x8)
    b = torch.randn(N, device=dev)
    r = torch.randn(M, N, device=dev)
    pre = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    y8 = torch.empty(M, N, device=dev, dtype=K.FP8)
    fl = 2.0 * M * N * Kd

    def epi_kw(on):
        if not on:
            return torch.empty(M, N, device=dev), {}
        if epi == "bias":
            return torch.empty(M, N, device=dev, dtype=torch.bfloat16), dict(bias=b)
        if epi == "gelu":
            return torch.empty(M, N, device=dev, dtype=torch.bfloat16), dict(bias=b, flags=_lib.EPI_GELU, aux=pre,
                                                                               ldaux=N)
        return torch.empty(M, N, device=dev), dict(bias=b, flags=_lib.EPI_RESID, resid=r, ldr=N, dropout_p=0.1, seed=5)

    res = {}
    forms = os.environ.get("FORMS", "bf16,bf16lo,fp8corr").split(",")
    for rnd in range(5):
        for on in ((True,) if os.environ.get("EPI_ONLY") else (False, True)):
            y, kw = epi_kw(on)
            tag = "epi" if on else "plain"
            if "bf16" in forms:
                res.setdefault(f"bf16/{tag}", []).append(timeit(lambda: K.linear_fwd(x, w2[0], y, **kw)))
            if "bf16lo" in forms:
                res.setdefault(f"bf16lo/{tag}", []).append(
                    timeit(lambda: K.linear_fwd(x, w2[0], y, w_lo=N * Kd, **kw)))
            kw8 = dict(kw)
            if on and epi == "gelu":
                kw8["out8"] = y8
            if "fp8corr" in forms:
                res.setdefault(f"fp8corr/{tag}", []).append(
                    timeit(lambda: K.linear_fwd(x, w2[0], y, x8=x8, w8=w8, lo8_exp=19, **kw8)))
    print(f"{name}[{epi}] {M}x{N}x{Kd}: " + "  ".join(
        f"{k} {statistics.median(v):.1f}us ({fl / statistics.median(v) / 1e6:.0f}TF/bf16-seg)" for k, v in res.items()),
        flush=True)
