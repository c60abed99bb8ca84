"""In-kernel timeline of the gen-3 256x256 GEMM (diagnostic build with NRSE_G3_STAMPS=1, loaded via
NRSE_LIB_PATH): per workgroup s_memtime at entry, after the prologue wait, after the main loop and
after the epilogue's stores retired. Prints the median phase lengths and the spread of entry
times, for the step's GEMM shapes."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "noise-robust-speech-embedding_amd"))
import torch
from nrse_amd import _lib, kernels as K

_lib.init_device(0)
K.gemm_select(3)
CLK_MHZ = float(os.environ.get("CLK_MHZ", "100"))  # s_memtime counts shader clocks; reported in kcycles


def run(M, N, Kd, rows=256, gelu=False, reps=5, layout="TT", fp8=False):
    """layout: TT = A and B k-contiguous (forward), FF = both m-contiguous (weight gradient:
    A = dy^T, B = x^T over the token axis K), TF = B m-contiguous (dgrad)."""
    K.gemm_tile_rows(rows)
    a = (torch.rand(M, Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = (torch.rand(N, Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    bias = torch.randn(N, device="cuda")
    nwg = -(-M // rows) * -(-N // 256)
    st = torch.zeros(8 * nwg, dtype=torch.int64, device="cuda")
    p = _lib.GemmParams()
    if layout == "TT":
        p.a = K.Operand(a, True, Kd).c()
        p.b = K.Operand(w, True, Kd).c()
    else:
        at, wt = a.t().contiguous(), w.t().contiguous()
        keep = (at, wt)
        p.a = K.Operand(a, True, Kd).c() if layout == "TF" else K.Operand(at, False, M).c()
        p.b = K.Operand(wt, False, N).c()
    p.M, p.N, p.K, p.nseg, p.splits, p.batch, p.zdiv = M, N, Kd, 1, 1, 1, 1
    if fp8:
        # the split-weight mode's fp8 correction segment (one K segment of fp8 x8 . w8 2^-19)
        a8 = torch.empty(M, Kd, device="cuda", dtype=K.FP8); K.cast_fp8(a, a8)
        w8 = torch.empty(N, Kd, device="cuda", dtype=K.FP8); K.split_lo8(w.float() * 1.001, w8, 19)
        keep8 = (a8, w8)
        p.a8, p.b8, p.nseg8, p.b8_exp = K.Operand(a8, True, Kd).c(), K.Operand(w8, True, Kd).c(), 1, 19
    p.alpha = 1.0
    p.c = c.data_ptr()
    p.c_dtype = _lib.BF16
    p.ldc = N
    p.colsum = st.data_ptr()
    if gelu:
        p.flags = _lib.EPI_BIAS | _lib.EPI_GELU
        p.bias = bias.data_ptr()
        p.aux = aux.data_ptr()
        p.aux_dtype = _lib.BF16
        p.ldaux = N
    for _ in range(reps):
        _lib.check(_lib.lib().nrse_gemm(ctypes.byref(p), K.stream_ptr()), "nrse_gemm")
    torch.cuda.synchronize()
    t = st.view(nwg, 8).cpu().double()
    t0 = t[:, 0].min()
    d = [(t[:, i + 1] - t[:, i]).median().item() / 1e3 for i in range(7)]
    names = ["prologue", "loop", "drain", "stage0", "pass0", "pass1", "pass2+3"]
    end = (t[:, 7] - t0)
    print(f"{layout}{'+fp8' if fp8 else ''} M={M} N={N} K={Kd} rows={rows} gelu={int(gelu)} wgs={nwg}: " +
          " ".join(f"{n} {v:.1f}" for n, v in zip(names, d)) +
          f" kcyc (loop {d[1] / (Kd // 64 + (Kd // 128 if fp8 else 0)):.2f}/K-tile); entry max {(t[:, 0] - t0).max().item() / 1e3:.1f}, "
          f"last end {end.max().item() / 1e3:.1f} kcyc", flush=True)


if os.environ.get("SHAPES") == "layouts":
    # the weight-gradient shapes of one slab split (token range 12768 / 4) and a dgrad
    for lay in ("TT", "TF", "FF"):
        run(1024, 4096, 3192, rows=256, layout=lay)
        run(4096, 1024, 3192, rows=256, layout=lay)
elif os.environ.get("SHAPES") == "fp8":
    # the bf16sw forward: bf16 segment + fp8 correction segment (the 256-row 32x32x64 form)
    for shape in ((12768, 1024, 1024), (12768, 3072, 1024), (12768, 4096, 1024), (12768, 1024, 4096)):
        run(*shape, rows=256)
        run(*shape, rows=256, fp8=True)
    run(12768, 4096, 1024, rows=256, gelu=True, fp8=True)
elif os.environ.get("SHAPES") == "short":
    run(12768, 1024, 1024, rows=256)
    run(12768, 1024, 4096, rows=256)
else:
    for shape in ((12768, 1024, 1024), (12768, 4096, 1024), (12768, 1024, 4096)):
        for rows in (256, 224):
            run(*shape, rows=rows)
    run(12768, 4096, 1024, rows=224, gelu=True)
