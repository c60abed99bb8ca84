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


def run(M, N, Kd, reps=5):
    a = (torch.rand(M, Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = (torch.rand(N, Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    nwg = -(-M // 256) * -(-N // 256)
    st = torch.zeros(4 * nwg, dtype=torch.int64, device="cuda")
    p = _lib.GemmParams()
    p.a = K.Operand(a, True, Kd).c()
    p.b = K.Operand(w, True, Kd).c()
    p.M, p.N, p.K, p.nseg, p.splits, p.batch, p.zdiv = M, N, Kd, 1, 1, 1, 1
    p.alpha = 1.0
    p.c = c.data_ptr()
    p.c_dtype = _lib.BF16
    p.ldc = N
    p.colsum = st.data_ptr()
    for _ in range(reps):
        _lib.check(_lib.lib().nrse_gemm(ctypes.byref(p), K.stream_ptr()), "nrse_gemm")
    torch.cuda.synchronize()
    t = st.view(nwg, 4).cpu().double()
    t0 = t[:, 0].min()
    pro = (t[:, 1] - t[:, 0]).median() / 1e3
    loop = (t[:, 2] - t[:, 1]).median() / 1e3
    epi = (t[:, 3] - t[:, 2]).median() / 1e3
    start = (t[:, 0] - t0)
    end = (t[:, 3] - t0)
    print(f"M={M} N={N} K={Kd} wgs={nwg}: prologue {pro:.1f} loop {loop:.1f} ({loop / (Kd // 64):.2f}/K-tile) "
          f"epilogue {epi:.1f} kcyc; entry spread p50 {start.median() / 1e3:.1f} max {start.max() / 1e3:.1f}; "
          f"last end {end.max() / 1e3:.1f} kcyc", flush=True)


for shape in ((12768, 1024, 1024), (12768, 3072, 1024), (12768, 4096, 1024), (12768, 1024, 4096),
              (16384, 1024, 1024), (16384, 4096, 1024), (16384, 1024, 256)):
    run(*shape)
