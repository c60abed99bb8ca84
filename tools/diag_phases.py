"""Per-barrier timeline of the 256-column GEMM main loop (diagnostic build with
NRSE_G3_PHASE_STAMPS=1 via NRSE_LIB_PATH): workgroup 0, one wave of each ping-pong group, s_memtime
after each of the 8 barriers of every K-tile. Prints the median interval length per barrier
slot (cycles) for K = 1024 and 4096 at M = 12768, N = 1024."""
import ctypes, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "noise-robust-speech-embedding_amd"))
import torch
from nrse_amd import _lib, kernels as K

_lib.init_device(0)
K.gemm_select(3)
for rows in (256, 224):
    K.gemm_tile_rows(rows)
    for Kd in (1024, 4096):
        M, N = 12768, 1024
        a = (torch.rand(M, Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = (torch.rand(N, Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        st = torch.zeros(2048, dtype=torch.int64, device="cuda")
        p = _lib.GemmParams()
        p.a = K.Operand(a, True, Kd).c(); p.b = K.Operand(w, True, Kd).c()
        p.M, p.N, p.K, p.nseg, p.splits, p.batch, p.zdiv = M, N, Kd, 1, 1, 1, 1
        p.alpha = 1.0; p.c = c.data_ptr(); p.c_dtype = _lib.BF16; p.ldc = N
        p.aux = st.data_ptr()
        for _ in range(3):
            _lib.check(_lib.lib().nrse_gemm(ctypes.byref(p), K.stream_ptr()), "nrse_gemm")
        torch.cuda.synchronize()
        t = st.view(2, 1024).cpu().double()
        nt = Kd // 64
        for grp in (0, 1):
            x = t[grp, :8 * nt]
            d = (x[1:] - x[:-1]).view(-1)
            # interval ending at barrier slot i (i = 1..7 within a K-tile, 0 = from the previous tile)
            per = [d[(i - 1) % 8::8][2:-2].median().item() for i in range(8)]
            print(f"rows={rows} K={Kd} group {grp}: per-K-tile {sum(per):.0f} cyc; intervals ending at barrier slot 0..7: "
                  + " ".join(f"{v:.0f}" for v in per), flush=True)
