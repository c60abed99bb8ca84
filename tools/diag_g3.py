"""Time the 256x256 GEMM (forced) on the step's forward shapes; with NRSE_LIB_PATH pointing at a
diagnostic build (tools/build_diag.sh) this prices one part of the kernel."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "noise-robust-speech-embedding_amd"))
import torch
from nrse_amd import kernels as K, _lib

_lib.init_device(0)
K.gemm_select(3)
tag = os.environ.get("NRSE_LIB_PATH", "product").split("/")[-1]
out = []
for name, M, N, Kd in [("qkv", 12768, 3072, 1024), ("ffn2", 12768, 1024, 4096), ("sq8k", 8192, 8192, 8192)]:
    a = (torch.rand(M, Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = (torch.rand(N, Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        K.linear_fwd(a, w, c)
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        K.linear_fwd(a, w, c)
    e.record(); torch.cuda.synchronize()
    t = s.elapsed_time(e) / 10
    out.append(f"{name} {2.0 * M * N * Kd / t / 1e9:.0f}TF ({t * 1e3:.0f}us)")
print(tag, " | ".join(out), flush=True)
