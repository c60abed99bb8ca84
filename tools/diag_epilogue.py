"""Time of the gen-3 GEMM with its epilogue ablated (diag_libs/libnrse_abl7.so: no global stores;
abl8: no LDS reads / stores) vs the product library, at the step's K = 1024 shapes."""
import os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r'''
import os, sys
sys.path.insert(0, os.path.join(%r, "noise-robust-speech-embedding_amd"))
import torch
from nrse_amd import kernels as K, _lib
_lib.init_device(0); K.gemm_select(3)
def timeit(fn, iters=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / iters
out = []
for M, N, Kd in ((12768, 1024, 1024), (12768, 4096, 1024), (16384, 1024, 1024)):
    a = (torch.rand(M, Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = (torch.rand(N, Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    t = timeit(lambda: K.linear_fwd(a, w, c))
    out.append(f"{M}x{N}x{Kd}: {t*1e3:7.1f} us ({2.0*M*N*Kd/t/1e9:5.0f} TF)")
print(" | ".join(out))
''' % ROOT
for lib in ("", "abl7", "abl8"):
    env = dict(os.environ)
    if lib:
        env["NRSE_LIB_PATH"] = os.path.join(ROOT, "noise-robust-speech-embedding_amd", "diag_libs", f"libnrse_{lib}.so")
    r = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=120)
    print(f"{lib or 'product':8s}", r.stdout.strip() or r.stderr[-500:], flush=True)
