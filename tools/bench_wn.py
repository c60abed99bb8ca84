"""Pos-conv weight-norm backward at WavLM-Large (H = 1024, cpg = 64, K = 128): us per call."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "noise-robust-speech-embedding_amd"))
import torch
from nrse_amd import _lib, kernels as K
_lib.init_device(0)
H, G, Kk = 1024, 16, 128
cpg = H // G
v = torch.randn(H, cpg, Kk, device="cuda"); gg = torch.rand(1, 1, Kk, device="cuda") + 0.5
norms = torch.empty(Kk, device="cuda"); wf = torch.empty(G, cpg, Kk * cpg, device="cuda", dtype=torch.bfloat16)
wd = torch.empty_like(wf)
K.weight_norm_fwd(gg, v, wf, wd, norms, H, cpg, Kk)
dWf = torch.randn(G, cpg, Kk * cpg, device="cuda"); dg = torch.zeros(1, 1, Kk, device="cuda"); dv = torch.zeros_like(v)
sc = torch.empty(Kk, device="cuda")
f = lambda: K.weight_norm_bwd(dWf, gg, v, norms, dg, dv, sc, H, cpg, Kk)
for _ in range(3): f()
torch.cuda.synchronize()
s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(20): f()
e.record(); torch.cuda.synchronize()
print(f"weight_norm_bwd {s.elapsed_time(e) / 20 * 1e3:.1f} us", flush=True)
