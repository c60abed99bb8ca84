"""Which gradients differ between two identical train steps (diagnostic for
tests/test_determinism_gpu.py): per parameter, the count of differing entries after step 0."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "noise-robust-speech-embedding_amd"))
import torch
from nrse_amd import arch as A, params as PR, _lib
from nrse_amd.engine import ByolEngine

_lib.init_device(0)
dt = torch.bfloat16 if os.environ.get("DT") == "bf16" else torch.float32
arch = A.TINY if os.environ.get("DET") != "1" else A.TINY.deterministic()
layout = PR.byol_layout(arch, 256, 512)
flat = PR.init_byol_flat(layout, 77)
E = [ByolEngine(arch, 256, 512, compute_dtype=dt, init_flat=flat) for _ in range(2)]
g = torch.Generator().manual_seed(5)
clean = (torch.randn(4, 16000, generator=g) * 0.1).cuda()
noisy = clean + 0.3 * torch.randn(4, 16000, generator=g).cuda()
for e in E:
    e.train_step(clean, noisy, lr=1e-4, step_seed=100)
torch.cuda.synchronize()
va = PR.named_views(layout, E[0].grad)
vb = PR.named_views(layout, E[1].grad)
n = 0
for k in va:
    d = int((va[k] != vb[k]).sum())
    if d:
        n += 1
        print(f"{k}: {d} / {va[k].numel()} differ, max |diff| {float((va[k] - vb[k]).abs().max()):.3e}", flush=True)
print("params with differences:", n)
