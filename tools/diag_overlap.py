import os, sys
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "noise-robust-speech-embedding_amd"))
import torch
from oracle import wavlm_byol as O
from nrse_amd import arch as A, params as PR
from nrse_amd.engine import ByolEngine
arch = A.TINY.deterministic()
layout = PR.byol_layout(arch, 256, 512)
flat = PR.init_byol_flat(layout, 1234)
g = torch.Generator().manual_seed(5)
clean = torch.randn(4, 16000, generator=g); noisy = clean + 0.3 * torch.randn(4, 16000, generator=g)
st = O.OracleState(layout, flat)
engs = {}
for ov in (False, True):
    e = ByolEngine(arch, 256, 512, compute_dtype=torch.float32, init_flat=flat)
    e.cfg.ema_decay = 0.99; e.cfg.overlap_optimizer = ov
    engs[ov] = e
for i in range(3):
    r = O.train_step(st, clean, noisy, lr=1e-4, weight_decay=engs[False].cfg.weight_decay, ema_decay=0.99, step_seed=i)
    line = f"step {i} oracle loss {r['loss']:.6f} gn {r['grad_norm']:.5f}"
    for ov, e in engs.items():
        l = float(e.train_step(clean.cuda(), noisy.cuda(), lr=1e-4, step_seed=i))
        line += f" | ov={ov} loss {l:.6f} gn {e.grad_norm():.5f}"
    print(line, flush=True)
