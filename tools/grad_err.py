"""Diagnostic: whole-gradient rel-L2 of one bf16/f32 engine train step vs the oracle (tiny arch)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.environ.get("NRSE_PKG_ROOT") or os.path.join(ROOT, "noise-robust-speech-embedding_amd")]
import torch
from oracle import wavlm_byol as O
from nrse_amd import arch as A, params as PR
from nrse_amd.engine import ByolEngine

arch = A.TINY.deterministic()
layout = PR.byol_layout(arch, 256, 512)
flat = PR.init_byol_flat(layout, 1234)
g = torch.Generator().manual_seed(5)
clean = torch.randn(8, 16000, generator=g)
noisy = clean + 0.3 * torch.randn(8, 16000, generator=g)
st = O.OracleState(layout, flat)
r = O.train_step(st, clean, noisy, lr=1e-4, weight_decay=1e-5, ema_decay=0.99, step_seed=3)
ref = r["grad"].double()
for dt in (torch.float32, torch.bfloat16):
    eng = ByolEngine(arch, 256, 512, compute_dtype=dt, init_flat=flat)
    eng.cfg.ema_decay = 0.99
    eng.train_step(clean.cuda(), noisy.cuda(), lr=1e-4, step_seed=3)
    gg = eng.grad.cpu().double()
    worst = []
    for gname, s in layout.specs:
        off, cnt, _ = layout.offsets[PR.GROUP_PREFIX[gname] + s.name]
        rr = ref[off:off + cnt]
        if rr.norm() > 0:
            worst.append((float((gg[off:off + cnt] - rr).norm() / rr.norm()), cnt, s.name))
    worst.sort(reverse=True)
    print(os.environ.get("NRSE_PKG_ROOT", "cur"), dt, "vec rel", float((gg - ref).norm() / ref.norm()),
          "worst", [(round(a, 3), c, n) for a, c, n in worst[:4]], flush=True)
