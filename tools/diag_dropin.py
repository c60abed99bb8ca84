"""Drift between the reference training loop over the drop-in model and the fused engine in bf16
(tests/test_dropin_gpu.py): repeats the comparison a few times in one process and prints the
per-step loss differences, and whether the loop and the engine are each run-to-run deterministic
on identical batches. Usage: python tools/diag_dropin.py [repeats]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "noise-robust-speech-embedding_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from test_dropin_gpu import cfg, reference_loop  # noqa: E402
from nrse_amd import arch as A  # noqa: E402
from nrse_amd.engine import ByolEngine  # noqa: E402
from src.data.noisy_speech_dataset import create_dataloaders  # noqa: E402
from src.models.byol import BYOLSpeechModel  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
dev = torch.device("cuda:0")
arch = A.TINY.deterministic()
config = cfg()
dtype = torch.bfloat16
for r in range(reps):
    model = BYOLSpeechModel(config, compute_dtype=dtype, arch=arch).to(dev)
    flat0 = model.engine.online.detach().clone()
    loader, _ = create_dataloaders(config, device=dev, synthetic_items=40)
    losses, batches = reference_loop(model, loader, config, dev, 3, 1e-5)
    eng = ByolEngine(arch, 256, 512, compute_dtype=dtype, init_flat=flat0.cpu())
    eng.cfg.ema_decay, eng.cfg.weight_decay = 0.99, 1e-5
    cur = 1e-5
    diffs = []
    for i, (c, n, nl) in enumerate(batches):
        le = float(eng.train_step(c.squeeze(1), n.squeeze(1), lr=cur, step_seed=i))
        diffs.append(le - losses[i])
        cur = nl[0]
    print(f"rep {r}: loop {['%.6f' % x for x in losses]}  engine-loop {['%+.2e' % d for d in diffs]}  "
          f"init sum {float(flat0.double().sum()):.6f} batch0 sum {float(batches[0][0].double().sum()):.6f}", flush=True)
