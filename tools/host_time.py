"""Host enqueue time vs device time of the bench step (configs[1]): is the step launch-bound?
Prints, per step, the host time to enqueue it (train_step returns without a sync) and the device
time per step over a synchronized run, with and without the GEMM event probe bench.py uses."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "noise-robust-speech-embedding_amd"))
import torch
from nrse_amd import arch as A, kernels as K
from nrse_amd.engine import ByolEngine, StepConfig

dev = torch.device("cuda", 0)
B, L = 32, 128000
eng = ByolEngine(A.LARGE, 1024, 2048, device=dev, compute_dtype=torch.bfloat16, seed=1234,
                 step_cfg=StepConfig(ema_decay=0.997, overlap_optimizer=os.environ.get("SERIAL_OPT") is None))
g = torch.Generator(device=dev); g.manual_seed(1)
clean = torch.randn(B, L, device=dev, generator=g) * 0.1
noisy = clean + torch.randn(B, L, device=dev, generator=g) * 0.1
for i in range(3):
    eng.train_step(clean, noisy, lr=1e-5, step_seed=i)
torch.cuda.synchronize()
for probe in (False, True):
    pr = [] if probe else None
    hs = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    K.set_gemm_probe(pr)
    for i in range(6):
        h0 = time.perf_counter()
        eng.train_step(clean, noisy, lr=1e-5, step_seed=10 + i)
        hs.append((time.perf_counter() - h0) * 1e3)
    K.set_gemm_probe(None)
    torch.cuda.synchronize()
    tot = (time.perf_counter() - t0) * 1e3 / 6
    print(f"probe={probe}: host enqueue ms/step {['%.1f' % h for h in hs]}  wall ms/step {tot:.1f}", flush=True)
