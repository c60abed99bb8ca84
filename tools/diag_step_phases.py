"""Wall time of the bench step's phases on the main stream (no profiler): HIP events recorded
before / after ByolEngine.forward (both views joined), the loss, backward (side streams joined)
and optimizer_step, over timed steps of the bench workload (configs[1], B = 32, 8 s). With the
overlapped optimizer the AdamW segments run on their own stream beside the next forward; the
'optimizer' phase is then only its enqueue point. Usage: python tools/diag_step_phases.py [bf16|bf16sw] [B]"""
import math
import os
import sys

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "noise-robust-speech-embedding_amd"))
import torch

from nrse_amd import arch as A, kernels as K
from nrse_amd.engine import ByolEngine, StepConfig, compute_mode

mode = sys.argv[1] if len(sys.argv) > 1 else "bf16"
B_ARG = int(sys.argv[2]) if len(sys.argv) > 2 else 32
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
B, L = B_ARG, 128000
gen = torch.Generator(device=dev)
gen.manual_seed(1234)
clean_raw = torch.randn(B, L, device=dev, generator=gen) * 0.1
noise_raw = torch.randn(B, L, device=dev, generator=gen)
noise_len = torch.full((B,), L, device=dev, dtype=torch.int32)
snr = torch.tensor([[4.0, 8.0][i % 2] for i in range(B)], device=dev)
clean_iv, noisy_iv = torch.empty(B, L, device=dev), torch.empty(B, L, device=dev)
status, kscale = torch.empty(B, device=dev, dtype=torch.int32), torch.empty(B, device=dev)
cdt, wsplit = compute_mode(mode)
eng = ByolEngine(A.LARGE, 1024, 2048, device=dev, compute_dtype=cdt, seed=1234, weight_split=wsplit,
                 step_cfg=StepConfig(ema_decay=0.997, overlap_optimizer=True, fused_zero_grad=True))

marks = []


def mark(tag):
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    marks.append((tag, e))


def wrap(name):
    f = getattr(eng, name)

    def g(*a, **k):
        mark(name + ">")
        r = f(*a, **k)
        mark(name + "<")
        return r
    setattr(eng, name, g)


for n in ("forward", "backward", "optimizer_step"):
    wrap(n)

import time
warm, steps = 3, 8
host = []
for i in range(warm + steps):
    if i == warm:
        torch.cuda.synchronize()
        marks.clear()
    h0 = time.perf_counter()
    mark("step>")
    K.snr_mix(clean_raw, noise_raw, noise_len, snr, clean_iv, noisy_iv, status, kscale, K.SNR_PEAK_ZMUV)
    eng.train_step(clean_iv, noisy_iv, lr=0.5e-5 * (1 + math.cos(math.pi * i / 1e6)), step_seed=i)
    if i >= warm:
        host.append((time.perf_counter() - h0) * 1e3)
mark("end")
torch.cuda.synchronize()
acc = {}
for (t0, e0), (t1, e1) in zip(marks, marks[1:]):
    key = f"{t0} -> {t1}"
    acc[key] = acc.get(key, 0.0) + e0.elapsed_time(e1)
total = marks[0][1].elapsed_time(marks[-1][1])
print(f"{mode} B={B}: {total / steps:.2f} ms per step over {steps} steps; host enqueue per step "
      f"{sum(host) / len(host):.2f} ms (min {min(host):.2f}, max {max(host):.2f})")
for k, v in acc.items():
    print(f"  {k:40s} {v / steps:8.2f} ms")
