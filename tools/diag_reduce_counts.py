"""How many ordered reductions each transformer layer of the bench step queues (ABI 9 deferral):
the pending count at every reduce_flush of one bench-shape step (configs[1], B = 32, 8 s).
Usage: python tools/diag_reduce_counts.py [bf16|bf16sw]"""
import collections
import os
import sys

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "noise-robust-speech-embedding_amd"))
import torch

from nrse_amd import _lib, arch as A, kernels as K
from nrse_amd.engine import ByolEngine, StepConfig, compute_mode

mode = sys.argv[1] if len(sys.argv) > 1 else "bf16"
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
B, L = 32, 128000
g = torch.Generator(device=dev)
g.manual_seed(1234)
clean = torch.randn(B, L, device=dev, generator=g) * 0.1
noisy = clean + 0.3 * torch.randn(B, L, device=dev, generator=g)
cdt, wsplit = compute_mode(mode)
eng = ByolEngine(A.LARGE, 1024, 2048, device=dev, compute_dtype=cdt, seed=1234, weight_split=wsplit,
                 step_cfg=StepConfig(ema_decay=0.997, overlap_optimizer=True, fused_zero_grad=True))
counts = []
flush = K.reduce_flush


def counting_flush(stream=None):
    counts.append(_lib.lib().nrse_reduce_pending())
    return flush(stream)


K.reduce_flush = counting_flush
for s in range(2):
    counts.clear()
    eng.train_step(clean, noisy, lr=1e-4, step_seed=s)
    torch.cuda.synchronize()
    print(f"step {s}: {len(counts)} flushes, jobs per flush {dict(collections.Counter(counts))}", flush=True)
