"""Repeatability probe for the training forward under concurrent load: engine B's step-0 forward
loss (WavLM-Large bf16, B = 8 x 8 s), computed on an idle GPU, is recomputed TRIALS times while
engine A runs full training steps (backward, overlapped optimizer) just before it on the same
device; prints how many recomputations differ bitwise, per variant (MODE = default | sync: a
device sync between A and B | serial: B's two views on one stream | syncserial: both | ovl: A's optimizer
overlapped on its own stream)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "noise-robust-speech-embedding_amd"))
import torch
from nrse_amd import arch as A, kernels as K, params as PR, engine as E, _lib

_lib.init_device(0)
layout = PR.byol_layout(A.LARGE, 1024, 2048)
flat = PR.init_byol_flat(layout, 77)
ea = E.ByolEngine(A.LARGE, 1024, 2048, compute_dtype=torch.bfloat16, init_flat=flat)
eb = E.ByolEngine(A.LARGE, 1024, 2048, compute_dtype=torch.bfloat16, init_flat=flat)
g = torch.Generator().manual_seed(5)
clean = (torch.randn(8, 128000, generator=g) * 0.1)
noisy = (clean + 0.3 * torch.randn(8, 128000, generator=g)).cuda()
clean = clean.cuda()


def b_loss():
    pred, tproj, ctx = eb.forward(clean, noisy, train=True, step_seed=100, need_grad=True)
    loss = torch.zeros(1, device="cuda")
    K.byol_loss(pred, tproj, loss, torch.empty_like(pred), None)
    return loss, pred, tproj, ctx["emb"]


ref = [t.clone() for t in b_loss()]
torch.cuda.synchronize()
trials = int(os.environ.get("TRIALS", "8"))
for mode in os.environ.get("MODES", "default,ovl,sync,serial").split(","):
    bad = []
    for i in range(trials):
        ea.cfg.overlap_optimizer = mode == "ovl"
        ea.train_step(clean, noisy, lr=1e-4, step_seed=200 + i)
        if mode in ("sync", "syncserial"):
            ea.sync_optimizer(); torch.cuda.synchronize()
        E._SERIAL_TARGET = mode in ("serial", "syncserial")
        out = b_loss()
        E._SERIAL_TARGET = False
        torch.cuda.synchronize()
        if not torch.equal(out[0], ref[0]):
            # which view: online pred / online embedding (main stream), target projection (side)
            bad.append("".join(n for n, a, r in zip(("P", "T", "E"), out[1:], ref[1:]) if not torch.equal(a, r)))
    print(f"{mode}: {len(bad)} of {trials} differ {bad[:8]} (P online pred, T target proj, E online emb)",
          flush=True)
