"""Full BYOL step on the HIP path vs the CPU oracle (oracle/wavlm_byol.py, itself pinned to the
reference by tests/test_oracle_golden.py), on the tiny WavLM arch.

Tolerances (stated per the north star): fp32 parity mode uses exact-f32 MFMA / f32 kernels,
so embeddings and loss agree to ~1e-5 rel-L2; bf16 mode (bf16 GEMM operands, f32 accumulate,
f32 residual stream) is checked at 2e-2 rel-L2 on embeddings against the f32 oracle and at 5e-3
against the oracle's bf16-operand mode.
"""
import numpy as np
import pytest
import torch

from oracle import wavlm_byol as O
from nrse_amd import arch as A, params as PR, rng as R

pytestmark = pytest.mark.gpu

PROJ, PRED = 256, 512


def rel(a, b):
    a = torch.as_tensor(a).double().cpu(); b = torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def make(arch, dtype, B=4, L=16000, seed=1234):
    from nrse_amd.engine import ByolEngine
    layout = PR.byol_layout(arch, PROJ, PRED)
    flat = PR.init_byol_flat(layout, seed)
    eng = ByolEngine(arch, PROJ, PRED, compute_dtype=dtype, init_flat=flat)
    st = O.OracleState(layout, flat)
    g = torch.Generator().manual_seed(5)
    clean = torch.randn(B, L, generator=g)
    noisy = clean + 0.3 * torch.randn(B, L, generator=g)
    return eng, st, clean, noisy


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-5), (torch.bfloat16, 2e-2)])
def test_eval_forward_matches_oracle(nrse_device, dtype, tol):
    arch = A.TINY.deterministic()
    eng, st, clean, noisy = make(arch, dtype)
    pred, tproj, loss = eng.eval_forward(clean.cuda(), noisy.cuda())
    with torch.no_grad():
        rp, rt, remb = O.forward(st, clean, noisy, train=False)
        rl = O.byol_loss(rp, rt)
    emb = eng.embed(clean.cuda())
    assert rel(emb, remb) < tol
    assert rel(pred, rp) < 5 * tol
    assert rel(tproj, rt) < 5 * tol
    assert abs(float(loss) - float(rl)) < 5 * tol
    if dtype == torch.bfloat16:
        # against the oracle's bf16-operand mode (same rounding points): 4x tighter
        O.set_operand_dtype(dtype)
        try:
            with torch.no_grad():
                rp16, rt16, remb16 = O.forward(st, clean, noisy, train=False)
        finally:
            O.set_operand_dtype(None)
        assert rel(emb, remb16) < tol / 4, (rel(emb, remb16), rel(emb, remb))
        assert rel(tproj, rt16) < 5 * tol / 4


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.bfloat16, 5e-2)])
def test_train_step_matches_oracle(nrse_device, dtype, tol):
    """One fused train step (forward, loss, backward, clip, AdamW, EMA) vs the oracle step.
    bf16: the oracle runs in its bf16-operand mode (same rounding points). The end-to-end
    gradient passes through the BYOL heads, whose BatchNorm over near-identical random-init
    embeddings amplifies rounding ~800x (test_oracle_golden.py::test_head_gradient_conditioning;
    the oracle's own bf16 and f32 modes differ by 0.27 rel-L2 here), so in bf16 only the loss,
    the gradient norm and the whole-gradient direction are bounded end to end; the gradient is
    pinned per tensor, with no exemptions but the zero-gradient k_proj biases, by
    tests/test_bf16_gpu.py under a fixed upstream gradient."""
    arch = A.TINY.deterministic()
    eng, st, clean, noisy = make(arch, dtype, B=8)
    flat0 = st.online.clone()
    lr, wd, ema = 1e-4, 1e-5, 0.99
    eng.cfg.ema_decay = ema
    eng.cfg.weight_decay = wd
    loss = eng.train_step(clean.cuda(), noisy.cuda(), lr=lr, step_seed=3)
    O.set_operand_dtype(dtype)
    try:
        r = O.train_step(st, clean, noisy, lr=lr, weight_decay=wd, ema_decay=ema, step_seed=3)
    finally:
        O.set_operand_dtype(None)
    assert abs(float(loss) - r["loss"]) < tol
    g = eng.grad.cpu()
    assert abs(eng.grad_norm() - r["grad_norm"]) / r["grad_norm"] < 10 * tol
    if dtype == torch.float32:
        assert rel(g, r["grad"]) < 10 * tol
        worst = []
        for gname, s in eng.layout.specs:
            off, cnt, _ = eng.layout.offsets[PR.GROUP_PREFIX[gname] + s.name]
            ref = r["grad"][off:off + cnt]
            if ref.norm() < 1e-6 * r["grad_norm"]:
                continue
            worst.append((rel(g[off:off + cnt], ref), s.name))
        worst.sort(reverse=True)
        assert worst[0][0] < 20 * tol, worst[:5]
    else:
        assert rel(g, r["grad"]) < 0.5
    # AdamW + EMA: parameter deltas in units of lr. The first Adam step is ~lr*sign(g), so
    # entries with near-zero gradients flip sign under bf16 rounding of the operands.
    d = (eng.online.cpu() - flat0)
    dr = (st.online - flat0)
    assert (torch.abs(d - dr) > 0.05 * lr).float().mean() < (0.002 if dtype == torch.float32 else 0.15)
    dt = eng.target.cpu() - flat0[:eng.layout.ema_numel]
    drt = st.target - flat0[:eng.layout.ema_numel]
    assert float(torch.abs(dt - drt).max()) < 0.05 * lr


def test_stochastic_step_matches_oracle_with_same_masks(nrse_device):
    """Dropout / attention dropout / LayerDrop / SpecAugment on: the oracle replays the same
    counter-hash masks and the engine's host-side LayerDrop + span decisions."""
    arch = A.TINY
    eng, st, clean, noisy = make(arch, torch.float32, B=8)
    lr = 1e-4
    eng.cfg.ema_decay = 0.99
    B, T = clean.shape[0], arch.frames(clean.shape[1])
    skips, seeds = eng.stochastic_inputs(11, B, T, True)
    masks = eng.spec_masks(seeds, B, T)     # drawn on the device (nrse_specaug_mask)
    assert all(m.any() for m in masks)
    loss = eng.train_step(clean.cuda(), noisy.cuda(), lr=lr, step_seed=11)
    r = O.train_step(st, clean, noisy, lr=lr, weight_decay=eng.cfg.weight_decay, ema_decay=0.99, step_seed=11,
                     layer_skip=skips, mask_time=masks)
    assert abs(float(loss) - r["loss"]) < 1e-4
    assert abs(eng.grad_norm() - r["grad_norm"]) / r["grad_norm"] < 1e-3


def test_varlen_steps_match_oracle(nrse_device):
    """Consecutive steps on different utterance lengths (config 5's bucketed batches): the
    engine re-derives T, the rel-pos bucket table and every launch shape per step."""
    arch = A.TINY.deterministic()
    eng, st, _, _ = make(arch, torch.float32, B=4)
    eng.cfg.ema_decay = 0.99
    for i, L in enumerate((24000, 16000, 40000)):
        g = torch.Generator().manual_seed(20 + i)
        clean = torch.randn(4, L, generator=g)
        noisy = clean + 0.3 * torch.randn(4, L, generator=g)
        loss = eng.train_step(clean.cuda(), noisy.cuda(), lr=1e-4, step_seed=i)
        r = O.train_step(st, clean, noisy, lr=1e-4, weight_decay=eng.cfg.weight_decay, ema_decay=0.99, step_seed=i)
        assert abs(float(loss) - r["loss"]) < 1e-4, (L, float(loss), r["loss"])
        assert abs(eng.grad_norm() - r["grad_norm"]) / r["grad_norm"] < 1e-3


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_overlapped_optimizer_is_bitwise_serial(nrse_device, dtype):
    """cfg.overlap_optimizer: clip/AdamW/EMA in per-layer segments on their own stream give
    bit-identical parameters, moments, EMA target and bf16 shadows to the one-launch serial
    update (segment boundaries cover the flat buffer exactly once), over three updates."""
    arch = A.TINY.deterministic()
    e1, _, _, _ = make(arch, dtype)
    e2, _, _, _ = make(arch, dtype)
    e2.cfg.overlap_optimizer = True
    segs = e2._segments
    assert segs[0][0] == 0 and segs[-1][1] == e2.layout.numel
    assert all(a[1] == b[0] for a, b in zip(segs, segs[1:])) and all(s % 4 == 0 for s, _ in segs)
    assert len(segs) == arch.layers + 1
    g = torch.Generator(device="cuda").manual_seed(9)
    for i in range(3):
        grad = torch.randn(e1.layout.numel, device="cuda", generator=g) * (10.0 ** (i - 2))
        e1.grad.copy_(grad)
        e2.sync_optimizer()
        e2.grad.copy_(grad)
        e1.optimizer_step(1e-3)
        e2.optimizer_step(1e-3)
    e2.sync_optimizer()
    torch.cuda.synchronize()
    for name in ("online", "target", "m", "v", "online_sh", "target_sh"):
        a, b = getattr(e1, name), getattr(e2, name)
        if a is None:
            continue
        assert torch.equal(a, b), name


def test_overlapped_optimizer_train_steps_match_oracle(nrse_device):
    """Consecutive fused steps with the overlapped optimizer (each step's forward waits per layer
    for the previous update) next to the serial engine path and the oracle. The gradient
    reductions are ordered (deterministic) and the segmented update is bitwise the serial one, so
    the overlapped and serial engines agree bit for bit at every step; both track the oracle (the
    heads' conditioning amplifies step-to-step f32 differences to ~2e-4 in the loss by step 3)."""
    arch = A.TINY.deterministic()
    eng, st, clean, noisy = make(arch, torch.float32, B=4)
    ser, _, _, _ = make(arch, torch.float32, B=4)
    for e in (eng, ser):
        e.cfg.ema_decay = 0.99
    eng.cfg.overlap_optimizer = True
    for i in range(3):
        loss = float(eng.train_step(clean.cuda(), noisy.cuda(), lr=1e-4, step_seed=i))
        ls = float(ser.train_step(clean.cuda(), noisy.cuda(), lr=1e-4, step_seed=i))
        r = O.train_step(st, clean, noisy, lr=1e-4, weight_decay=eng.cfg.weight_decay, ema_decay=0.99, step_seed=i)
        assert loss == ls, (i, loss, ls)
        assert eng.grad_norm() == ser.grad_norm(), (i, eng.grad_norm(), ser.grad_norm())
        assert abs(loss - r["loss"]) < 5e-4, (i, loss, r["loss"])
        if i == 0:
            assert abs(eng.grad_norm() - r["grad_norm"]) / r["grad_norm"] < 1e-4
    eng.sync_optimizer()
    for a, b in ((eng.online, ser.online), (eng.target, ser.target)):
        assert torch.equal(a, b)
    # vs the oracle: three Adam steps of ~lr each, near-zero-gradient entries free to flip
    for a, b in ((eng.online.cpu(), st.online), (eng.target.cpu(), st.target)):
        d = torch.abs(a - b)
        assert float(d.max()) < 3 * 2 * 1e-4 * 1.05
        assert (d > 0.5 * 1e-4).float().mean() < 0.05
