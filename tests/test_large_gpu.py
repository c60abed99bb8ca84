"""WavLM-Large end to end on the HIP path against the REFERENCE's own outputs
(tests/golden/byol_large.npz, written by tests/golden/make_golden.py from the reference
BYOLSpeechModel / byol_loss / AdamW / _update_target_network on WavLM-Large, B = 4, 8 s; and
byol_large_3s.npz / byol_large_12s.npz at the two ends of configs[4]'s 3-12 s range, T = 149
and 599 frames, reference src/utils/audio_utils.py:38-49 crop/pad lengths through
src/models/encoder.py:17-29).

This is the north-star tolerance check: embeddings within 1e-3 rel-L2 of the reference
(BASELINE.json north_star; reference src/models/byol.py:75-128, src/models/encoder.py:17-32,
train_byol.py:56-74).

* f32 parity mode (exact-f32 MFMA GEMMs, f32 attention / norms): the bound 1e-3 is asserted on
  embeddings, online_pred, target_proj and the pre-clip gradient norm; the gradient sample, the
  per-tensor gradient norms, the AdamW update and the EMA update are checked too.
* bf16 mode (the benchmarked configs[1] path: bf16 GEMM / attention operands, f32 accumulation,
  f32 residual stream and master weights): the deviation from the reference is measured,
  printed and bounded (stated tolerances in DESIGN.md §6).
"""
import json
import os

import numpy as np
import pytest
import torch

from nrse_amd import arch as A, params as PR

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIXTURES = {"8s": "byol_large.npz", "3s": "byol_large_3s.npz", "12s": "byol_large_12s.npz"}
OUT = os.path.join(ROOT, "gpurun_out")


def rel(a, b):
    a = torch.as_tensor(np.asarray(a) if not torch.is_tensor(a) else a).double().cpu()
    b = torch.as_tensor(np.asarray(b) if not torch.is_tensor(b) else b).double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def make_inputs(B, L, seed):
    """Identical to tests/golden/make_golden.py:make_inputs (seed = SEED + 1 = 1235)."""
    g = torch.Generator().manual_seed(seed)
    clean = torch.randn(B, 1, L, generator=g)
    noisy = clean + 0.3 * torch.randn(B, 1, L, generator=g)
    return clean.squeeze(1), noisy.squeeze(1)


@pytest.fixture(scope="module", params=list(FIXTURES))
def large(request):
    z = np.load(os.path.join(ROOT, "tests", "golden", FIXTURES[request.param]))
    arch = A.LARGE.deterministic()
    layout = PR.byol_layout(arch, int(z["proj_dim"]), int(z["pred_dim"]))
    flat = PR.init_byol_flat(layout, int(z["seed"]))
    clean, noisy = make_inputs(int(z["B"]), int(z["L"]), int(z["seed"]) + 1)
    return dict(z=z, arch=arch, layout=layout, flat=flat, clean=clean, noisy=noisy, tag=request.param)


def _engine(large, dtype, wsplit=False, lo8=None):
    from nrse_amd.engine import ByolEngine
    z = large["z"]
    eng = ByolEngine(large["arch"], int(z["proj_dim"]), int(z["pred_dim"]), compute_dtype=dtype,
                     init_flat=large["flat"], weight_split=wsplit, split_lo8=lo8)
    eng.cfg.ema_decay = float(z["ema"])
    eng.cfg.weight_decay = float(z["wd"])
    return eng


def _run(large, dtype, wsplit=False, lo8=None):
    """Eval forward, last_hidden_state, one det train step; returns the measured deviations."""
    z = large["z"]
    eng = _engine(large, dtype, wsplit, lo8)
    if lo8:
        assert eng.online_lo8 is not None
    clean, noisy = large["clean"].cuda(), large["noisy"].cuda()
    m = {}
    pred, tproj, loss = eng.eval_forward(clean, noisy)
    emb = eng.embed(clean)
    hs, _, _ = eng.encoder_forward(eng.weights("online"), clean, train=False, hidden_dtype=torch.float32)
    m["eval_emb"] = rel(emb, z["eval_emb"])
    m["eval_pred"] = rel(pred, z["eval_pred"])
    m["eval_tproj"] = rel(tproj, z["eval_tproj"])
    m["eval_loss_abs"] = abs(float(loss) - float(z["eval_loss"]))
    m["hidden_norms"] = rel(hs.norm(dim=-1), z["eval_hidden_norms"])
    m["hidden_sample"] = rel(hs[:, ::37, ::13], z["eval_hidden_sample"])
    del hs
    lr = float(z["lr"])
    l1 = eng.train_step(clean, noisy, lr=lr, step_seed=0)
    torch.cuda.synchronize()
    m["train_loss_abs"] = abs(float(l1) - float(z["train_loss"]))
    m["grad_norm_rel"] = abs(eng.grad_norm() - float(z["train_grad_norm"])) / float(z["train_grad_norm"])
    g = eng.grad.cpu()
    idx = torch.from_numpy(z["grad_idx"])
    m["grad_sample"] = rel(g[idx], z["grad_sample"])
    # per-tensor gradient norms (505 tensors, layout order)
    norms = []
    for gname, s in eng.layout.specs:
        off, cnt, _ = eng.layout.offsets[PR.GROUP_PREFIX[gname] + s.name]
        norms.append(float(g[off:off + cnt].norm()))
    ref_n = z["grad_tensor_norms"]
    norms = np.array(norms)
    sig = ref_n > 1e-4 * float(z["train_grad_norm"])
    tn = np.abs(norms[sig] - ref_n[sig]) / ref_n[sig]
    m["tensor_norm_worst"] = float(tn.max())
    m["tensor_norm_median"] = float(np.median(tn))
    m["tensor_norm_worst_name"] = [f"{gn}.{s.name}" for (gn, s), keep in zip(eng.layout.specs, sig) if keep][
        int(tn.argmax())]
    # AdamW update (first step ~ lr * sign(g)) and EMA of it, at the sampled indices
    d = (eng.online.cpu()[idx] - large["flat"][idx]).numpy()
    dr = z["online_delta_sample"]
    m["online_delta"] = rel(d, dr)
    m["online_delta_flip_frac"] = float((np.abs(d - dr) > 0.05 * lr).mean())
    tidx = torch.from_numpy(z["target_idx"])
    dt = (eng.target.cpu()[tidx] - large["flat"][tidx]).numpy()
    m["target_delta"] = rel(dt, z["target_delta_sample"])
    # BatchNorm running statistics after one train-mode forward of each view
    bn = torch.cat([eng.bn["online_projector.layers.1"][0], eng.bn["online_projector.layers.1"][1],
                    eng.bn["target_projector.layers.4"][1]]).cpu()
    m["bn_running"] = rel(bn, z["bn_running"])
    del eng
    torch.cuda.empty_cache()
    return m


def _record(tag, m):
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, f"large_parity_{tag}.json"), "w") as f:
        json.dump(m, f, indent=1)
    print(tag, json.dumps(m))


def test_large_f32_matches_reference(nrse_device, large):
    m = _run(large, torch.float32)
    _record(f"f32_{large['tag']}", m)
    tol = 1e-3   # north-star bound on embeddings
    assert m["eval_emb"] < tol, m
    assert m["eval_pred"] < tol and m["eval_tproj"] < tol, m
    assert m["eval_loss_abs"] < 1e-4, m
    assert m["hidden_norms"] < tol and m["hidden_sample"] < tol, m
    assert m["train_loss_abs"] < 1e-4, m
    assert m["grad_norm_rel"] < tol, m
    assert m["grad_sample"] < 1e-2, m
    assert m["tensor_norm_worst"] < 1e-2, m
    assert m["online_delta_flip_frac"] < 0.01, m
    assert m["online_delta"] < 0.05 and m["target_delta"] < 0.05, m
    assert m["bn_running"] < tol, m


def test_large_bf16_deviation(nrse_device, large):
    """The benchmarked mode. Measured deviations are written to gpurun_out/large_parity_bf16.json
    and quoted in DESIGN.md §6; the bounds below are the stated bf16 tolerances."""
    m = _run(large, torch.bfloat16)
    _record(f"bf16_{large['tag']}", m)
    assert m["eval_emb"] < 1e-2, m
    assert m["eval_pred"] < 3e-2 and m["eval_tproj"] < 3e-2, m
    assert m["hidden_norms"] < 1e-2, m
    assert m["train_loss_abs"] < 1e-2, m
    # the end-to-end gradient goes through the heads' BatchNorm over 4 near-identical random-init
    # embeddings (ill-conditioned: test_oracle_golden.py::test_head_gradient_conditioning), so a
    # 5e-3 embedding deviation moves it by O(0.1-1); measured: norm 0.11, sample 0.71 rel-L2. The
    # bf16 gradient is pinned under a fixed upstream gradient by tests/test_bf16_gpu.py.
    assert m["grad_norm_rel"] < 0.25, m
    assert m["grad_sample"] < 1.0, m
    assert m["bn_running"] < 3e-2, m


@pytest.mark.parametrize("lo8", [True, False], ids=["fp8corr", "bf16lo"])
def test_large_bf16sw_matches_reference(nrse_device, large, lo8):
    """The north-star mode at bf16 activation cost: bf16 activations, the forward
    GEMMs against the weights' split hi + lo pair. The oracle's site ablation
    (tools/ablate_bf16_sites.py) puts 5.1e-3 of the bf16 mode's 5.15e-3 embedding deviation on
    the WEIGHT rounding (a perturbation shared by every frame, which the time mean keeps) and
    0.7e-3 on the activations; with the weights carried to ~2^-13 (fp8corr: the correction
    x (w - w_hi) as fp8 e4m3 x times the residual plane scaled by one exponent, the default) or ~2^-17 (bf16lo: a second bf16 segment) the
    embeddings meet the 1e-3 bound."""
    m = _run(large, torch.bfloat16, wsplit=True, lo8=lo8)
    _record(f"bf16sw{'' if lo8 else '_bf16lo'}_{large['tag']}", m)
    assert m["eval_emb"] < 1e-3, m          # north-star bound on embeddings
    assert m["hidden_norms"] < 1e-3, m
    assert m["eval_pred"] < 1e-3 and m["eval_tproj"] < 1e-3, m
    assert m["eval_loss_abs"] < 1e-4 and m["train_loss_abs"] < 3e-3, m
    assert m["bn_running"] < 3e-3, m
    # the backward is the bf16 path's (dgrad on the hi plane): its end-to-end gradient at the bf16
    # test's bounds (the heads' conditioning, test_large_bf16_deviation)
    assert m["grad_norm_rel"] < 0.25, m
    assert m["grad_sample"] < 1.0, m


def test_large_bf16_heads_match_reference(nrse_device, large):
    """the bf16 mode's heads, loss, head gradients and optimizer at f32-level
    bounds against the reference. The f32-mode encoder's embeddings of both views (2-4e-7 from
    the reference) are injected into the bf16-mode engine's projector / predictor / BYOL loss
    and their backward, then its AdamW (with the reference's clip coefficient: the sum of squares
    set to the reference's pre-clip norm) and EMA update the head parameters. Compared with
    byol_large*.npz: online_pred, target_proj, loss, every head tensor's gradient norm, the
    sampled head gradients, AdamW and EMA deltas (reference src/models/byol.py:75-128,
    train_byol.py:62-71)."""
    from nrse_amd import kernels as K, params as PR
    z = large["z"]
    clean, noisy = large["clean"].cuda(), large["noisy"].cuda()
    e32 = _engine(large, torch.float32)
    emb = e32.embed(clean, "online").clone()
    temb = e32.embed(noisy, "target").clone()
    del e32
    torch.cuda.empty_cache()
    assert rel(emb, z["eval_emb"]) < 1e-5
    eng = _engine(large, torch.bfloat16)
    eng.sync_optimizer()
    Pon = eng.group_views(eng.online, "projector")
    Ppr = eng.group_views(eng.online, "predictor")
    Ptp = eng.group_views(eng.target, "projector")
    proj, pc = eng.projector_forward(emb, Pon, "online_projector", True)
    pred, qc = eng.predictor_forward(proj, Ppr, True)
    tproj, _ = eng.projector_forward(temb, Ptp, "target_projector", True)
    loss = torch.zeros(1, device=emb.device)
    dpred = torch.empty_like(pred)
    K.byol_loss(pred, tproj, loss, dpred)
    eng.grad.zero_()
    Gp = eng.group_views(eng.grad, "predictor")
    Gj = eng.group_views(eng.grad, "projector")
    dproj = eng.predictor_backward(dpred, qc, Ppr, Gp)
    eng.projector_backward(dproj, pc, Pon, Gj)
    torch.cuda.synchronize()
    m = {"pred": rel(pred, z["train_pred"]), "tproj": rel(tproj, z["train_tproj"]),
         "loss_abs": abs(float(loss) - float(z["train_loss"]))}
    # head tensors: layout spec index -> reference per-tensor gradient norm
    g = eng.grad.cpu()
    worst, worst_name, head_lo, head_hi = 0.0, None, None, 0
    floor = 1e-4 * float(z["train_grad_norm"])   # as the f32 test: tensors with a significant gradient
    for i, (gname, s) in enumerate(eng.layout.specs):
        if gname == "encoder":
            continue
        off, cnt, _ = eng.layout.offsets[PR.GROUP_PREFIX[gname] + s.name]
        head_lo = off if head_lo is None else min(head_lo, off)
        head_hi = max(head_hi, off + cnt)
        ref_n = float(z["grad_tensor_norms"][i])
        if ref_n > floor:
            e = abs(float(g[off:off + cnt].norm()) - ref_n) / ref_n
            if e > worst:
                worst, worst_name = e, f"{gname}.{s.name}"
    m["head_tensor_norm_worst"] = worst
    m["head_tensor_norm_worst_name"] = worst_name
    idx = torch.from_numpy(z["grad_idx"])
    sel = (idx >= head_lo) & (idx < head_hi)
    m["head_samples"] = int(sel.sum())
    m["head_grad_sample"] = rel(g[idx[sel]], z["grad_sample"][sel.numpy()])
    # AdamW on the heads with the reference's clip coefficient, then the EMA of the target heads
    lr = float(z["lr"])
    eng.sumsq_buf.fill_(float(z["train_grad_norm"]) ** 2)
    c = eng.cfg
    K.adamw(eng.online[head_lo:head_hi], eng.grad[head_lo:head_hi], eng.m[head_lo:head_hi],
            eng.v[head_lo:head_hi], eng.online_sh[head_lo:head_hi], lr=lr, beta1=c.betas[0], beta2=c.betas[1],
            eps=c.eps, weight_decay=c.weight_decay, step=1, max_norm=c.max_norm, sumsq_buf=eng.sumsq_buf)
    ne = eng.layout.ema_numel
    K.ema(eng.target[head_lo:ne], eng.online[head_lo:ne], eng.target_sh[head_lo:ne], c.ema_decay)
    torch.cuda.synchronize()
    d = (eng.online.cpu()[idx[sel]] - large["flat"][idx[sel]]).numpy()
    m["head_online_delta"] = rel(d, z["online_delta_sample"][sel.numpy()])
    tidx = torch.from_numpy(z["target_idx"])
    tsel = (tidx >= head_lo) & (tidx < ne)
    dt = (eng.target.cpu()[tidx[tsel]] - large["flat"][tidx[tsel]]).numpy()
    m["head_target_delta"] = rel(dt, z["target_delta_sample"][tsel.numpy()])
    m["head_target_samples"] = int(tsel.sum())
    _record(f"bf16_heads_{large['tag']}", m)
    assert m["pred"] < 1e-3 and m["tproj"] < 1e-3, m
    assert m["loss_abs"] < 1e-4, m
    assert m["head_tensor_norm_worst"] < 1e-3, m
    assert m["head_samples"] > 20 and m["head_grad_sample"] < 1e-3, m
    assert m["head_online_delta"] < 1e-3, m
    # the EMA delta (1 - ema) * d_online ~ 3e-8 sits at ~1 ulp of the 0.02-sized f32 weights it is
    # added to: f32-rounding-limited on both sides (the f32 test's bound)
    assert m["head_target_delta"] < 0.05, m
