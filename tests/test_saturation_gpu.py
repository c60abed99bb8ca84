"""The split-weight mode's fp8 exponents under weights that grow and
the small-batch fallback of its layer GEMMs:

* every fp8 correction producer counts its saturated conversions (ABI 10 sat_count): nrse_split_lo8,
  the AdamW / fused-EMA plane writer, the LayerNorm y8 copies (both forms) -- exact counts against
  torch computations of the same values;
* the exponents follow the weights: lo8_exp from the layer weights' range, the conv stack's exponent
  from the conv LayerNorms' gamma / beta (|x| <= sqrt(C) max|gamma| + max|beta|) and the conv
  weights; with the conv gamma and the layer weights scaled by 4 both move, and the embeddings stay
  within 1e-3 of the oracle's split8 restatement at the moved exponents (and of the f32 oracle);
* weights that grow past the headroom during training make the AdamW pass's counter fire, the
  lagged HealthMonitor calls rederive_split_exponents(), the exponent moves and the counter clears;
* a batch under 128 frames (no fp8 segments: the 256x256 kernel's M) runs the bf16 lo plane, rebuilt
  first when the overlapped optimizer skipped it (bitwise the forward after a full refresh);
* the drop-in _update_target_network() rewrites the target's fp8 plane after the EMA.
"""
import numpy as np
import pytest
import torch

from oracle import wavlm_byol as O
from nrse_amd import arch as A, params as PR

pytestmark = pytest.mark.gpu
E4M3 = torch.float8_e4m3fn


def rel(a, b):
    a = torch.as_tensor(a).double().cpu(); b = torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def resid(x: torch.Tensor) -> torch.Tensor:
    """x - bf16(x), exact in f32."""
    x = x.detach().float().cpu()
    return x - x.to(torch.bfloat16).float()


def counter():
    return torch.zeros(1, device="cuda", dtype=torch.int32)


def test_split_lo8_counts_saturations(nrse_device):
    from nrse_amd import kernels as K
    g = torch.Generator().manual_seed(4)
    w = (torch.randn(70001, generator=g) * 0.03)
    w[::997] *= 300.0                                  # a few weights far outside the exponent's range
    wd = w.cuda()
    for e in (12, 19, 23):
        sat = counter()
        lo = torch.empty(w.numel(), device="cuda", dtype=E4M3)
        K.split_lo8(wd, lo, e, sat=sat)
        torch.cuda.synchronize()
        want = int(((resid(w) * 2.0 ** e).abs() > 448).sum())
        assert int(sat) == want, (e, int(sat), want)
    assert want > 0


def test_adamw_counts_plane_saturations(nrse_device):
    from nrse_amd import kernels as K
    n, ne = 40003, 30001
    p = torch.randn(n, device="cuda") * 0.05
    p[::501] *= 200.0
    g = torch.randn(n, device="cuda") * 1e-3
    m, v = torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
    t = p[:ne].clone()
    sumsq = torch.tensor([float((g.double() ** 2).sum())], device="cuda", dtype=torch.float64)
    sh, tsh = torch.empty(n, device="cuda", dtype=torch.bfloat16), torch.empty(ne, device="cuda", dtype=torch.bfloat16)
    lo8, tlo8 = torch.empty(n, device="cuda", dtype=E4M3), torch.empty(ne, device="cuda", dtype=E4M3)
    e = 20
    sat = counter()
    K.adamw(p, g, m, v, sh, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=1e-5, step=1, max_norm=1.0,
            sumsq_buf=sumsq, ema_t=t, ema_shadow=tsh, ema_decay=0.99, shadow_lo8=lo8, ema_shadow_lo8=tlo8,
            lo8_exp=e, sat=sat)
    torch.cuda.synchronize()
    want = int(((resid(p) * 2.0 ** e).abs() > 448).sum()) + int(((resid(t) * 2.0 ** e).abs() > 448).sum())
    assert want > 0 and int(sat) == want, (int(sat), want)


def test_layernorm_y8_counts_saturations(nrse_device):
    """fp8(bf16 y) saturates where |bf16 y| > 448 (the stored values decide: exact); the split form's
    hi plane likewise and its correction plane where |(o - bf16 o) 2^e| > 448 (the exact f32 output
    o is not stored: counted against a float64 restatement, to within the f32 rounding at the edge)."""
    from nrse_amd import kernels as K
    import torch.nn.functional as F
    rows, C = 2001, 512
    x = torch.randn(rows, C, device="cuda")
    gam = torch.full((C,), 1.0, device="cuda")
    gam[::7] = 200.0                                   # some outputs beyond e4m3's 448
    b = torch.zeros(C, device="cuda")
    y = torch.empty(rows, C, device="cuda", dtype=torch.bfloat16)
    y8 = torch.empty(rows, C, device="cuda", dtype=E4M3)
    mean, rstd = torch.empty(rows, device="cuda"), torch.empty(rows, device="cuda")
    sat = counter()
    K.ln_fwd(x, gam, b, y, mean, rstd, 1e-5, y8=y8, sat=sat)
    torch.cuda.synchronize()
    want = int((y.float().abs() > 448).sum())
    assert want > 0 and int(sat) == want, (int(sat), want)
    # the split form (conv stack): y8 [2, rows, C] = [fp8((o - bf16 o) 2^e) | fp8(bf16 o)]
    y82 = torch.empty(2, rows, C, device="cuda", dtype=E4M3)
    sat2 = counter()
    e = 14
    K.ln_fwd(x, gam, b, y, mean, rstd, 1e-5, y8=y82, y8_exp=e, sat=sat2)
    torch.cuda.synchronize()
    o = F.layer_norm(x.double(), (C,), gam.double(), b.double(), 1e-5).float().cpu()
    hi_sat = int((y.float().abs() > 448).sum())
    lo_sat = int(((resid(o) * 2.0 ** e).abs() > 448).sum())
    got = int(sat2)
    assert hi_sat > 0 and lo_sat > 0
    assert abs(got - (hi_sat + lo_sat)) <= 0.01 * (hi_sat + lo_sat) + 2, (got, hi_sat, lo_sat)


def _large_3s():
    arch = A.LARGE.deterministic()
    layout = PR.byol_layout(arch, 1024, 2048)
    flat = PR.init_byol_flat(layout, 1234)
    g = torch.Generator().manual_seed(21)
    clean = torch.randn(2, 48000, generator=g)
    return arch, layout, flat, clean


def _lo8_names(arch):
    out = []
    for li in range(arch.layers):
        for n in ("attention.q_proj.weight", "attention.k_proj.weight", "attention.v_proj.weight",
                  "attention.out_proj.weight", "feed_forward.intermediate_dense.weight",
                  "feed_forward.output_dense.weight"):
            out.append(f"encoder.layers.{li}.{n}")
    return out


def _oracle_split8_emb(layout, arch, flat, clean, e, c):
    P = O.split_flat(layout, flat)["encoder"]
    O.set_operand_dtype(torch.bfloat16, O.SPLIT_WEIGHT_SITES)
    O.set_split8(O.SPLIT8_SITES, e, c)
    try:
        with torch.no_grad():
            return O.encoder_forward(P, arch, clean, train=False).mean(1)
    finally:
        O.set_operand_dtype(None)
        O.set_split8(None)


def test_exponents_follow_scaled_conv_gamma_and_layer_weights(nrse_device):
    """VERDICT r05 #4's done-criterion: the conv LayerNorms' gamma x4 and the fp8-corrected layer
    weights x4 (max|w| x4) move both exponents (conv 11 -> 9, lo8_exp by -2), derived as the oracle
    restates them, nothing saturates, and the embeddings stay within 1e-3 of the oracle's split8
    restatement at the moved exponents and of f32."""
    from nrse_amd.engine import ByolEngine
    torch.set_num_threads(min(16, torch.get_num_threads()))
    arch, layout, flat, clean = _large_3s()
    eng = ByolEngine(arch, 1024, 2048, compute_dtype=torch.bfloat16, init_flat=flat, weight_split=True,
                     split_lo8=True)
    e0, c0 = eng.lo8_exp, eng.conv_lo8_exp
    P0 = O.split_flat(layout, flat)["encoder"]
    assert c0 == O.conv_lo8_exponent(P0, arch) == 11
    assert e0 == O.lo8_exponent([P0[n] for n in _lo8_names(arch)])
    scaled = flat.clone()
    V = PR.named_views(layout, scaled)
    for i in range(len(arch.conv_dim)):
        V[f"online_encoder.model.feature_extractor.conv_layers.{i}.layer_norm.weight"].mul_(4.0)
    # the layer weights x4 where the function allows it exactly: q, v (and their biases) x4 with k and
    # the out-projection x1/4 keep every score q.k and every attention output (scaling all of them x4
    # would sharpen the softmax 16-fold: another network, whose bf16 activation roundings alone move
    # the embeddings by ~3e-3); max|w| of the corrected matrices grows 4x either way
    pre = "online_encoder.model.encoder.layers."
    for li in range(arch.layers):
        at = f"{pre}{li}.attention."
        for n, f in (("q_proj", 4.0), ("v_proj", 4.0), ("k_proj", 0.25)):
            V[at + n + ".weight"].mul_(f)
            V[at + n + ".bias"].mul_(f)
        V[at + "out_proj.weight"].mul_(0.25)
    ne = layout.ema_numel
    eng.online.copy_(scaled.cuda())
    eng.target.copy_(scaled[:ne].cuda())
    eng.refresh_shadows()
    assert eng.conv_lo8_exp == c0 - 2 == O.conv_lo8_exponent(O.split_flat(layout, scaled)["encoder"], arch)
    P1 = O.split_flat(layout, scaled)["encoder"]
    assert eng.lo8_exp == O.lo8_exponent([P1[n] for n in _lo8_names(arch)]) < e0
    emb = eng.embed(clean.cuda()).cpu()
    torch.cuda.synchronize()
    assert int(eng.sat_buf.abs().sum()) == 0, eng.sat_buf
    assert eng.conv_split8_used
    r8 = _oracle_split8_emb(layout, arch, scaled, clean, eng.lo8_exp, eng.conv_lo8_exp)
    P = O.split_flat(layout, scaled)["encoder"]
    with torch.no_grad():
        rf = O.encoder_forward(P, arch, clean, train=False).mean(1)
    d8, df = rel(emb, r8), rel(emb, rf)
    print(f"scaled x4: exponents ({e0}, {c0}) -> ({eng.lo8_exp}, {eng.conv_lo8_exp}); emb vs oracle split8 "
          f"{d8:.2e}, vs f32 {df:.2e}")
    assert d8 < 1e-3 and df < 1e-3, (d8, df)


def test_growing_weights_fire_the_counter_and_move_the_exponent(nrse_device):
    """Weights that grow 8x without a refresh (what a long run could do): the next AdamW pass writes
    the planes with the stale exponent and its counter fires (only the layer matrices count: the
    planes of norms / biases / heads are outside the exponent's range and never read); the lagged
    HealthMonitor re-derives (lo8_exp -3), the counter clears, the planes are the new exponent's
    bit for bit, and the next AdamW pass counts nothing."""
    from nrse_amd.engine import ByolEngine
    from nrse_amd.health import HealthMonitor
    from nrse_amd import kernels as K
    arch = A.TINY.deterministic()
    layout = PR.byol_layout(arch, 256, 512)
    flat = PR.init_byol_flat(layout, 7)
    eng = ByolEngine(arch, 256, 512, compute_dtype=torch.bfloat16, init_flat=flat, weight_split=True,
                     split_lo8=True)
    e0 = eng.lo8_exp
    eng.grad.zero_()
    eng.optimizer_step(1e-12)          # at the derived exponent: nothing saturates
    torch.cuda.synchronize()
    assert int(eng.sat_buf.abs().sum()) == 0, eng.sat_buf
    for s, e in eng._lo8_ranges():
        eng.online[s:e].mul_(8.0)
        eng.target[s:e].mul_(8.0)
    eng.optimizer_step(1e-12)          # rewrites every plane with the stale exponent
    mon = HealthMonitor(lag=1)
    mon.record(0, eng.health_buf, engine=eng)
    torch.cuda.synchronize()
    assert int(eng.sat_buf[0]) > 0, eng.sat_buf
    mon.flush()
    assert mon.rederived and mon.rederived[0][1]["new"][0] == e0 - 3, mon.rederived
    assert eng.lo8_exp == e0 - 3 and int(eng.sat_buf.abs().sum()) == 0 and eng.sat_epoch == 1
    assert any("saturated" in m for _, m in mon.warnings)
    for flat_, plane in ((eng.online, eng.online_lo8), (eng.target, eng.target_lo8)):
        fresh = torch.empty_like(plane)
        K.split_lo8(flat_, fresh, eng.lo8_exp)
        torch.cuda.synchronize()
        for s, e in eng._lo8_ranges():
            assert torch.equal(fresh[s:e].view(torch.uint8), plane[s:e].view(torch.uint8))
    eng.optimizer_step(1e-12)
    mon.record(1, eng.health_buf, engine=eng)
    mon.flush()
    assert int(eng.sat_buf.abs().sum()) == 0 and len(mon.rederived) == 1


def test_short_batch_bf16sw_forward_uses_current_lo_planes(nrse_device):
    """a bf16sw forward over fewer than 128 frames (one 1 s clip: T = 49) has no fp8
    segments (the 256x256 kernel needs M >= 128). It takes the bf16 lo plane, which the overlapped
    optimizer's layer segments skip in the fp8 form: rebuilt first, so the embedding equals the one
    after an explicit refresh of every plane bit for bit, and differs from a forward that skips the
    rebuild (the stale plane)."""
    from nrse_amd.engine import ByolEngine
    arch = A.TINY.deterministic()
    layout = PR.byol_layout(arch, 256, 512)
    flat = PR.init_byol_flat(layout, 11)
    g = torch.Generator().manual_seed(5)
    clean = torch.randn(4, 48000, generator=g)
    noisy = clean + 0.3 * torch.randn(4, 48000, generator=g)
    one = torch.randn(1, 16000, generator=g).cuda()
    engs = []
    for _ in range(2):
        eng = ByolEngine(arch, 256, 512, compute_dtype=torch.bfloat16, init_flat=flat, weight_split=True,
                         split_lo8=True)
        eng.cfg.overlap_optimizer = True
        for i in range(2):
            eng.train_step(clean.cuda(), noisy.cuda(), lr=1e-3, step_seed=i)   # large lr: the lo planes move
        assert eng._lo_stale["online"] and eng._lo_stale["target"]
        engs.append(eng)
    a, b = engs
    emb, temb = a.embed(one).clone(), a.embed(one, "target").clone()
    assert not a._lo_stale["online"] and not a._lo_stale["target"]
    b._ensure_lo_planes = lambda W: None          # the stale plane (before the fix)
    stale = b.embed(one)
    a.refresh_shadows()
    torch.cuda.synchronize()
    assert torch.equal(emb, a.embed(one)) and torch.equal(temb, a.embed(one, "target"))
    assert not torch.equal(emb, stale), "the stale lo plane should change the embedding"
    assert rel(stale, emb) > 1e-4


def test_dropin_update_target_network_rewrites_fp8_plane(nrse_device):
    """the drop-in loop's _update_target_network() (nrse_ema) leaves the target's
    fp8 correction plane at the pre-EMA weights unless rewritten; it now equals split_lo8 of the
    updated target bit for bit."""
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "noise-robust-speech-embedding_amd"))
    from src.models.byol import BYOLSpeechModel, byol_loss
    from nrse_amd import kernels as K
    cfg = {"model": {"name": "nrse/wavlm-tiny", "projection_dim": 256, "prediction_dim": 512, "ema_decay": 0.9},
           "training": {"learning_rate": 1e-3, "weight_decay": 1e-5, "seed": 3}}
    model = BYOLSpeechModel(cfg, arch=A.TINY.deterministic(), weight_split=True)
    e = model.engine
    assert e.target_lo8 is not None
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3, weight_decay=1e-5)
    g = torch.Generator().manual_seed(2)
    clean = torch.randn(4, 48000, generator=g).cuda()
    noisy = clean + 0.3 * torch.randn(4, 48000, generator=g).cuda()
    for _ in range(2):
        p, z = model(clean, noisy)
        loss = byol_loss(p, z)
        opt.zero_grad()
        loss.backward()
        opt.step()
        model._update_target_network()
    e.sync_optimizer()
    fresh = torch.empty_like(e.target_lo8)
    K.split_lo8(e.target, fresh, e.lo8_exp)
    torch.cuda.synchronize()
    assert torch.equal(fresh.view(torch.uint8), e.target_lo8.view(torch.uint8))
