"""Pin the CPU oracle (oracle/) against golden fixtures produced by the reference itself
(tests/golden/make_golden.py). CPU only."""
import os

import numpy as np
import pytest
import torch

from oracle import snr_mix as SM
from oracle import wavlm_byol as O
from nrse_amd import arch as A, params as PR

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def rel(a, b):
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def test_buckets_match_reference():
    z = np.load(os.path.join(GOLD, "buckets.npz"))
    for key in z.files:
        T = int(key[1:])
        np.testing.assert_array_equal(O.bucket_vector(T).astype(np.int32), z[key])


def test_snr_mix_matches_reference():
    z = np.load(os.path.join(GOLD, "snr_mix.npz"))
    for i in range(int(z["n_cases"])):
        s, n, snr = z[f"c{i}_speech"], z[f"c{i}_noise"], float(z[f"c{i}_snr"])
        c, y, st, k = SM.mix_pair(s, n, snr, do_normalize=True)
        if int(z[f"c{i}_ok"]) == 0:
            assert st != SM.OK, i
            continue
        assert st == SM.OK, (i, st)
        yraw, _, _ = SM.add_noise(s, n, snr)
        assert rel(yraw, z[f"c{i}_noisy_raw"]) < 1e-6
        assert rel(c, z[f"c{i}_clean_iv"]) < 1e-5
        assert rel(y, z[f"c{i}_noisy_iv"]) < 1e-5


def inputs(z):
    """Fixture inputs: stored (tiny) or regenerated from the seed (large), as make_golden did."""
    if "clean" in z.files:
        return torch.from_numpy(z["clean"]), torch.from_numpy(z["noisy"])
    g = torch.Generator().manual_seed(int(z["seed"]) + 1)
    B, L = int(z["B"]), int(z["L"])
    clean = torch.randn(B, 1, L, generator=g)
    noisy = clean + 0.3 * torch.randn(B, 1, L, generator=g)
    return clean.squeeze(1), noisy.squeeze(1)


def _state(tag, arch):
    z = np.load(os.path.join(GOLD, f"byol_{tag}.npz"))
    layout = PR.byol_layout(arch, int(z["proj_dim"]), int(z["pred_dim"]))
    flat = PR.init_byol_flat(layout, int(z["seed"]))
    return z, layout, O.OracleState(layout, flat)


# the WavLM-Large 8 s / 12 s pins take ~5-13 CPU-minutes each (one oracle train step of 317 M
# weights): opt-in (NRSE_ORACLE_FULL=1) so the default CPU suite stays within minutes; the 3 s
# pin of the same code path, the tiny ones and the 8 s split-weight check always run
_FULL = os.environ.get("NRSE_ORACLE_FULL") == "1"
_LONG = pytest.mark.skipif(not _FULL, reason="WavLM-Large 8 s / 12 s oracle pins: NRSE_ORACLE_FULL=1")
_TAGS = ["tiny", pytest.param("large", marks=_LONG), "large_3s", pytest.param("large_12s", marks=_LONG)]


@pytest.mark.parametrize("tag", _TAGS)
def test_oracle_eval_forward(tag):
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    arch = (A.TINY if tag == "tiny" else A.LARGE).deterministic()
    z, layout, st = _state(tag, arch)
    clean, noisy = inputs(z)
    with torch.no_grad():
        pred, tproj, emb = O.forward(st, clean, noisy, train=False)
        loss = O.byol_loss(pred, tproj)
    assert rel(emb, z["eval_emb"]) < 1e-5
    assert rel(pred, z["eval_pred"]) < 1e-4
    assert rel(tproj, z["eval_tproj"]) < 1e-4
    assert abs(float(loss) - float(z["eval_loss"])) < 1e-4
    if tag == "tiny":
        on = O.split_flat(layout, st.online)
        h = O.encoder_forward(on["encoder"], arch, clean)
        assert rel(h, z["eval_hidden"]) < 1e-5


@pytest.mark.parametrize("tag", _TAGS)
def test_oracle_train_step(tag):
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    arch = (A.TINY if tag == "tiny" else A.LARGE).deterministic()
    z, layout, st = _state(tag, arch)
    flat0 = st.online.clone()
    clean, noisy = inputs(z)
    r = O.train_step(st, clean, noisy, lr=float(z["lr"]), weight_decay=float(z["wd"]), ema_decay=float(z["ema"]))
    assert abs(r["loss"] - float(z["train_loss"])) < 1e-4
    # BatchNorm backward in the heads amplifies fp32 summation-order differences (~1e-4)
    assert abs(r["grad_norm"] - float(z["train_grad_norm"])) / float(z["train_grad_norm"]) < 1e-3
    norms = []
    for gname, s in layout.specs:
        off, cnt, _ = layout.offsets[PR.GROUP_PREFIX[gname] + s.name]
        norms.append(float(r["grad"][off:off + cnt].norm()))
    norms = np.array(norms)
    ref = z["grad_tensor_norms"]
    big = ref > 1e-3 * ref.max()
    assert np.max(np.abs(norms[big] - ref[big]) / ref[big]) < 1e-3
    idx = z["grad_idx"]
    assert rel(r["grad"][idx].numpy(), z["grad_sample"]) < 1e-3
    # AdamW first step moves each weight by ~lr*sign(g) (+ decoupled wd): compare in units of lr
    lr = float(z["lr"])
    d = (st.online - flat0)[idx].numpy()
    mism = np.abs(d - z["online_delta_sample"]) > 0.05 * lr
    assert mism.mean() < 0.01, mism.mean()
    tidx = z["target_idx"]
    dt = (st.target - flat0[:layout.ema_numel])[tidx].numpy()
    assert np.max(np.abs(dt - z["target_delta_sample"])) < 0.05 * lr


def test_emotion_head_oracle_matches_reference_fixture():
    """oracle/emotion_head.py vs the reference EmotionClassifier (+ its pooling and ccc_loss) on
    the same hidden states, ragged masks and parameters (tests/golden/make_golden_emotion.py)."""
    from oracle import emotion_head as E
    z = np.load(os.path.join(GOLD, "emotion_head.npz"))
    P = {k[6:]: torch.from_numpy(z[k]).clone().requires_grad_(True) for k in z.files if k.startswith("param/")}
    hidden = torch.from_numpy(z["hidden"])
    lens = E.feat_lengths(torch.from_numpy(z["mask"]))
    assert lens == z["feat_lens"].tolist()
    out, _ = E.dimensional_forward(hidden, lens, P)
    assert torch.allclose(out, torch.from_numpy(z["dim"]), rtol=1e-5, atol=1e-6)
    loss = E.ccc_loss(out, torch.from_numpy(z["labels"]))
    assert abs(float(loss) - float(z["loss"])) < 1e-6
    loss.backward()
    for k in z.files:
        if k.startswith("grad/"):
            g = P[k[5:]].grad
            ref = torch.from_numpy(z[k])
            assert torch.allclose(g, ref, rtol=1e-4, atol=1e-7), k


def _tiny_setup(B=8, L=16000):
    arch = A.TINY.deterministic()
    layout = PR.byol_layout(arch, 256, 512)
    flat = PR.init_byol_flat(layout, 1234)
    g = torch.Generator().manual_seed(5)
    clean = torch.randn(B, L, generator=g)
    noisy = clean + 0.3 * torch.randn(B, L, generator=g)
    return arch, layout, flat, clean, noisy


def test_head_gradient_conditioning():
    """Documents why end-to-end bf16 gradients cannot be compared tightly at random init: the
    heads' BatchNorm over a batch of near-identical embeddings amplifies a 1e-4 relative
    perturbation of the embedding into a >1e-2 change of d(loss)/d(emb) (measured ~8e-2)."""
    arch, layout, flat, clean, noisy = _tiny_setup()
    st = O.OracleState(layout, flat)
    with torch.no_grad():
        _, tproj, emb = O.forward(st, clean, noisy, train=True)

    def demb(e):
        s2 = O.OracleState(layout, flat)
        on = O.split_flat(layout, s2.online)
        e = e.clone().requires_grad_(True)
        proj = O.projector(on["projector"], e, s2.buffers["online_projector"], True)
        O.byol_loss(O.predictor(on["predictor"], proj, s2.buffers["online_predictor"], True), tproj).backward()
        return e.grad
    g0 = demb(emb)
    g1 = demb(emb * (1 + 1e-4 * torch.randn(emb.shape, generator=torch.Generator().manual_seed(1))))
    assert rel(g1.numpy(), g0.numpy()) > 1e-2


def test_oracle_bf16_operand_mode():
    """The oracle's bf16-operand mode (the engine's bf16 numerics): embeddings within bf16
    rounding of f32, encoder gradient under a fixed upstream gradient within 2e-2, and the
    default f32 mode is untouched afterwards."""
    arch, layout, flat, clean, _ = _tiny_setup(B=4)
    R = torch.randn(4, arch.hidden, generator=torch.Generator().manual_seed(9))
    out = {}
    for dt in (None, torch.bfloat16):
        O.set_operand_dtype(dt)
        try:
            P = O.split_flat(layout, flat.clone(), leaves=True)
            e = O.encoder_forward(P["encoder"], arch, clean, train=True).mean(1)
            (e * R).sum().backward()
        finally:
            O.set_operand_dtype(None)
        out[dt] = (e.detach(), O.gather_grad(layout, P))
    assert O.operand_dtype() is None
    e_rel = rel(out[torch.bfloat16][0].numpy(), out[None][0].numpy())
    g_rel = rel(out[torch.bfloat16][1].numpy(), out[None][1].numpy())
    assert 1e-4 < e_rel < 1e-2, e_rel      # rounded (not a no-op), but only at bf16 level
    assert g_rel < 2e-2, g_rel


def test_oracle_split_weight_mode_meets_north_star():
    """The split-weight mode's numerics (the weights and the conv stack's activations exact, every
    other activation operand in bf16: O.SPLIT_WEIGHT_SITES) at WavLM-Large, 8 s, against the
    reference's own embeddings
    (byol_large.npz): within the north-star 1e-3, while the full bf16-operand mode is not --
    the weight rounding, shared by every frame and kept by the time mean, carries the bf16
    mode's deviation (tools/ablate_bf16_sites.py)."""
    from nrse_amd import arch as A, params as PR
    z = np.load(os.path.join(GOLD, "byol_large.npz"))
    arch = A.LARGE.deterministic()
    layout = PR.byol_layout(arch, int(z["proj_dim"]), int(z["pred_dim"]))
    flat = PR.init_byol_flat(layout, int(z["seed"]))
    g = torch.Generator().manual_seed(int(z["seed"]) + 1)
    clean = torch.randn(int(z["B"]), 1, int(z["L"]), generator=g).squeeze(1)[:2]
    P = O.split_flat(layout, flat)["encoder"]
    ref = z["eval_emb"][:2]
    # the fp8 form's exponent as the engine picks it (ByolEngine._set_lo8_planes)
    e8 = O.lo8_exponent([P[f"encoder.layers.{li}.{n}"] for li in range(arch.layers)
                         for n in ("attention.q_proj.weight", "attention.k_proj.weight", "attention.v_proj.weight",
                                   "attention.out_proj.weight", "feed_forward.intermediate_dense.weight",
                                   "feed_forward.output_dense.weight")])
    out = {}
    for name, sites, s8 in (("split", O.SPLIT_WEIGHT_SITES, None),
                            ("split_fp8", O.SPLIT_WEIGHT_SITES, O.SPLIT8_SITES),
                            ("bf16", None, None)):
        O.set_operand_dtype(torch.bfloat16, sites)
        O.set_split8(s8, e8)
        try:
            with torch.no_grad():
                out[name] = rel(O.encoder_forward(P, arch, clean, train=False).mean(1).numpy(), ref)
        finally:
            O.set_operand_dtype(None)
            O.set_split8(None)
    print("split-weight oracle rel-L2 vs reference:", out)
    assert out["split"] < 1e-3, out
    assert out["split_fp8"] < 1e-3, out     # the engine's default bf16sw (fp8 correction segments, ABI 6 / 7)
    # (ABI 8-10's MXFP6 form of the corrections measured 3.80e-4 here, profiles/r05_mx6_ab.txt, and
    # was retired in ABI 11: slower on this part at the same accuracy)
    assert out["bf16"] > 3e-3, out
