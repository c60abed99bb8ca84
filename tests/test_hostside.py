"""Host-side logic: relative-position buckets, SpecAugment / LayerDrop sampling, parameter
inventory and naming, config schema, RNG contract (CPU only)."""
import os

import numpy as np
import pytest
import torch

from nrse_amd import arch as A, hostside as HS, params as PR, rng as R
from oracle import masks as MK

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_bucket_vector_matches_reference_fixture():
    z = np.load(os.path.join(GOLD, "buckets.npz"))
    for key in z.files:
        np.testing.assert_array_equal(HS.bucket_vector(int(key[1:])), z[key])


def test_span_masks():
    rng = np.random.default_rng(0)
    for T in (49, 399, 599):
        m = HS.compute_mask_indices(rng, 16, T, 0.075, 10, 2)
        n = m.sum(1)
        assert (n >= 10).all() and (n <= 10 * max(2, int(0.075 * T / 10 + 1))).all()
    assert not HS.compute_mask_indices(rng, 4, 100, 0.0, 10, 2).any()


def test_layerdrop_never_drops_layer0():
    rng = np.random.default_rng(1)
    drops = np.array([HS.layerdrop_decisions(rng, 24, 0.1) for _ in range(2000)])
    assert not drops[:, 0].any()
    assert abs(drops[:, 1:].mean() - 0.1) < 0.01


def test_large_param_inventory_matches_wavlm_large():
    # 315,453,120 = WavLM-Large
    assert PR.count_params(PR.encoder_specs(A.LARGE)) == 315_453_120
    L = PR.byol_layout(A.LARGE, 1024, 2048)
    assert sum(n for _, n, _ in L.offsets.values()) == 315_453_120 + 2_103_296 + 8_401_920


@pytest.mark.parametrize("arch", [A.TINY, A.TINY.deterministic()])
def test_state_dict_names_match_transformers(arch):
    from transformers import WavLMConfig, WavLMModel
    m = WavLMModel(WavLMConfig(**arch.to_hf_config()))
    ref = {k: tuple(v.shape) for k, v in m.named_parameters()}
    ours = {s.name: tuple(s.shape) for s in PR.encoder_specs(arch)}
    assert ref == ours


def test_fused_views_are_contiguous():
    L = PR.byol_layout(A.LARGE, 1024, 2048)
    o = L.offsets
    p = "online_encoder.model.encoder.layers.3.attention."
    H = 1024
    assert o[p + "k_proj.weight"][0] == o[p + "q_proj.weight"][0] + H * H
    assert o[p + "v_proj.bias"][0] == o[p + "k_proj.bias"][0] + H


def test_init_is_portable_and_seeded():
    L = PR.byol_layout(A.TINY, 256, 512)
    a = PR.init_byol_flat(L, 5)
    b = PR.init_byol_flat(L, 5)
    c = PR.init_byol_flat(L, 6)
    assert torch.equal(a, b) and not torch.equal(a, c)


def test_rng_contract_matches_oracle_hash():
    for x in (0, 1, 12345, 0xFFFFFFFF, 0xDEADBEEF):
        assert R.mix32(x) == int(MK.mix32(x))
    keep = MK.keep_mask(R.site_seed(7, 3), 0.1, 200000)
    assert abs(keep.mean() - 0.9) < 0.005
    seeds = {R.site_seed(R.forward_seed(s, b, r), site) for s in range(4) for b in (0, 1) for r in range(2)
             for site in range(30)}
    assert len(seeds) == 4 * 2 * 2 * 30


def test_config_schema_and_cli_overrides(tmp_path):
    import yaml
    from nrse_amd.config import get_config
    cfg = {"model": {"name": "microsoft/wavlm-large", "projection_dim": 1024, "prediction_dim": 2048,
                     "ema_decay": 0.997},
           "training": {"batch_size": 36, "num_epochs": 100, "learning_rate": 1e-5, "weight_decay": 1e-5,
                        "checkpoint_dir": "c", "log_dir": "l", "seed": 42},
           "data": {"sample_rate": 16000, "max_audio_length": 5.0, "snr_range": [2, 5, 10, 15, 20]},
           "logging": {"level": "INFO"}}
    p = tmp_path / "c.yaml"
    p.write_text(yaml.safe_dump(cfg))
    out = get_config(["--config", str(p), "--batch_size", "32", "--lr", "3e-5", "--device", "cuda:1"])
    assert out["training"]["batch_size"] == 32 and out["training"]["learning_rate"] == 3e-5
    assert out["device"] == "cuda:1" and out["model"]["ema_decay"] == 0.997
    assert A.arch_from_name(out["model"]["name"]) == A.LARGE


def test_frames():
    assert A.LARGE.frames(128000) == 399 and A.LARGE.frames(80000) == 249


def test_mock_pairs_follow_create_mock_dataset_rule():
    from nrse_amd.data import MockPairs
    ds = MockPairs(10, 800, [0, 5, 10, 15, 20], seed=1)
    assert [int(ds[i]["snr"]) for i in range(10)] == [0, 5, 10, 15, 20] * 2
    for i in range(10):
        d = ds[i]["noisy_input_values"] - ds[i]["clean_input_values"]
        assert abs(float(d.std()) * (int(ds[i]["snr"]) + 1) - 1.0) < 0.15


def test_attention_pair_hash_mask_statistics():
    """The attention-probability dropout mask (one hash per key pair, 16 bits per element): drop
    rate p, and the two elements of a pair independent (joint drop rate p^2)."""
    import numpy as np
    from oracle import masks as MK
    p, rows, T = 0.1, 600, 399
    keep = MK.attn_keep_mask(1234, p, rows, T)
    assert abs(1 - keep.mean() - p) < 0.004
    pairs = keep[:, : T - 1].reshape(rows, -1, 2)
    both = float((~pairs[..., 0] & ~pairs[..., 1]).mean())
    assert abs(both - p * p) < 0.002
    assert MK.threshold16(0.0) == 0 and MK.threshold16(1.0) == 65536
    # ABI 10's full-rate mixer (attn_mix): neighbouring pairs and rows independent too, and the
    # 16-bit halves uniform (chi-square over the top byte within its expectation)
    d = (~keep).astype(np.float64)
    for joint in ((d[:, 1:T - 1:2] * d[:, 2:T:2]).mean(), (d[:-1] * d[1:]).mean(), (d[:-8] * d[8:]).mean()):
        assert abs(joint - p * p) < 0.002, joint
    r = np.arange(rows, dtype=np.uint64)[:, None]
    kp = np.arange((T + 1) // 2, dtype=np.uint64)[None, :]     # one hash per key pair
    h = MK.attn_mix(((r * np.uint64((T + 1) // 2) + kp) & MK.M32) ^ MK.site_key(1234))
    for sh in (0, 8, 16, 24):
        cnt = np.bincount(((h >> np.uint64(sh)) & np.uint64(255)).astype(np.int64).ravel(), minlength=256)
        e = h.size / 256
        assert ((cnt - e) ** 2 / e).sum() / 255 < 1.4, sh
    m = MK.attn_dropout_mask(7, p, (2, 3, T, T))
    assert set(np.unique(m)).issubset({0.0, np.float32(1 / (1 - p))})


def test_bucket_runs_invert_the_bucket_vector():
    """The gather form of the rel-pos bias backward (nrse_rel_bias_bwd) sums bucket k's diagonals
    over order[offsets[k]:offsets[k+1]]: every offset d exactly once, increasing within a bucket."""
    from nrse_amd.hostside import bucket_runs, bucket_vector
    for T in (1, 7, 149, 399):
        b = bucket_vector(T, 320, 800)
        order, offsets = bucket_runs(b, 320)
        assert offsets[0] == 0 and offsets[-1] == 2 * T - 1 and len(offsets) == 321
        assert sorted(order.tolist()) == list(range(2 * T - 1))
        for k in range(320):
            run = order[offsets[k]:offsets[k + 1]]
            assert (b[run] == k).all() and (np.diff(run) > 0).all()


def test_device_span_mask_restatement_semantics():
    """oracle/masks.py specaug_mask (what nrse_specaug_mask draws on the device, ABI 10) keeps the
    reference's span semantics ([TF]modeling_wavlm.py:834-954): n = int(p T / L + eps) spans clamped
    to [min_masks, T // L], shared by the batch; each utterance's n starts distinct and uniformly
    spread over the T - L + 1 candidates; every span L frames; deterministic in the seed."""
    p, L, mn = 0.075, 10, 2
    for T in (49, 149, 399, 599):
        m = MK.specaug_mask(1234, 64, T, p, L, mn)
        assert (m == MK.specaug_mask(1234, 64, T, p, L, mn)).all()
        counts = m.sum(1)
        n_lo = max(int(p * T / L), mn)
        n_hi = max(int(p * T / L + 1), mn)
        # frames covered: n spans of L minus overlaps, never more than n L
        assert (counts <= n_hi * L).all() and (counts >= L).all()
        for b in range(64):
            row = m[b]
            # a masked run's length is a multiple-span union: at least L
            runs = np.diff(np.flatnonzero(np.diff(np.concatenate([[0], row.astype(int), [0]]))))[::2]
            assert (runs >= L).all()
        assert n_lo >= 1
    # uniform starts: over many utterances every candidate is chosen about n / C of the time
    T = 149
    C = T - L + 1
    big = MK.specaug_mask(7, 20000, T, p, L, mn)
    first = np.array([np.flatnonzero(r)[0] for r in big])     # the first span's start (its smallest)
    assert first.min() == 0 and first.max() <= C - 1
    n = mn                                                   # int(0.075 * 149 / 10 + eps) <= 2
    cover = big.mean(0)                                      # per-frame mask rate, flat in the middle
    mid = cover[L:T - L]
    assert abs(mid.mean() - n * L / C) < 0.05 and mid.std() < 0.02, (mid.mean(), mid.std())
    assert not MK.specaug_mask(3, 4, 100, 0.0, 10, 2).any()
    with pytest.raises(ValueError):
        MK.specaug_mask(3, 4, 5, 0.5, 10, 2)
