"""Drop-in API on the GPU: reference-style training loop over BYOLSpeechModel / byol_loss /
_update_target_network matches the fused engine step and the oracle; state_dict round trip;
add_noise_to_speech; the train_byol CLI runs end to end on synthetic data."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from oracle import wavlm_byol as O
from nrse_amd import arch as A, params as PR

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "noise-robust-speech-embedding_amd")


def cfg(name="nrse/wavlm-tiny"):
    return {"model": {"name": name, "projection_dim": 256, "prediction_dim": 512, "ema_decay": 0.99},
            "training": {"learning_rate": 1e-4, "weight_decay": 1e-5, "seed": 3}}


def test_reference_style_loop_matches_oracle(nrse_device):
    sys.path.insert(0, PKG)
    from src.models.byol import BYOLSpeechModel, byol_loss   # the reference import path
    arch = A.TINY.deterministic()
    model = BYOLSpeechModel(cfg(), compute_dtype=torch.float32, arch=arch)
    flat0 = model.engine.online.detach().cpu().clone()
    st = O.OracleState(model.engine.layout, flat0.clone())
    g = torch.Generator().manual_seed(9)
    clean = torch.randn(8, 1, 16000, generator=g)
    noisy = clean + 0.3 * torch.randn(8, 1, 16000, generator=g)
    model.train()
    pred, tproj = model(clean.cuda(), noisy.cuda())
    loss = byol_loss(pred, tproj)
    loss.backward()
    grad = model.online_flat.grad
    r = O.train_step(st, clean.squeeze(1), noisy.squeeze(1), lr=1e-4, weight_decay=1e-5, ema_decay=0.99)
    assert abs(float(loss) - r["loss"]) < 1e-4
    assert float((grad.cpu() - r["grad"]).norm() / r["grad"].norm()) < 1e-3
    # torch optimizer over the flat parameter + reference clip + EMA
    torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=1e-5)
    opt.step()
    model._update_target_network()
    # Adam's first step is ~lr*sign(g): entries whose gradient is at the fp32 noise floor may flip
    # sign, so compare the update vectors (rel-L2) and bound the fraction of flipped entries.
    d_ours = model.engine.online.cpu() - flat0
    d_ref = st.online - flat0
    assert float((d_ours - d_ref).norm() / d_ref.norm()) < 0.05
    assert float(((d_ours - d_ref).abs() > 1e-6).float().mean()) < 0.01
    t_ours = model.engine.target.cpu() - flat0[:st.target.numel()]
    t_ref = st.target - flat0[:st.target.numel()]
    assert float((t_ours - t_ref).norm() / t_ref.norm()) < 0.05


def test_state_dict_roundtrip_and_keys(nrse_device):
    from nrse_amd.model import BYOLSpeechModel
    m = BYOLSpeechModel(cfg(), arch=A.TINY)
    sd = m.state_dict()
    assert "online_encoder.model.encoder.pos_conv_embed.conv.parametrizations.weight.original0" in sd
    assert "target_projector.layers.4.running_var" in sd and "online_predictor.layers.6.bias" in sd
    assert not any(k.startswith("target_predictor") for k in sd)
    m2 = BYOLSpeechModel({**cfg(), "training": {**cfg()["training"], "seed": 99}}, arch=A.TINY)
    m2.load_state_dict(sd)
    assert torch.equal(m2.engine.online, m.engine.online) and torch.equal(m2.engine.target, m.engine.target)
    emb1 = m.get_encoder()(torch.randn(2, 1, 16000).cuda())
    assert emb1.shape == (2, 256)


def test_add_noise_to_speech_dropin(nrse_device):
    sys.path.insert(0, PKG)
    from src.data.augment import add_noise_to_speech
    z = np.load(os.path.join(ROOT, "tests", "golden", "snr_mix.npz"))
    for i in range(int(z["n_cases"])):
        s = torch.from_numpy(z[f"c{i}_speech"])[None].cuda()
        n = torch.from_numpy(z[f"c{i}_noise"])[None].cuda()
        y = add_noise_to_speech(s, n, float(z[f"c{i}_snr"]))
        if int(z[f"c{i}_ok"]) == 0:
            assert y is None
        else:
            ref = torch.from_numpy(z[f"c{i}_noisy_raw"]).cuda()
            assert float((y[0] - ref).norm() / ref.norm()) < 1e-6


def test_train_cli_synthetic(nrse_device, tmp_path):
    import yaml
    c = {"model": {"name": "nrse/wavlm-tiny", "projection_dim": 256, "prediction_dim": 512, "ema_decay": 0.996},
         "training": {"batch_size": 4, "num_workers": 0, "num_epochs": 1, "learning_rate": 1e-5,
                      "weight_decay": 1e-5, "checkpoint_dir": str(tmp_path / "ck"), "log_dir": str(tmp_path / "lg"),
                      "seed": 42, "early_stopping_metric": "val_loss", "early_stopping_patience": 4},
         "data": {"clean_data_path": "/nonexistent", "noise_data_path": "/nonexistent", "sample_rate": 16000,
                  "max_audio_length": 1.0, "snr_range": [0, 5, 10, 15, 20], "validation_ratio": 0.15,
                  "synthetic": 256},
         "logging": {"level": "WARNING"}}
    p = tmp_path / "c.yaml"
    p.write_text(yaml.safe_dump(c))
    out = subprocess.run([sys.executable, os.path.join(PKG, "train_byol.py"), "--config", str(p), "--device",
                          "cuda:0", "--max_steps", "6"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    assert "Epoch 1/1" in out.stdout
    ck = torch.load(tmp_path / "ck" / "last_model.pt", weights_only=True, map_location="cpu")
    assert "online_encoder.model.encoder.layers.0.attention.rel_attn_embed.weight" in ck["model_state_dict"]


def test_dev_yaml_cli_on_mock_dataset(nrse_device, tmp_path):
    """configs[0]: the reference's dev YAML (config/dev_wavlm-large_byol.yaml, as a fixture) through
    the train_byol CLI at batch 2 on test/create_mock_dataset.py-style pairs (SNR cycling through
    snr_range, noise level 1/(snr+1)), WavLM-Large, one epoch capped at 3 steps."""
    conf = os.path.join(ROOT, "tests", "golden", "configs", "dev_wavlm-large_byol.yaml")
    out = subprocess.run([sys.executable, os.path.join(PKG, "train_byol.py"), "--config", conf, "--device", "cuda:0",
                          "--batch_size", "2", "--epochs", "1", "--mock_items", "16", "--max_steps", "3"],
                         capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    assert out.returncode == 0, out.stderr[-3000:]
    assert "Epoch 1/1" in out.stdout, out.stdout
    ck = torch.load(tmp_path / "checkpoints/byol/wavlm_large-val_loss/last_model.pt", weights_only=True,
                    map_location="cpu")
    sd = ck["model_state_dict"]
    assert sd["online_encoder.model.encoder.layers.23.feed_forward.output_dense.weight"].shape == (1024, 4096)
    assert sd["online_predictor.layers.6.weight"].shape == (1024, 2048)
    assert np.isfinite(ck["loss"])


def test_checkpoint_interop_reference_layout(nrse_device, tmp_path):
    """f3: checkpoints in the reference format. (1) state_dict() has exactly the reference
    BYOLSpeechModel's keys, shapes and dtypes (tests/golden/state_manifest.json, dumped from
    the reference by make_golden.py --manifest-only). (2) A checkpoint written the way
    train_byol.py:207-240 writes it ({'model_state_dict': ...}, the reference's weights of the
    byol_tiny fixture) loads strictly, after torch.load(weights_only=True), and reproduces the
    reference's eval outputs. (3) torch semantics: unexpected keys and shape mismatches raise."""
    import json
    from nrse_amd.model import BYOLSpeechModel
    man = json.load(open(os.path.join(ROOT, "tests", "golden", "state_manifest.json")))["tiny"]
    z = np.load(os.path.join(ROOT, "tests", "golden", "byol_tiny.npz"))
    c = cfg()
    c["model"].update(projection_dim=int(z["proj_dim"]), prediction_dim=int(z["pred_dim"]), ema_decay=float(z["ema"]))
    m = BYOLSpeechModel(c, arch=A.TINY.deterministic(), compute_dtype=torch.float32)
    sd = m.state_dict()
    ours = {k: [list(v.shape), str(v.dtype).replace("torch.", "")] for k, v in sd.items()}
    assert ours == {k: [shp, dt] for k, shp, dt in man}   # (load_state_dict matches by key, not order)
    # the reference's weights of the fixture, keyed as its state_dict (target = online copy)
    layout = PR.byol_layout(A.TINY.deterministic(), int(z["proj_dim"]), int(z["pred_dim"]))
    views = PR.named_views(layout, PR.init_byol_flat(layout, int(z["seed"])))
    ref_sd = {}
    for k, shp, dt in man:
        src = k.replace("target_", "online_", 1) if k.startswith("target_") else k
        if src in views:
            ref_sd[k] = views[src].clone().reshape(shp)
        elif k.endswith("running_mean"):
            ref_sd[k] = torch.zeros(shp)
        elif k.endswith("running_var"):
            ref_sd[k] = torch.ones(shp)
        else:
            ref_sd[k] = torch.zeros(shp, dtype=torch.long)
    torch.save({"epoch": 0, "model_state_dict": ref_sd, "optimizer_state_dict": {}, "loss": 0.0, "similarity": 0.0},
               tmp_path / "best_val_loss.pt")
    ck = torch.load(tmp_path / "best_val_loss.pt", weights_only=True, map_location="cpu")
    m2 = BYOLSpeechModel({**c, "training": {**c["training"], "seed": 77}}, arch=A.TINY.deterministic(),
                         compute_dtype=torch.float32)
    res = m2.load_state_dict(ck["model_state_dict"])
    assert res.missing_keys == [] and res.unexpected_keys == []
    m2.eval()
    with torch.no_grad():
        pred, tproj = m2(torch.from_numpy(z["clean"]).cuda()[:, None], torch.from_numpy(z["noisy"]).cuda()[:, None])
    for got, key in ((pred, "eval_pred"), (tproj, "eval_tproj")):
        ref = torch.from_numpy(z[key])
        assert float((got.cpu() - ref).norm() / ref.norm()) < 1e-4, key
    bad = dict(ck["model_state_dict"])
    bad["online_projector.layers.9.weight"] = torch.zeros(3)
    with pytest.raises(RuntimeError, match="Unexpected"):
        m2.load_state_dict(bad)
    assert m2.load_state_dict(bad, strict=False).unexpected_keys == ["online_projector.layers.9.weight"]
    bad = dict(ck["model_state_dict"])
    bad["online_predictor.layers.0.weight"] = bad["online_predictor.layers.0.weight"].t().contiguous()
    with pytest.raises(RuntimeError, match="size mismatch"):
        m2.load_state_dict(bad)


def test_validate_model_matches_oracle(nrse_device):
    """f2: train.validate_model (evaluate_byol.py:12-123: per-SNR mean cosine similarity of the
    online encoder's clean vs noisy embeddings, mean eval-mode BYOL loss over batches) equals the
    same computation on the oracle, for a model after one training step (non-trivial BN running
    statistics), over ragged SNR groups and a short last batch."""
    from nrse_amd import train as TR
    from nrse_amd.model import BYOLSpeechModel
    arch = A.TINY.deterministic()
    c = cfg()
    m = BYOLSpeechModel(c, arch=arch, compute_dtype=torch.float32, seed=5)
    layout = PR.byol_layout(arch, 256, 512)
    g = torch.Generator().manual_seed(11)
    wav = torch.randn(9, 16000, generator=g) * 0.1
    noise = torch.randn(9, 16000, generator=g) * 0.1
    snr_range = [0, 5, 10, 15, 20]
    snrs = torch.tensor([0, 5, 5, 10, 20, 20, 20, 0, 15])
    noisy = wav + noise / (snrs[:, None].float() + 1)
    # one fused step first, so the BN running buffers are not at their init values
    m.engine.train_step(wav[:4].cuda(), noisy[:4].cuda(), lr=1e-4, step_seed=3)
    batches = [dict(clean_input_values=wav[i:i + 4, None], noisy_input_values=noisy[i:i + 4, None], snr=snrs[i:i + 4])
               for i in range(0, 9, 4)]
    val_loss, met = TR.validate_model(m, batches, "cuda", {"data": {"snr_range": snr_range}})
    # oracle: the same weights and BN buffers, eval mode
    st = O.OracleState(layout, m.engine.online.detach().cpu())
    st.target = m.engine.target.detach().cpu().clone()
    sd = m.state_dict()
    for key in sd:
        if key.endswith("running_mean") or key.endswith("running_var"):
            net, rest = key.split(".", 1)
            st.buffers[net][rest].copy_(sd[key].cpu())
    assert float(st.buffers["online_projector"]["layers.1.running_var"].sub(1).abs().max()) > 0
    sims = {s: [] for s in snr_range}
    losses = []
    with torch.no_grad():
        for b in batches:
            cl, nz = b["clean_input_values"][:, 0], b["noisy_input_values"][:, 0]
            pred, tproj, ec = O.forward(st, cl, nz, train=False)
            _, _, en = O.forward(st, nz, cl, train=False)
            s = torch.nn.functional.cosine_similarity(ec, en, dim=1)
            for i, snr in enumerate(b["snr"].tolist()):
                sims[snr].append(float(s[i]))
            losses.append(float(O.byol_loss(pred, tproj)))
    ref = {k: sum(v) / len(v) for k, v in sims.items()}
    for k in snr_range:
        assert abs(met["val_similarities"][k] - ref[k]) < 1e-5, (k, met["val_similarities"][k], ref[k])
    assert abs(met["val_avg_similarity"] - sum(ref.values()) / len(ref)) < 1e-5
    assert abs(val_loss - sum(losses) / len(losses)) < 1e-4 * max(1.0, abs(val_loss))


def test_cli_early_stop_precedes_checkpoints(nrse_device, tmp_path):
    """train_byol.py:192-196 before :207-240: on the epoch where early stopping fires the loop
    breaks before saving anything. patience 1 and an unreachable min_delta stop at epoch 2, so
    every checkpoint holds epoch 0 and no last_model.pt exists; the checkpoint's
    optimizer_state_dict carries the AdamW moments (exp_avg / exp_avg_sq per parameter)."""
    import yaml
    c = {"model": {"name": "nrse/wavlm-tiny", "projection_dim": 256, "prediction_dim": 512, "ema_decay": 0.996},
         "training": {"batch_size": 4, "num_workers": 0, "num_epochs": 3, "learning_rate": 1e-5,
                      "weight_decay": 1e-5, "checkpoint_dir": str(tmp_path / "ck"), "log_dir": str(tmp_path / "lg"),
                      "seed": 42, "early_stopping_metric": "val_loss", "early_stopping_patience": 1,
                      "early_stopping_min_delta": 1e9},
         "data": {"clean_data_path": "/nonexistent", "noise_data_path": "/nonexistent", "sample_rate": 16000,
                  "max_audio_length": 0.5, "snr_range": [0, 5, 10, 15, 20], "validation_ratio": 0.15,
                  "synthetic": 256},
         "logging": {"level": "WARNING"}}
    p = tmp_path / "c.yaml"
    p.write_text(yaml.safe_dump(c))
    out = subprocess.run([sys.executable, os.path.join(PKG, "train_byol.py"), "--config", str(p), "--device",
                          "cuda:0"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    assert "Early stopping triggered after epoch 2" in out.stdout, out.stdout
    assert not (tmp_path / "ck" / "last_model.pt").exists()
    ck = torch.load(tmp_path / "ck" / "best_val_loss.pt", weights_only=True, map_location="cpu")
    assert ck["epoch"] == 0
    osd = ck["optimizer_state_dict"]
    names = osd["param_groups"][0]["param_names"]
    assert len(osd["state"]) == len(names) > 0
    i = names.index("online_predictor.layers.6.weight")
    assert osd["state"][i]["exp_avg"].shape == ck["model_state_dict"][names[i]].shape
    assert float(osd["state"][i]["exp_avg_sq"].abs().sum()) > 0


def test_optimizer_state_roundtrip_resumes(nrse_device, tmp_path):
    """FusedAdamW.state_dict / load_state_dict (the optimizer half of train_byol.py:209-215):
    a model + optimizer restored from a torch.save'd checkpoint take the same next step as the
    run they were saved from."""
    from nrse_amd import arch as A
    from nrse_amd.model import BYOLSpeechModel
    from nrse_amd.train import FusedAdamW
    cfg = {"model": {"name": "nrse/wavlm-tiny", "projection_dim": 256, "prediction_dim": 512, "ema_decay": 0.996},
           "training": {"learning_rate": 1e-4, "weight_decay": 1e-5, "seed": 42}}
    det = A.TINY.deterministic()   # no dropout / SpecAugment / LayerDrop draws tied to the model's seed
    g = torch.Generator().manual_seed(11)
    clean = (torch.randn(4, 16000, generator=g) * 0.1).cuda()
    noisy = clean + 0.05 * torch.randn(4, 16000, generator=g).cuda()
    m1 = BYOLSpeechModel(cfg, compute_dtype=torch.float32, arch=det)
    o1 = FusedAdamW(m1, lr=1e-4, weight_decay=1e-5)
    for i in range(2):
        m1.engine.train_step(clean, noisy, lr=o1.lr, step_seed=i)
    torch.save({"model_state_dict": m1.state_dict(), "optimizer_state_dict": o1.state_dict()}, tmp_path / "ck.pt")
    ck = torch.load(tmp_path / "ck.pt", weights_only=True, map_location="cpu")
    assert int(ck["optimizer_state_dict"]["state"][0]["step"]) == 2
    m2 = BYOLSpeechModel(cfg, compute_dtype=torch.float32, seed=7, arch=det)
    o2 = FusedAdamW(m2, lr=1e-4, weight_decay=1e-5)
    m2.load_state_dict(ck["model_state_dict"])
    o2.load_state_dict(ck["optimizer_state_dict"])
    assert torch.equal(m2.engine.m, m1.engine.m) and torch.equal(m2.engine.v, m1.engine.v)
    assert m2.engine.step_count == 2
    before = m1.engine.online.clone()
    for m, o in ((m1, o1), (m2, o2)):
        m.engine.train_step(clean, noisy, lr=o.lr, step_seed=5)
    torch.cuda.synchronize()
    # the two third steps differ only by the float-atomic summation order of the gradients (the
    # k_proj biases, whose exact gradient is 0, carry pure rounding noise that Adam normalises
    # to O(lr) steps): compare against the size of the step itself
    step = (m1.engine.online - before).double()
    d = float((m2.engine.online - m1.engine.online).double().norm() / step.norm())
    assert d < 1e-2, d
    # a fresh optimizer (no moments) takes a visibly different step: the restored state matters
    m3 = BYOLSpeechModel(cfg, compute_dtype=torch.float32, arch=det)
    m3.load_state_dict(ck["model_state_dict"])
    m3.engine.train_step(clean, noisy, lr=1e-4, step_seed=5)
    torch.cuda.synchronize()
    assert float((m3.engine.online - m1.engine.online).double().norm() / step.norm()) > 0.1
