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
                  "max_audio_length": 1.0, "snr_range": [0, 5, 10, 15, 20], "validation_ratio": 0.15},
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
