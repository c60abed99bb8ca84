"""Generate the golden fixtures in tests/golden/ by running the REFERENCE itself.

Runs only in the build container (it imports /root/reference and the third-party
transformers 5.15.0 that the reference calls into); the GPU box only reads the .npz outputs.

What is generated (SURVEY.md §8c recipe):
  * snr_mix.npz   — add_noise_to_speech (src/data/augment.py:4) + peak normalisation
                    (src/data/noisy_speech_dataset.py:88-103) + Wav2Vec2FeatureExtractor
                    normalisation ([TF] feature_extraction_wav2vec2.py:78-97), incl. None cases
  * buckets.npz   — WavLMAttention._relative_positions_bucket ([TF]modeling_wavlm.py:253-271)
  * byol_tiny.npz — reference BYOLSpeechModel + byol_loss on a tiny WavLM arch: eval forward and
                    one deterministic train step (train_byol.py:56-74 loop body)
  * byol_large.npz— WavLM-Large arch, 4 x 8 s, eval forward and one det train step
  * byol_large_3s.npz / byol_large_12s.npz — the same at the ends of configs[4]'s 3-12 s
                    range (T = 149 and 599 frames), 4 utterances each (--varlen)
  * traj_large_3s.npz — WavLM-Large det-train trajectory, 6 steps of B = 4 x 3 s with the
                    reference's AdamW + CosineAnnealingLR, per-step loss / pre-clip grad norm, a
                    held-out batch's embeddings after the last step (--trajectory)
Weights come from nrse_amd.params (portable seeded init), written to a local HF directory the
reference loads through AutoModel.from_pretrained(config['model']['name']) (src/models/
encoder.py:14). The reference's 3-D encoder output is pooled with a time-mean monkeypatch
(documented deviation); reference files are not modified.

Usage: PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [--skip-large]
"""
from __future__ import annotations

import argparse
import os
import sys
import tempfile

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, os.path.join(ROOT, "noise-robust-speech-embedding_amd"))
sys.path.insert(0, REF)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from nrse_amd import arch as A, params as PR  # noqa: E402

SEED = 1234


def build_reference_model(arch, proj_dim, pred_dim, ema, tmpdir):
    from safetensors.torch import save_file
    from transformers import WavLMConfig, Wav2Vec2FeatureExtractor
    import src.models.encoder as enc_mod
    from src.models.byol import BYOLSpeechModel

    # time-mean pooling shim: the reference returns last_hidden_state [B,T,H]
    if not getattr(enc_mod.WavLMEncoder, "_nrse_shim", False):
        orig = enc_mod.WavLMEncoder.forward

        def pooled(self, input_values, attention_mask=None):
            out = orig(self, input_values, attention_mask)
            return out.mean(dim=1) if out.dim() == 3 else out
        enc_mod.WavLMEncoder.forward = pooled
        enc_mod.WavLMEncoder._nrse_shim = True

    layout = PR.byol_layout(arch, proj_dim, pred_dim)
    flat = PR.init_byol_flat(layout, SEED)
    views = PR.named_views(layout, flat)
    enc_sd = {k[len("online_encoder.model."):]: v.clone() for k, v in views.items()
              if k.startswith("online_encoder.model.")}
    cfg = WavLMConfig(**arch.to_hf_config())
    cfg.save_pretrained(tmpdir)
    save_file({k: v.contiguous() for k, v in enc_sd.items()}, os.path.join(tmpdir, "model.safetensors"))
    Wav2Vec2FeatureExtractor(do_normalize=True).save_pretrained(tmpdir)
    config = {"model": {"name": tmpdir, "projection_dim": proj_dim, "prediction_dim": pred_dim, "ema_decay": ema}}
    model = BYOLSpeechModel(config)
    sd = model.state_dict()
    for k, v in views.items():
        assert k in sd, k
        sd[k] = v.clone()
    for k in list(sd):
        if k.startswith("target_"):
            src = k.replace("target_", "online_", 1)
            if src in views:
                sd[k] = views[src].clone()
    missing = model.load_state_dict(sd, strict=True)
    return model, layout, flat


def flat_from_model(model, layout, target=False):
    sd = model.state_dict()
    n = layout.ema_numel if target else layout.numel
    out = torch.zeros(n)
    for gname, s in layout.specs:
        key = PR.GROUP_PREFIX[gname] + s.name
        off, cnt, _ = layout.offsets[key]
        if target:
            if gname == "predictor":
                continue
            key = PR.TARGET_PREFIX[gname] + s.name
        out[off:off + cnt] = sd[key].reshape(-1).float()
    return out


def flat_grad(model, layout):
    out = torch.zeros(layout.numel)
    named = dict(model.named_parameters())
    for gname, s in layout.specs:
        key = PR.GROUP_PREFIX[gname] + s.name
        off, cnt, _ = layout.offsets[key]
        g = named[key].grad
        if g is not None:
            out[off:off + cnt] = g.reshape(-1)
    return out


def sample_idx(n, count=4096, seed=0):
    r = np.random.default_rng(seed)
    return np.sort(r.choice(n, size=min(n, count), replace=False)).astype(np.int64)


def per_tensor_norms(flat, layout):
    out = []
    for gname, s in layout.specs:
        off, cnt, _ = layout.offsets[PR.GROUP_PREFIX[gname] + s.name]
        out.append(float(flat[off:off + cnt].norm()))
    return np.array(out, np.float64)


def make_inputs(B, L, seed=SEED + 1):
    """Inputs of the BYOL fixtures (regenerated identically by the tests from the seed)."""
    g = torch.Generator().manual_seed(seed)
    clean = torch.randn(B, 1, L, generator=g)
    noisy = clean + 0.3 * torch.randn(B, 1, L, generator=g)
    return clean, noisy


def run_byol(arch, B, L, proj_dim, pred_dim, ema, lr, wd, tag, full_hidden, store_inputs):
    from src.models.byol import byol_loss
    with tempfile.TemporaryDirectory() as td:
        model, layout, flat0 = build_reference_model(arch, proj_dim, pred_dim, ema, td)
        clean, noisy = make_inputs(B, L)
        res = {"B": B, "L": L, "proj_dim": proj_dim, "pred_dim": pred_dim, "ema": ema, "lr": lr, "wd": wd,
               "seed": SEED}
        if store_inputs:
            res.update(clean=clean.squeeze(1).numpy(), noisy=noisy.squeeze(1).numpy())
        # eval-mode forward
        model.eval()
        with torch.no_grad():
            pred, tproj = model(clean, noisy)
            loss = byol_loss(pred, tproj)
            emb_c = model.get_encoder()(clean)
            hs = model.online_encoder.model(clean.squeeze(1)).last_hidden_state
        res.update(eval_pred=pred.numpy(), eval_tproj=tproj.numpy(), eval_loss=float(loss), eval_emb=emb_c.numpy())
        if full_hidden:
            res["eval_hidden"] = hs.numpy()
        else:
            res["eval_hidden_norms"] = hs.norm(dim=-1).numpy()
            res["eval_hidden_sample"] = hs[:, ::37, ::13].numpy()
        # one deterministic train step (train_byol.py:56-74 loop body; the function itself calls
        # torch.cuda.device(), which fails on CPU)
        model.train()
        opt = torch.optim.AdamW(model.parameters(), lr=lr, weight_decay=wd)
        pred, tproj = model(clean, noisy)
        loss = byol_loss(pred, tproj)
        opt.zero_grad()
        loss.backward()
        gflat = flat_grad(model, layout)
        gn = torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1.0)
        opt.step()
        model._update_target_network()
        on1 = flat_from_model(model, layout)
        tg1 = flat_from_model(model, layout, target=True)
        idx = sample_idx(layout.numel)
        tidx = sample_idx(layout.ema_numel, seed=1)
        res.update(train_pred=pred.detach().numpy(), train_tproj=tproj.detach().numpy(), train_loss=float(loss),
                   train_grad_norm=float(gn), grad_tensor_norms=per_tensor_norms(gflat, layout),
                   grad_idx=idx, grad_sample=gflat[idx].numpy(),
                   online_delta_sample=(on1 - flat0)[idx].numpy(),
                   target_delta_sample=(tg1 - flat0[:layout.ema_numel])[tidx].numpy(), target_idx=tidx,
                   bn_running=np.concatenate([model.state_dict()[k].numpy().ravel() for k in
                                              ("online_projector.layers.1.running_mean",
                                               "online_projector.layers.1.running_var",
                                               "target_projector.layers.4.running_var")]))
        np.savez_compressed(os.path.join(HERE, f"byol_{tag}.npz"), **res)
        print(f"byol_{tag}: eval loss {res['eval_loss']:.6f} train loss {res['train_loss']:.6f} "
              f"grad norm {res['train_grad_norm']:.4f}")


def run_trajectory(arch, B, L, steps, proj_dim, pred_dim, ema, lr, wd, tag):
    """A det-train TRAJECTORY on the reference: `steps` iterations of the
    train_byol.py:56-74 loop body (zero_grad, forward, byol_loss, backward, clip_grad_norm_(1.0),
    AdamW.step, _update_target_network, CosineAnnealingLR.step) on a fresh seeded batch each step;
    per step the loss, the pre-clip gradient norm and the lr; after the last step a held-out batch's
    online / target embeddings and eval-mode online_pred / target_proj / loss, and a sample of the
    final online weights. The tests replay the batches from the seeds (make_inputs)."""
    from src.models.byol import byol_loss
    with tempfile.TemporaryDirectory() as td:
        model, layout, flat0 = build_reference_model(arch, proj_dim, pred_dim, ema, td)
        opt = torch.optim.AdamW(model.parameters(), lr=lr, weight_decay=wd)
        sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=steps)
        res = {"B": B, "L": L, "steps": steps, "proj_dim": proj_dim, "pred_dim": pred_dim, "ema": ema, "lr": lr,
               "wd": wd, "seed": SEED}
        losses, norms, lrs = [], [], []
        model.train()
        for i in range(steps):
            clean, noisy = make_inputs(B, L, seed=SEED + 100 + i)
            lrs.append(opt.param_groups[0]["lr"])
            opt.zero_grad()
            pred, tproj = model(clean, noisy)
            loss = byol_loss(pred, tproj)
            loss.backward()
            gn = torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1.0)
            opt.step()
            model._update_target_network()
            sched.step()
            losses.append(float(loss))
            norms.append(float(gn))
            print(f"  {tag} step {i}: loss {losses[-1]:.6f} grad norm {norms[-1]:.5f} lr {lrs[-1]:.3e}", flush=True)
        held_c, held_n = make_inputs(B, L, seed=SEED + 99)
        model.eval()
        with torch.no_grad():
            emb = model.get_encoder()(held_c)
            temb = model.target_encoder(held_n)
            pred, tproj = model(held_c, held_n)
            hl = byol_loss(pred, tproj)
        on = flat_from_model(model, layout)
        idx = sample_idx(layout.numel, seed=2)
        res.update(losses=np.array(losses), grad_norms=np.array(norms), lrs=np.array(lrs),
                   held_emb=emb.numpy(), held_temb=temb.numpy(), held_pred=pred.numpy(), held_tproj=tproj.numpy(),
                   held_loss=float(hl), w_idx=idx, w_delta_sample=(on - flat0)[idx].numpy(),
                   w_delta_norm=float((on - flat0).norm()))
        np.savez_compressed(os.path.join(HERE, f"traj_{tag}.npz"), **res)
        print(f"traj_{tag}: losses {np.round(losses, 6).tolist()} held loss {float(hl):.6f}")


def make_snr():
    from src.data.augment import add_noise_to_speech
    from transformers import Wav2Vec2FeatureExtractor
    fe = Wav2Vec2FeatureExtractor(do_normalize=True)
    rng = np.random.default_rng(7)
    L = 4000
    cases = []
    for i, (ln, snr) in enumerate([(L, 0), (L, 2), (L // 3, 4), (3 * L, 5), (L - 1, 8), (1000, 10), (L, 15),
                                   (L + 17, 20), (L, 5), (L, 5), (L, 5), (777, -5)]):
        s = (rng.standard_normal(L) * 0.1).astype(np.float32)
        n = rng.standard_normal(ln).astype(np.float32)
        if i == 8:
            s[:] = 0          # zero speech -> None
        if i == 9:
            n[:] = 0          # zero noise -> None
        if i == 10:
            s[100] = np.nan   # NaN input -> None
        cases.append((s, n, snr))
    out = {}
    for i, (s, n, snr) in enumerate(cases):
        y = add_noise_to_speech(torch.from_numpy(s)[None], torch.from_numpy(n)[None], snr)
        out[f"c{i}_speech"] = s
        out[f"c{i}_noise"] = n
        out[f"c{i}_snr"] = np.float32(snr)
        if y is None:
            out[f"c{i}_ok"] = np.int32(0)
            continue
        clean_s = torch.from_numpy(s)[None]
        cm = torch.max(torch.abs(clean_s))
        nm = torch.max(torch.abs(y))
        cs = clean_s / (cm + 1e-8)
        ns = y / (nm + 1e-8)
        out[f"c{i}_ok"] = np.int32(1)
        out[f"c{i}_noisy_raw"] = y.squeeze(0).numpy()
        out[f"c{i}_clean_peak"] = cs.squeeze(0).numpy()
        out[f"c{i}_noisy_peak"] = ns.squeeze(0).numpy()
        out[f"c{i}_clean_iv"] = fe(cs.squeeze().numpy(), sampling_rate=16000, return_tensors="np").input_values[0]
        out[f"c{i}_noisy_iv"] = fe(ns.squeeze().numpy(), sampling_rate=16000, return_tensors="np").input_values[0]
    out["n_cases"] = np.int32(len(cases))
    np.savez_compressed(os.path.join(HERE, "snr_mix.npz"), **out)
    print("snr_mix:", len(cases), "cases")


def make_buckets():
    from transformers.models.wavlm.modeling_wavlm import WavLMAttention
    att = WavLMAttention(64, 1, num_buckets=320, max_distance=800)
    out = {}
    for T in (49, 249, 399, 599, 1200):
        d = torch.arange(-(T - 1), T, dtype=torch.long)
        out[f"T{T}"] = att._relative_positions_bucket(d).numpy().astype(np.int32)
    np.savez_compressed(os.path.join(HERE, "buckets.npz"), **out)
    print("buckets: ok")


def make_configs():
    """The reference's YAML configs as data fixtures (yaml.safe_load -> safe_dump), so the
    configs[0] plumbing test runs the dev config on the GPU box, where /root/reference is absent."""
    import yaml
    out = os.path.join(HERE, "configs")
    os.makedirs(out, exist_ok=True)
    for name in ("dev_wavlm-large_byol.yaml", "default_wavlm-large_byol.yaml"):
        with open(os.path.join(REF, "config", name)) as f:
            cfg = yaml.safe_load(f)
        with open(os.path.join(out, name), "w") as f:
            yaml.safe_dump(cfg, f, sort_keys=False)
    print("configs: ok")


def make_state_manifest():
    """state_manifest.json: the reference BYOLSpeechModel.state_dict() key / shape / dtype list, in
    its order, for the tiny arch and WavLM-Large (the checkpoint format train_byol.py:207-240
    saves as 'model_state_dict' and src/train/dimentional_emotions.py:43-45 and
    baseline/train_ft_cat_ser_weighted_checkpoint.py:137-158 load)."""
    import json
    out = {}
    for tag, arch, pp in (("tiny", A.TINY, (256, 512)), ("large", A.LARGE, (1024, 2048))):
        with tempfile.TemporaryDirectory() as td:
            model, _, _ = build_reference_model(arch.deterministic(), pp[0], pp[1], 0.99, td)
            out[tag] = [[k, list(v.shape), str(v.dtype).replace("torch.", "")] for k, v in model.state_dict().items()]
        print(f"state manifest {tag}: {len(out[tag])} entries")
    with open(os.path.join(HERE, "state_manifest.json"), "w") as fh:
        json.dump(out, fh, indent=0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-large", action="store_true")
    ap.add_argument("--configs-only", action="store_true")
    ap.add_argument("--manifest-only", action="store_true")
    ap.add_argument("--varlen", action="store_true",
                    help="only the WavLM-Large 3 s / 12 s fixtures (configs[4]'s length range)")
    ap.add_argument("--trajectory", action="store_true",
                    help="only the WavLM-Large det-train trajectory (B = 4 x 3 s, 6 steps)")
    args = ap.parse_args()
    if args.trajectory:
        torch.set_num_threads(8)
        run_trajectory(A.LARGE.deterministic(), 4, 48000, 6, 1024, 2048, 0.997, 1e-5, 1e-5, "large_3s")
        return
    if args.varlen:
        torch.set_num_threads(8)
        for secs in (3, 12):
            run_byol(A.LARGE.deterministic(), 4, 16000 * secs, 1024, 2048, 0.997, 1e-5, 1e-5, f"large_{secs}s",
                     False, False)
        return
    if args.manifest_only:
        make_state_manifest()
        return
    make_configs()
    if args.configs_only:
        return
    torch.set_num_threads(8)
    make_buckets()
    make_snr()
    # batch >= 4: BatchNorm1d backward at batch 2 is dominated by fp32 cancellation
    # (dx ~ eps/(var+eps)), which makes B=2 gradients rounding noise even in the reference.
    run_byol(A.TINY.deterministic(), 8, 16000, 256, 512, 0.996, 1e-5, 1e-5, "tiny", True, True)
    if not args.skip_large:
        run_byol(A.LARGE.deterministic(), 4, 128000, 1024, 2048, 0.997, 1e-5, 1e-5, "large", False, False)


if __name__ == "__main__":
    main()
