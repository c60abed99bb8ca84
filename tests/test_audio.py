"""Host-side audio feed (CPU): discovery of .wav/.flac/.mp3 (src/utils/audio_utils.py:67-73),
resampling to the configured rate (:33-36), the load-error path for files this build cannot
decode (:62-64), and per-rank item draws under DDP.

Resampler parity is UNPINNED (torchaudio is not importable here and the reference holds no
resampled fixture): the checks below are properties of torchaudio's published sinc_interp_hann
filter that any faithful restatement has -- output length ceil(new*n/orig), unit DC gain, a tone
below the cut-off kept at its frequency and amplitude, the identity at equal rates."""
import math
import os
import wave

import numpy as np
import pytest
import torch

from nrse_amd import audio as AU, data as D


def _write_wav(path, x, sr, ch=1):
    x = np.clip(np.asarray(x, np.float64), -1, 1 - 1 / 32768)
    pcm = (x * 32768).astype("<i2")
    if ch > 1:
        pcm = np.repeat(pcm[:, None], ch, axis=1).reshape(-1)
    with wave.open(str(path), "wb") as w:
        w.setnchannels(ch)
        w.setsampwidth(2)
        w.setframerate(sr)
        w.writeframes(pcm.tobytes())


def test_resample_length_dc_and_identity():
    x = np.ones(48000, np.float32)
    for orig, new in ((8000, 16000), (44100, 16000), (22050, 16000), (48000, 16000), (16000, 8000)):
        y = AU.resample(x[: orig // 2], orig, new)
        assert y.shape[0] == math.ceil(new * (orig // 2) / orig), (orig, new, y.shape)
        mid = y[len(y) // 4: 3 * len(y) // 4]           # away from the zero-padded edges
        assert np.allclose(mid, 1.0, atol=2e-3), (orig, new, mid.min(), mid.max())
    z = np.random.default_rng(0).standard_normal(1000).astype(np.float32)
    assert np.array_equal(AU.resample(z, 16000, 16000), z)


def test_resample_keeps_a_tone():
    for orig in (8000, 22050, 44100, 48000):
        t = np.arange(orig) / orig
        x = np.sin(2 * np.pi * 440.0 * t).astype(np.float32)
        y = AU.resample(x, orig, 16000)
        tt = np.arange(y.shape[0]) / 16000
        ref = np.sin(2 * np.pi * 440.0 * tt)
        sl = slice(2000, 14000)
        err = np.abs(y[sl] - ref[sl]).max()
        assert err < 5e-3, (orig, err)


def test_discovery_resampling_and_undecodable_files(tmp_path):
    clean = tmp_path / "clean"
    noise = tmp_path / "noise"
    for d in (clean, noise):
        d.mkdir()
    rng = np.random.default_rng(1)
    _write_wav(clean / "a.wav", 0.1 * rng.standard_normal(8000), 8000)            # 1 s at 8 kHz
    _write_wav(clean / "b.WAV", 0.1 * rng.standard_normal(16000), 16000, ch=2)     # stereo
    (clean / "c.flac").write_bytes(b"fLaC\x00not-really")
    (clean / "d.mp3").write_bytes(b"ID3\x03junk")
    (clean / "e.txt").write_text("not audio")
    _write_wav(noise / "n.wav", rng.standard_normal(44100), 44100)
    files = AU.get_audio_files(str(clean))
    assert [os.path.basename(f) for f in files] == ["a.wav", "b.WAV", "c.flac", "d.mp3"]
    ds = D.WavPairs(files, AU.get_audio_files(str(noise)), 16000, 1.0, [5])
    a = ds._load(files[0])
    assert a.shape == (16000,) and np.abs(a).max() > 0.05     # 8 kHz -> 16 kHz, not zero padding
    assert ds._load(files[2]) is None and ds._load(files[3]) is None   # load-error path -> None
    n = ds._load(AU.get_audio_files(str(noise))[0])
    assert n.shape == (16000,)
    it = ds[2]                                   # c.flac fails -> the next file (d.mp3) fails -> a.wav
    assert int(it["index"]) == 0 and int(it["attempts"]) == 3
    vl = D.WavVarLenPairs(files, AU.get_audio_files(str(noise)), 16000, 12.0, [4, 8])
    assert vl.lengths == [16000, 16000]           # undecodable clean files left out, 8 kHz counted at 16 kHz
    assert vl[0]["clean"].shape[0] == 16000


def _draws(tmp_path, rank, world, workers):
    clean = tmp_path / "c"
    noise = tmp_path / "n"
    if not clean.exists():
        clean.mkdir()
        noise.mkdir()
        rng = np.random.default_rng(2)
        for i in range(48):
            _write_wav(clean / f"{i:03d}.wav", 0.1 * rng.standard_normal(1600), 16000)
        for i in range(16):
            _write_wav(noise / f"{i:03d}.wav", rng.standard_normal(1600 + 37 * i), 16000)
    cfg = {"data": {"clean_data_path": str(clean), "noise_data_path": str(noise), "sample_rate": 16000,
                    "max_audio_length": 0.1, "snr_range": [0, 2, 5, 10, 15, 20, 25, 30], "validation_ratio": 0.0},
           "training": {"batch_size": 4, "num_workers": workers, "seed": 42}}
    torch.manual_seed(42)                        # what every rank's train.main does
    D.seed_host_rng(42, rank)
    train, _, _ = D.create_raw_dataloaders(cfg, rank=rank, world=world)
    snr, nlen = [], []
    for b in train:
        snr += b["snr"].tolist()
        nlen += b["noise"][:, 0].tolist()   # identifies the noise file (and its crop)
    return snr, nlen


def test_item_draws_differ_across_ranks_and_repeat_per_rank(tmp_path):
    """with one torch seed on every rank, a rank-independent DataLoader generator
    gave item k of every rank the same noise file and SNR. Per-rank generators (workers) and a
    per-rank host `random` (num_workers = 0) make the draws differ across ranks and repeat per
    rank."""
    for workers in (0, 2):
        r0 = _draws(tmp_path, 0, 2, workers)
        r0b = _draws(tmp_path, 0, 2, workers)
        r1 = _draws(tmp_path, 1, 2, workers)
        assert r0 == r0b, workers                # reproducible
        assert r0[0] != r1[0] and r0[1] != r1[1], workers


def test_mostly_undecodable_corpus_is_refused(tmp_path):
    """a corpus the build cannot decode (FLAC / MP3 without torchaudio) fails
    loudly when the dataset is built instead of training on load errors and retries."""
    clean = tmp_path / "clean"
    noise = tmp_path / "noise"
    for d in (clean, noise):
        d.mkdir()
    rng = np.random.default_rng(3)
    _write_wav(clean / "a.wav", 0.1 * rng.standard_normal(16000), 16000)
    for i in range(3):
        (clean / f"f{i}.flac").write_bytes(b"fLaC\x00not-really")
    _write_wav(noise / "n.wav", rng.standard_normal(16000), 16000)
    files = AU.get_audio_files(str(clean))
    assert AU.undecodable_share(files) == 0.75
    with pytest.raises(AU.AudioDecodeError, match="cannot be decoded"):
        D.WavPairs(files, AU.get_audio_files(str(noise)), 16000, 1.0, [5])
    with pytest.raises(AU.AudioDecodeError, match="cannot be decoded"):
        D.WavVarLenPairs(files, AU.get_audio_files(str(noise)), 16000, 12.0, [5])
    # a broken WAV header counts as undecodable too
    (noise / "m.wav").write_bytes(b"RIFF0000WAVEjunk")
    (noise / "k.wav").write_bytes(b"RIFF0000WAVEjunk")
    with pytest.raises(AU.AudioDecodeError):
        D.WavPairs([str(clean / "a.wav")], AU.get_audio_files(str(noise)), 16000, 1.0, [5])


def test_varlen_substitute_keeps_bucket_length(tmp_path, monkeypatch):
    """an invalid clean file is replaced by the next one, cropped / padded to the
    length the sampler bucketed the item by, and the item keeps the sampled index."""
    clean = tmp_path / "clean"
    noise = tmp_path / "noise"
    for d in (clean, noise):
        d.mkdir()
    rng = np.random.default_rng(4)
    _write_wav(clean / "a.wav", 0.1 * rng.standard_normal(16000), 16000)       # 1 s
    _write_wav(clean / "b.wav", 0.1 * rng.standard_normal(48000), 16000)       # 3 s
    _write_wav(noise / "n.wav", rng.standard_normal(16000), 16000)
    vl = D.WavVarLenPairs(AU.get_audio_files(str(clean)), AU.get_audio_files(str(noise)), 16000, 12.0, [5])
    assert vl.lengths == [16000, 48000]
    real = vl._load
    monkeypatch.setattr(vl, "_load", lambda p, crop: None if p.endswith("a.wav") else real(p, crop))
    it = vl[0]                       # a.wav invalid -> b.wav (3 s) stands in, cut to a.wav's 1 s
    assert it["clean"].shape[0] == 16000
    assert int(it["index"]) == 0 and int(it["attempts"]) == 2


def _corpus(tmp_path, n_clean, n_noise=3):
    clean = tmp_path / "clean10"
    noise = tmp_path / "noise10"
    clean.mkdir()
    noise.mkdir()
    rng = np.random.default_rng(5)
    for i in range(n_clean):
        _write_wav(clean / f"{i:02d}.wav", 0.1 * rng.standard_normal(1600), 16000)
    for i in range(n_noise):
        _write_wav(noise / f"{i:02d}.wav", rng.standard_normal(1600), 16000)
    return clean, noise


def _cfg(clean, noise, bs, ratio):
    return {"data": {"clean_data_path": str(clean), "noise_data_path": str(noise), "sample_rate": 16000,
                     "max_audio_length": 0.1, "snr_range": [5, 10], "validation_ratio": ratio},
            "training": {"batch_size": bs, "num_workers": 0, "seed": 42}}


def test_missing_or_empty_data_directory_raises(tmp_path):
    """a configured data directory that does not exist, or holds no audio file,
    fails loudly (the build used to fall back to synthetic pairs silently); synthetic pairs only
    when asked for (`data.synthetic` / synthetic_items)."""
    clean, noise = _corpus(tmp_path, 4)
    cfg = _cfg(clean, tmp_path / "no_such_dir", 2, 0.0)
    with pytest.raises(FileNotFoundError, match="noise_data_path"):
        D.create_raw_dataloaders(cfg)
    empty = tmp_path / "empty"
    empty.mkdir()
    with pytest.raises(FileNotFoundError, match="holds no"):
        D.create_raw_dataloaders(_cfg(empty, noise, 2, 0.0))
    cfg["data"]["synthetic"] = 8                    # explicit opt-in
    train, _, ds = D.create_raw_dataloaders(cfg)
    assert isinstance(ds, D.SyntheticPairs) and len(ds) == 8


def test_loader_lengths_match_reference_ragged_split(tmp_path):
    """The reference's DataLoaders have no drop_last (noisy_speech_dataset.py:178-192): 10 items,
    validation_ratio 0.3, batch 4 -> val_size = int(10 * 0.3) = 3, train 7 -> ceil(7/4) = 2 train
    batches (4 + 3) and 1 validation batch of 3 -- the CosineAnnealingLR T_max = len(loader) *
    epochs (train_byol.py:149-150) follows. The one deviation: a final training batch of exactly
    one pair is dropped (BatchNorm1d in train mode cannot normalise one row; the reference raises)."""
    clean, noise = _corpus(tmp_path, 10)
    train, val, _ = D.create_raw_dataloaders(_cfg(clean, noise, 4, 0.3))
    assert len(train) == math.ceil(7 / 4) == 2 and len(val) == 1
    assert sorted(len(b["snr"]) for b in train) == [3, 4]
    assert [len(b["snr"]) for b in val] == [3]
    # 10 items, ratio 0.1: train 9 = 4 + 4 + 1 -> the single-pair tail is dropped, val keeps its 1
    train, val, _ = D.create_raw_dataloaders(_cfg(clean, noise, 4, 0.1))
    assert len(train) == 2 and [len(b["snr"]) for b in train] == [4, 4]
    assert len(val) == 1 and [len(b["snr"]) for b in val] == [1]
