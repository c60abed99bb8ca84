"""ORACLE (test infrastructure only — imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product path).

numpy restatement of the per-pair noise augmentation + normalisation the reference runs in its
DataLoader workers:
  add_noise_to_speech            src/data/augment.py:4-66
  peak normalisation             src/data/noisy_speech_dataset.py:88-103
  feature-extractor normalise    [TF]models/wav2vec2/feature_extraction_wav2vec2.py:78-97
                                 (zero_mean_unit_var_norm, applied when do_normalize)
Status codes (the reference returns None / `continue`s; here one int32 per pair):
  0 ok, 1 NaN in speech, 2 NaN in noise, 3 speech power < 1e-10, 4 noise power < 1e-10,
  5 noise scaling inf/nan, 6 noise scaling > 1e6, 7 NaN after mixing,
  8 clean peak < 1e-8, 9 noisy peak < 1e-8
"""
from __future__ import annotations

import numpy as np

OK, NAN_SPEECH, NAN_NOISE, LOW_SPEECH, LOW_NOISE, BAD_SCALE, HUGE_SCALE, NAN_MIX, LOW_CLEAN_PEAK, LOW_NOISY_PEAK = \
    range(10)


def tile_noise(noise: np.ndarray, L: int) -> np.ndarray:
    """augment.py:10-15: truncate, or repeat then truncate."""
    if noise.shape[0] > L:
        return noise[:L]
    if noise.shape[0] < L:
        reps = L // noise.shape[0] + 1
        return np.tile(noise, reps)[:L]
    return noise


def add_noise(speech: np.ndarray, noise: np.ndarray, snr_db: float):
    """augment.py:4-66 -> (noisy or None, status, k)."""
    if np.isnan(speech).any():
        return None, NAN_SPEECH, 0.0
    if np.isnan(noise).any():
        return None, NAN_NOISE, 0.0
    n = tile_noise(noise, speech.shape[0])
    ps = np.mean(speech.astype(np.float32) ** 2, dtype=np.float32)
    pn = np.mean(n.astype(np.float32) ** 2, dtype=np.float32)
    if ps < 1e-10:
        return None, LOW_SPEECH, 0.0
    if pn < 1e-10:
        return None, LOW_NOISE, 0.0
    snr_lin = 10 ** (snr_db / 10)
    k = np.float32(np.sqrt(np.float32(ps / np.float32(pn * np.float32(snr_lin)))))
    if not np.isfinite(k):
        return None, BAD_SCALE, float(k)
    if k > 1e6:
        return None, HUGE_SCALE, float(k)
    y = (speech + n * k).astype(np.float32)
    if np.isnan(y).any():
        return None, NAN_MIX, float(k)
    return y, OK, float(k)


def zero_mean_unit_var(x: np.ndarray) -> np.ndarray:
    return ((x - x.mean()) / np.sqrt(x.var() + 1e-7)).astype(np.float32)


def mix_pair(clean: np.ndarray, noise: np.ndarray, snr_db: float, do_normalize: bool = True):
    """noisy_speech_dataset.py:77-129 for one pair -> (clean_iv, noisy_iv, status, k)."""
    y, st, k = add_noise(clean, noise, snr_db)
    if st != OK:
        return None, None, st, k
    cm = np.max(np.abs(clean))
    nm = np.max(np.abs(y))
    if cm < 1e-8:
        return None, None, LOW_CLEAN_PEAK, k
    if nm < 1e-8:
        return None, None, LOW_NOISY_PEAK, k
    c = (clean / (cm + np.float32(1e-8))).astype(np.float32)
    n = (y / (nm + np.float32(1e-8))).astype(np.float32)
    if do_normalize:
        c = zero_mean_unit_var(c)
        n = zero_mean_unit_var(n)
    return c, n, OK, k
