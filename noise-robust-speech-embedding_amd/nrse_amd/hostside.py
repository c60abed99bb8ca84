"""Host-side setup of the step: relative-position buckets and SpecAugment span sampling.

Both are tiny integer computations done once per sequence length / per step on the host,
exactly as the reference does them on the host:
  * bucket(j - i)   [TF]modeling_wavlm.py:253-271 (float32 log, like torch's `.float()` path);
    uploaded once per T as an int32 vector of length 2T-1 and cached on the device.
  * span masks      [TF]modeling_wavlm.py:834-954 (_compute_mask_indices, numpy RNG), the
    [B, T] bool mask is copied to the device each step (non-blocking).
"""
from __future__ import annotations

import math

import numpy as np


def bucket_vector(T: int, num_buckets: int = 320, max_distance: int = 800) -> np.ndarray:
    """int32 [2T-1]: bucket of relative position d = j - i at index d + T - 1."""
    d = np.arange(-(T - 1), T, dtype=np.int64)
    nb = num_buckets // 2
    out = (d > 0).astype(np.int64) * nb
    rp = np.abs(d)
    max_exact = nb // 2
    small = rp < max_exact
    with np.errstate(divide="ignore"):
        lg = np.log(rp.astype(np.float32) / np.float32(max_exact)).astype(np.float32)
    lg = (lg / np.float32(math.log(max_distance / max_exact))).astype(np.float32)
    lg = (lg * np.float32(nb - max_exact)).astype(np.float32)
    large = np.float32(max_exact) + lg
    large = np.where(np.isfinite(large), large, 0).astype(np.int64)
    large = np.minimum(large, nb - 1)
    return (out + np.where(small, rp, large)).astype(np.int32)


def bucket_runs(bucket: np.ndarray, nb: int) -> tuple[np.ndarray, np.ndarray]:
    """(order, offsets) of the relative-position buckets: the offsets d sorted by bucket (stable,
    so increasing d within a bucket) and each bucket's start in that list ([nb + 1]); the gather
    form nrse_rel_bias_bwd sums a bucket's diagonals in this fixed order."""
    b = np.asarray(bucket, dtype=np.int64)
    order = np.argsort(b, kind="stable").astype(np.int32)
    offsets = np.searchsorted(b[order], np.arange(nb + 1)).astype(np.int32)
    return order, offsets


def compute_mask_indices(rng: np.random.Generator, batch: int, T: int, mask_prob: float, mask_length: int,
                         min_masks: int = 0) -> np.ndarray:
    """SpecAugment time masks with the reference's span algorithm (no attention mask: every
    utterance has the full length, src/models/encoder.py:23-25 ignores padding masks)."""
    mask = np.zeros((batch, T), dtype=bool)
    if mask_prob <= 0 or mask_length < 1:
        return mask
    if mask_length > T:
        raise ValueError(f"mask_length {mask_length} > sequence_length {T}")
    eps = rng.random()

    def num_spans(length):
        n = int(mask_prob * length / mask_length + eps)
        n = max(n, min_masks)
        if n * mask_length > T:
            n = T // mask_length
        if length - (mask_length - 1) < n:
            n = max(length - (mask_length - 1), 0)
        return n

    n = num_spans(T)
    if n == 0:
        return mask
    for b in range(batch):
        starts = rng.choice(np.arange(T - (mask_length - 1)), n, replace=False)
        idx = (starts[:, None] + np.arange(mask_length)[None, :]).reshape(-1)
        idx = np.minimum(idx, T - 1)
        mask[b, idx] = True
    return mask


def layerdrop_decisions(rng: np.random.Generator, layers: int, p: float) -> list:
    """LayerDrop ([TF]modeling_wavlm.py:493-495): layer i > 0 skipped when U(0,1) < p; decided
    once per forward for the whole batch (rank-shared seed under data parallelism)."""
    if p <= 0:
        return [False] * layers
    u = rng.random(layers)
    return [bool(i > 0 and u[i] < p) for i in range(layers)]
