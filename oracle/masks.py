"""ORACLE (test infrastructure only — imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product path).

numpy restatement of the counter-hash dropout masks the HIP kernels draw
(noise-robust-speech-embedding_amd/csrc/common.h: mix32 / site_key / dropout_keep), so the CPU
oracle can replay a stochastic training step with the identical masks. The reference draws its
masks from torch's Philox stream (torch.nn.Dropout, [TF]modeling_wavlm.py:99/287-294/482) which
no other implementation can bit-match; what is pinned against the reference is the semantics
(keep probability 1-p, scale 1/(1-p), mask per element) — see tests/test_stochastic_gpu.py.
"""
from __future__ import annotations

import numpy as np

M32 = np.uint64(0xFFFFFFFF)


def mix32(x):
    x = np.asarray(x, dtype=np.uint64) & M32
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & M32
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & M32
    x ^= x >> np.uint64(16)
    return x


def site_key(seed: int) -> np.uint64:
    return mix32((np.uint64(seed) * np.uint64(0x9E3779B9) + np.uint64(0x632BE5AB)) & M32)


def threshold(p: float) -> int:
    """16-bit keep threshold round(p * 65536) (csrc/common.h dropout_threshold)."""
    t = p * 65536.0 + 0.5
    return 65536 if t >= 65536.0 else int(t)


def keep_mask(seed: int, p: float, n: int, start: int = 0) -> np.ndarray:
    """keep[i] for flat element indices start..start+n-1 of one dropout site: one mix32 hash per
    pair of elements (i >> 1), 16 bits per element (odd i: high half)."""
    idx = np.arange(start, start + n, dtype=np.uint64)
    h = mix32((idx >> np.uint64(1)) ^ site_key(seed))
    half = np.where((idx & np.uint64(1)) == 1, h >> np.uint64(16), h & np.uint64(0xFFFF))
    return half >= np.uint64(threshold(p))


def dropout_mask(seed: int, p: float, shape) -> np.ndarray:
    """Multiplicative mask (0 or 1/(1-p)) over a row-major tensor of `shape`."""
    n = int(np.prod(shape))
    k = keep_mask(seed, p, n).reshape(shape)
    return k.astype(np.float32) * np.float32(1.0 / (1.0 - p)) if p < 1 else np.zeros(shape, np.float32)


def threshold16(p: float) -> int:
    t = p * 65536.0 + 0.5
    return 65536 if t >= 65536.0 else int(t)


def attn_mix(x):
    """csrc/common.h attn_mix (ABI 10): the attention pair hash of full-rate VALU ops, two 24-bit
    multiplies (v_mul_u32_u24) between xor-shifts."""
    x = np.asarray(x, dtype=np.uint64) & M32
    x ^= x >> np.uint64(16)
    x = ((x & np.uint64(0xFFFFFF)) * np.uint64(0xEBCA6B)) & M32
    x ^= x >> np.uint64(13)
    x = ((x & np.uint64(0xFFFFFF)) * np.uint64(0xB2AE35)) & M32
    x ^= x >> np.uint64(16)
    return x


def attn_keep_mask(seed: int, p: float, rows: int, T: int) -> np.ndarray:
    """keep[row, k] of the attention-probability site (csrc/common.h attn_keep): one attn_mix hash
    per pair of keys of a query row, 16 bits per element; row = (b*H + h)*T + q."""
    r = np.arange(rows, dtype=np.uint64)[:, None]
    kk = np.arange(T, dtype=np.uint64)[None, :]
    tp2 = np.uint64((T + 1) // 2)
    h = attn_mix(((r * tp2 + (kk >> np.uint64(1))) & M32) ^ site_key(seed))
    half = np.where((kk & np.uint64(1)) == 1, h >> np.uint64(16), h & np.uint64(0xFFFF))
    return half >= np.uint64(threshold16(p))


def attn_dropout_mask(seed: int, p: float, shape) -> np.ndarray:
    """Multiplicative mask (0 or 1/(1-p)) over attention probabilities of shape [..., T, T]."""
    T = int(shape[-1])
    rows = int(np.prod(shape[:-1]))
    k = attn_keep_mask(seed, p, rows, T).reshape(shape)
    return k.astype(np.float32) * np.float32(1.0 / (1.0 - p)) if p < 1 else np.zeros(shape, np.float32)


def specaug_mask(seed: int, batch: int, T: int, mask_prob: float, mask_length: int, min_masks: int) -> np.ndarray:
    """[batch, T] bool SpecAugment time masks as nrse_specaug_mask draws them (csrc/misc.hip
    specaug_mask_kernel): the reference's span count and span semantics ([TF]modeling_wavlm.py:
    834-954, _compute_mask_indices over full-length utterances) with a counter-hash stream -- eps =
    24 bits of the seed's key; per utterance the starts are the n candidates (of C = T - L + 1) with
    the smallest keys (mix32((b C + k) ^ key2) << 32 | k), a uniformly random n-subset."""
    mask = np.zeros((batch, T), dtype=bool)
    if mask_prob <= 0 or mask_length < 1:
        return mask
    if mask_length > T:
        raise ValueError(f"mask_length {mask_length} > sequence_length {T}")
    key = site_key(seed)
    eps = float(mix32(key ^ np.uint64(0x2545F491)) >> np.uint64(8)) / 16777216.0
    n = int(mask_prob * T / mask_length + eps)
    n = max(n, min_masks)
    if n * mask_length > T:
        n = T // mask_length
    if T - (mask_length - 1) < n:
        n = max(T - (mask_length - 1), 0)
    if n == 0:
        return mask
    C = T - mask_length + 1
    key2 = mix32(key ^ np.uint64(0x5BD1E995))
    k = np.arange(C, dtype=np.uint64)
    for b in range(batch):
        h = mix32(((np.uint64(b) * np.uint64(C) + k) & M32) ^ key2)
        starts = np.argsort((h << np.uint64(32)) | k, kind="stable")[:n]
        idx = (starts[:, None] + np.arange(mask_length)[None, :]).reshape(-1)
        mask[b, idx] = True
    return mask
