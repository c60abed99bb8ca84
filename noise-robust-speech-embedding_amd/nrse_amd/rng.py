"""Seeding contract for the stochastic features of the training step.

The reference draws dropout / LayerDrop / SpecAugment randomness from torch's and numpy's
global generators (train_byol.py:44 puts BOTH branches in train mode; [TF]modeling_wavlm.py:
493-495 LayerDrop, 99/287-294/482 dropout, 834-954 SpecAugment; src/utils/setup_utils.py:4-7
seeds them). Here every dropout site gets a 32-bit seed derived from (forward base seed, site
id); kernels turn (seed, element index) into the keep decision with a stateless hash, so the
backward pass regenerates the forward masks and graph replays need no host RNG.
"""
from __future__ import annotations

M = 0xFFFFFFFF

SITE_FEAT_PROJ = 1
SITE_POS = 2
SITE_SPEC = 3     # the SpecAugment time-mask draw of a forward (nrse_specaug_mask)


def site_attn_probs(layer: int) -> int:
    return 16 + 4 * layer


def site_attn_out(layer: int) -> int:
    return 17 + 4 * layer


def site_act(layer: int) -> int:
    return 18 + 4 * layer


def site_ffn_out(layer: int) -> int:
    return 19 + 4 * layer


def mix32(x: int) -> int:
    x &= M
    x ^= x >> 16
    x = (x * 0x7FEB352D) & M
    x ^= x >> 15
    x = (x * 0x846CA68B) & M
    x ^= x >> 16
    return x


def site_seed(base: int, site: int) -> int:
    return mix32((base * 0x85EBCA6B) ^ mix32(site + 0x27D4EB2F))


def forward_seed(step_seed: int, branch: int, rank: int = 0) -> int:
    """Base seed of one encoder forward: branch 0 = online (clean), 1 = target (noisy).
    Rank-distinct, so data-parallel replicas draw independent dropout masks."""
    return mix32(mix32(step_seed * 2 + branch) ^ mix32(0x5BD1E995 + rank))
