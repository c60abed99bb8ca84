"""Bitwise repeatability of the training step (VERDICT r02 "Next round" #6): every gradient
reduction adds per-workgroup partial rows in a fixed order (nrse_rows_reduce, the slab split-Ks,
the ordered f64 sum of squares) instead of f32 atomics, so two engines built from the same weights
and fed the same batch and step seeds produce identical losses, gradients, moments and parameters.

Covered: the tiny architecture with every dropout, SpecAugment and LayerDrop site live (the
element / pair-hash masks, the fused LN-backward dropout column sums, the gate and rel-pos
gradients), and WavLM-Large at B=8 x 8 s in bf16, where the step's GEMMs run on the 256x256 kernel
(its COLSUM epilogue, the slab weight gradients) and the attention kernels at T=399."""
import pytest
import torch

from nrse_amd import arch as A, kernels as K, params as PR

pytestmark = pytest.mark.gpu

PROJ, PRED = 256, 512


def _pair(arch, proj, pred, dtype, seed=77):
    from nrse_amd.engine import ByolEngine
    layout = PR.byol_layout(arch, proj, pred)
    flat = PR.init_byol_flat(layout, seed)
    return [ByolEngine(arch, proj, pred, compute_dtype=dtype, init_flat=flat) for _ in range(2)]


def _batch(B, L, seed=5):
    g = torch.Generator().manual_seed(seed)
    clean = torch.randn(B, L, generator=g) * 0.1
    noisy = clean + 0.3 * torch.randn(B, L, generator=g)
    return clean.cuda(), noisy.cuda()


def _steps_equal(engines, clean, noisy, steps):
    for i in range(steps):
        losses = [e.train_step(clean, noisy, lr=1e-4, step_seed=100 + i) for e in engines]
        torch.cuda.synchronize()
        assert torch.equal(losses[0], losses[1]), (i, float(losses[0]), float(losses[1]))
        a, b = engines[0].grad, engines[1].grad
        diff = int((a != b).sum())
        assert diff == 0, f"step {i}: {diff} of {a.numel()} gradient entries differ"
    for e in engines:
        e.sync_optimizer()
    torch.cuda.synchronize()
    for name in ("online", "target", "m", "v"):
        assert torch.equal(getattr(engines[0], name), getattr(engines[1], name)), name


def test_deterministic_reductions_are_the_default():
    assert K.DETERMINISTIC


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_tiny_stochastic_steps_are_bitwise_repeatable(nrse_device, dtype):
    engines = _pair(A.TINY, PROJ, PRED, dtype)
    clean, noisy = _batch(4, 16000)
    _steps_equal(engines, clean, noisy, steps=3)


def test_large_bf16_steps_are_bitwise_repeatable(nrse_device):
    engines = _pair(A.LARGE, 1024, 2048, torch.bfloat16)
    clean, noisy = _batch(8, 128000)
    _steps_equal(engines, clean, noisy, steps=2)
