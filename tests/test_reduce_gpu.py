"""The ordered partial-row reduction (nrse_rows_reduce) and its ABI 9 deferred, batched form
(nrse_reduce_defer / nrse_reduce_flush): every queued reduction's result is bitwise the immediate
launch's, across the three kernel forms (16 / 64 row groups, one column per thread), batched row
groups, more jobs than one batched launch holds, accumulate and overwrite; and the training step's
gradients are bitwise the same with the backward's per-layer reductions deferred to the side stream
or launched in place (engine.py encoder_backward, NRSE_DEFER_REDUCE)."""
import pytest
import torch

from nrse_amd import kernels as K

pytestmark = pytest.mark.gpu


def _jobs(g):
    """(slab, S, batch, destination shapes, accumulate) covering the forms and the layouts."""
    out = []
    for S, n, batch, parts, acc in [
        (512, 3072, 1, (1024, 1024, 1024), True),   # RG 64 (few column blocks, many rows)
        (100, 4096, 1, (4096,), True),              # RG 16
        (224, 797, 16, (797,), True),               # one column per thread (odd n), batched
        (37, 1024, 4, (512, 512), False),           # RG 16, overwrite, batched
        (3, 9, 1, (4, 3, 2), True),                 # scalar form, three destinations
    ]:
        slab = torch.randn(batch * S * n, generator=g).cuda()
        dst = [torch.randn(batch * m, generator=g).cuda() for m in parts]
        out.append((slab, S, batch, dst, acc))
    return out


def _run(jobs, defer):
    res = [[d.clone() for d in dst] for _, _, _, dst, _ in jobs]
    if defer:
        K.reduce_defer(True)
    for (slab, S, batch, _, acc), d in zip(jobs, res):
        K.rows_reduce(slab, S, *d, batch=batch, accumulate=acc)
    if defer:
        K.reduce_defer(False)
        assert K._lib.lib().nrse_reduce_pending() == len(jobs)
        K.reduce_flush()
        assert K._lib.lib().nrse_reduce_pending() == 0
    torch.cuda.synchronize()
    return res


@pytest.mark.parametrize("reps", [1, 3])   # 5 jobs (one batched launch) and 15 (two launches)
def test_deferred_reductions_bitwise_equal_immediate(nrse_device, reps):
    g = torch.Generator().manual_seed(11)
    jobs = _jobs(g) * reps
    a = _run(jobs, False)
    b = _run(jobs, True)
    for x, y in zip(a, b):
        for u, v in zip(x, y):
            assert torch.equal(u, v)
    # and against float64 (the order is fixed, the values are the sums)
    for (slab, S, batch, dst, acc), r in zip(jobs[:5], a[:5]):
        n = sum(d.numel() // batch for d in dst)
        ref = slab.double().view(batch, S, n).sum(1)
        off = 0
        for d0, d in zip(dst, r):
            m = d0.numel() // batch
            exp = ref[:, off:off + m].reshape(-1) + (d0.double() if acc else 0)
            assert torch.allclose(d.double(), exp, rtol=1e-5, atol=1e-4)
            off += m


def test_single_deferred_job_and_empty_flush(nrse_device):
    g = torch.Generator().manual_seed(3)
    slab, S, batch, dst, acc = _jobs(g)[1]
    a = [d.clone() for d in dst]
    K.rows_reduce(slab, S, *a, batch=batch, accumulate=acc)
    b = [d.clone() for d in dst]
    K.reduce_defer(True)
    K.rows_reduce(slab, S, *b, batch=batch, accumulate=acc)
    K.reduce_defer(False)
    K.reduce_flush()
    K.reduce_flush()   # nothing queued: no launch, no error
    torch.cuda.synchronize()
    assert all(torch.equal(u, v) for u, v in zip(a, b))


def test_step_gradients_equal_with_deferred_layer_reductions(nrse_device, monkeypatch):
    """One bf16 training step of the tiny engine, the backward's per-layer reductions deferred to
    the side stream (default) or launched in place: bitwise the same gradient and loss."""
    from nrse_amd import arch as A, params as PR
    from nrse_amd import engine as E
    arch = A.TINY.deterministic()
    layout = PR.byol_layout(arch, 256, 512)
    flat = PR.init_byol_flat(layout, 1234)
    g = torch.Generator().manual_seed(5)
    clean = torch.randn(4, 16000, generator=g).cuda()
    noisy = clean + 0.3 * torch.randn(4, 16000, generator=g).cuda()
    out = {}
    for d in (False, True):
        monkeypatch.setattr(E, "_DEFER_REDUCE", d)
        eng = E.ByolEngine(arch, 256, 512, compute_dtype=torch.bfloat16, init_flat=flat,
                           step_cfg=E.StepConfig(overlap_optimizer=False))
        loss = eng.train_step(clean, noisy, lr=1e-4, step_seed=0)
        torch.cuda.synchronize()
        out[d] = (float(loss), eng.online.clone())
    assert out[True][0] == out[False][0]
    assert torch.equal(out[True][1], out[False][1])
