"""Data-parallel engine step on the GPU: two ranks sharing cuda:0 (gloo, since RCCL refuses two
ranks on one device; NRSE_SHARE_DEVICE=1), each with its own pairs. The per-layer gradient
all-reduce overlapped with backward (nrse_amd/engine.py backward) must produce the sum of the
two ranks' local gradients, and both replicas must take the identical optimizer step."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), NRSE_SHARE_DEVICE="1", NRSE_DDP_BACKEND="gloo")
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "noise-robust-speech-embedding_amd"))
    import torch.distributed as dist
    from nrse_amd import arch as A, ddp, params as PR
    from nrse_amd.engine import ByolEngine
    r, w, local = ddp.init_from_env()
    torch.cuda.set_device(local)
    arch = A.TINY
    layout = PR.byol_layout(arch, 256, 512)
    flat = PR.init_byol_flat(layout, 1234)
    g = torch.Generator().manual_seed(50 + r)
    clean = (torch.randn(4, 16000, generator=g) * 0.1).cuda()
    noisy = clean + 0.05 * torch.randn(4, 16000, generator=g).cuda()
    loc = ByolEngine(arch, 256, 512, device="cuda:0", compute_dtype=torch.float32, init_flat=flat)
    loc.train_step(clean, noisy, lr=1e-4, step_seed=3, rank=r)
    g_local = loc.grad.cpu()
    del loc
    eng = ByolEngine(arch, 256, 512, device="cuda:0", compute_dtype=torch.float32, init_flat=flat)
    ar = ddp.GradAllReduce(bucket_bytes=1 << 20)
    eng.train_step(clean, noisy, lr=1e-4, step_seed=3, rank=r, allreduce=ar, world_size=w)
    torch.cuda.synchronize()
    out[r] = (g_local, eng.grad.cpu(), eng.online.cpu(), ar.issued_elems, layout.numel)
    dist.destroy_process_group()


def test_overlapped_allreduce_engine_two_ranks(nrse_device):
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
    (gl0, gs0, p0, n0, numel), (gl1, gs1, p1, _, _) = out[0], out[1]
    ref = gl0.double() + gl1.double()
    err = float((gs0.double() - ref).norm() / ref.norm())
    assert err < 1e-5, err
    assert torch.equal(gs0, gs1)
    assert torch.equal(p0, p1)
    assert 0 < n0 <= numel


def _syncbn_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), NRSE_SHARE_DEVICE="1", NRSE_DDP_BACKEND="gloo")
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "noise-robust-speech-embedding_amd"))
    import torch.distributed as dist
    from nrse_amd import arch as A, ddp, params as PR
    from nrse_amd.engine import ByolEngine
    r, w, local = ddp.init_from_env()
    torch.cuda.set_device(local)
    arch = A.TINY.deterministic()
    layout = PR.byol_layout(arch, 256, 512)
    flat = PR.init_byol_flat(layout, 1234)
    g = torch.Generator().manual_seed(60)
    clean = torch.randn(8, 16000, generator=g) * 0.1
    noisy = clean + 0.05 * torch.randn(8, 16000, generator=g)
    sl = slice(4 * r, 4 * r + 4)
    eng = ByolEngine(arch, 256, 512, device="cuda:0", compute_dtype=torch.float32, init_flat=flat)
    eng.sync_bn = ddp.SyncBN()
    with torch.no_grad():
        pred, tproj, _ = eng.forward(clean[sl].cuda(), noisy[sl].cuda(), train=True)
    loss = eng.train_step(clean[sl].cuda(), noisy[sl].cuda(), lr=1e-4, step_seed=0, rank=r,
                          allreduce=ddp.GradAllReduce(), world_size=w)
    lsum = loss.clone()
    dist.all_reduce(lsum)
    torch.cuda.synchronize()
    out[r] = (pred.cpu(), tproj.cpu(), float(lsum) / w, eng.grad.cpu() / w, eng.online.cpu(),
              eng.bn["online_projector.layers.1"][1].cpu())
    dist.destroy_process_group()


def test_sync_batchnorm_two_ranks_equal_one_rank_of_both(nrse_device):
    """SyncBN (nrse_amd/ddp.SyncBN): 2 ranks x B/2 rows give the rows, loss, averaged gradient,
    running statistics and parameter update of 1 rank x B (the two forwards per rank also update
    the running stats twice, as on the single rank below)."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "noise-robust-speech-embedding_amd"))
    from nrse_amd import arch as A, params as PR
    from nrse_amd.engine import ByolEngine
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_syncbn_worker, args=(2, port, out), nprocs=2, join=True)
    arch = A.TINY.deterministic()
    layout = PR.byol_layout(arch, 256, 512)
    flat = PR.init_byol_flat(layout, 1234)
    g = torch.Generator().manual_seed(60)
    clean = torch.randn(8, 16000, generator=g) * 0.1
    noisy = clean + 0.05 * torch.randn(8, 16000, generator=g)
    eng = ByolEngine(arch, 256, 512, device="cuda:0", compute_dtype=torch.float32, init_flat=flat)
    with torch.no_grad():
        pred, tproj, _ = eng.forward(clean.cuda(), noisy.cuda(), train=True)
    loss = float(eng.train_step(clean.cuda(), noisy.cuda(), lr=1e-4, step_seed=0))

    def rel(a, b):
        return float((a.double() - b.double()).norm() / b.double().norm())
    p2 = torch.cat([out[0][0], out[1][0]])
    t2 = torch.cat([out[0][1], out[1][1]])
    assert rel(p2, pred.cpu()) < 1e-4 and rel(t2, tproj.cpu()) < 1e-4
    assert abs(out[0][2] - loss) < 1e-5 and abs(out[1][2] - loss) < 1e-5
    assert rel(out[0][3], eng.grad.cpu()) < 1e-3
    assert rel(out[0][5], eng.bn["online_projector.layers.1"][1].cpu()) < 1e-4
    assert torch.equal(out[0][4], out[1][4])


def _rccl_worker(rank, world, port, out):
    """One-rank RCCL ("nccl") group: the overlapped per-layer all-reduce path of the engine runs
    through RCCL itself (GradAllReduce(force=True) exchanges even at world size 1)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
                      HSA_ENABLE_IPC_MODE_LEGACY="0")
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "noise-robust-speech-embedding_amd"))
    import torch.distributed as dist
    from nrse_amd import arch as A, ddp, params as PR
    from nrse_amd.engine import ByolEngine
    torch.cuda.set_device(0)
    dist.init_process_group(backend="nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"
    arch = A.TINY.deterministic()
    layout = PR.byol_layout(arch, 256, 512)
    flat = PR.init_byol_flat(layout, 1234)
    g = torch.Generator().manual_seed(70)
    clean = (torch.randn(4, 16000, generator=g) * 0.1).cuda()
    noisy = clean + 0.05 * torch.randn(4, 16000, generator=g).cuda()
    res = {}
    for tag, wire in (("local", None), ("f32", "f32"), ("bf16", "bf16")):
        eng = ByolEngine(arch, 256, 512, device="cuda:0", compute_dtype=torch.float32, init_flat=flat)
        ar = None if wire is None else ddp.GradAllReduce(bucket_bytes=1 << 20, force=True,
                                                         wire_dtype=torch.bfloat16 if wire == "bf16" else None)
        eng.train_step(clean, noisy, lr=1e-4, step_seed=3, allreduce=ar)
        torch.cuda.synchronize()
        res[tag] = (eng.grad.cpu(), 0 if ar is None else ar.issued_elems)
        del eng
    out[0] = (res, layout.numel)
    dist.destroy_process_group()


def test_rccl_overlapped_allreduce_one_rank(nrse_device):
    """The engine's overlapped all-reduce through RCCL (backend "nccl"): at world size 1 the sum
    is the identity, so the exchanged f32 gradient equals the local one and the bf16 wire equals
    it rounded to bf16 (one bf16 ulp, 2^-8 relative, per element); every parameter range is sent."""
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_rccl_worker, args=(1, port, out), nprocs=1, join=True)
    res, numel = out[0]
    g_local = res["local"][0].double()

    def rel(a):
        return float((a.double() - g_local).norm() / g_local.norm())
    assert rel(res["f32"][0]) < 1e-5, rel(res["f32"][0])
    assert rel(res["bf16"][0]) < 4e-3, rel(res["bf16"][0])
    assert rel(res["bf16"][0]) > 0  # the wire really was bf16
    assert res["f32"][1] == numel and res["bf16"][1] == numel
