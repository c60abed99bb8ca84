"""Data parallelism: one process per GPU, torch.distributed over RCCL ("nccl" backend on ROCm)
over xGMI. The reference has no distribution; this adds the single exchange
step the path needs: a sum all-reduce of the online gradients, bucketed over
the flat f32 gradient buffer in reverse layout order (the order backward finishes them).
Everything else (clip, AdamW, EMA, target network) runs replicated and identical on every rank;
the optimizer applies grad_scale = 1/world_size, so the update equals the single-process
update on the concatenated batch (up to BatchNorm batch statistics, which stay per-replica
like the reference's BatchNorm1d would under plain DDP).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def init_from_env(backend: str | None = None):
    """Initialise the default process group from torchrun's env (RANK/WORLD_SIZE/MASTER_*)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return 0, 1, int(os.environ.get("LOCAL_RANK", "0"))
    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local)
    if not dist.is_initialized():
        dist.init_process_group(backend=backend)
    return rank, world, local


class GradAllReduce:
    """Sum all-reduce of a flat gradient buffer in fixed-size buckets, issued asynchronously
    back to front and waited before the optimizer (64 MiB buckets by default: large enough to
    run at link bandwidth on the point-to-point xGMI ring, small enough to pipeline)."""

    def __init__(self, group=None, bucket_bytes: int = 64 << 20):
        self.group = group
        self.bucket_bytes = bucket_bytes

    def __call__(self, flat: torch.Tensor) -> None:
        if not dist.is_initialized() or dist.get_world_size(self.group) == 1:
            return
        n = flat.numel()
        step = max(1, self.bucket_bytes // flat.element_size())
        works = []
        end = n
        while end > 0:
            start = max(0, end - step)
            works.append(dist.all_reduce(flat[start:end], op=dist.ReduceOp.SUM, group=self.group, async_op=True))
            end = start
        for w in works:
            w.wait()


def world_size() -> int:
    return dist.get_world_size() if dist.is_initialized() else 1
