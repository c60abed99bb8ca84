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
    # NRSE_SHARE_DEVICE=1: every rank on device 0 (a rehearsal of the N-rank path on a one-GPU
    # box, with NRSE_DDP_BACKEND=gloo since RCCL refuses two ranks on one device)
    if os.environ.get("NRSE_SHARE_DEVICE", "0") == "1":
        local = 0
    if backend is None:
        backend = os.environ.get("NRSE_DDP_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    if backend == "nccl":
        torch.cuda.set_device(local)
    if not dist.is_initialized():
        dist.init_process_group(backend=backend)
    return rank, world, local


class GradAllReduce:
    """Sum all-reduce of a flat gradient buffer in buckets.

    Two ways to drive it:
      * `allreduce(flat)`: the whole buffer in fixed-size buckets (64 MiB by default: large
        enough to run at link bandwidth on the point-to-point xGMI ring, small enough to
        pipeline), issued asynchronously back to front and waited before returning;
      * overlapped with backward: `start()`, then `issue(view)` for each contiguous gradient
        range as soon as backward has finished writing it (the engine issues one transformer
        layer, ~50 MB of f32, at a time, on the stream that produced it), then `finish()`
        before the optimizer. `finish()` makes the current stream wait for every issued
        all-reduce (a device-side dependency, no host sync under NCCL/RCCL).
    """

    def __init__(self, group=None, bucket_bytes: int = 64 << 20, wire_dtype=None, force: bool = False):
        self.group = group
        # force=True: exchange even in a one-rank group (exercises the RCCL path on a one-GPU box)
        self.force = force
        self.bucket_bytes = bucket_bytes
        # wire_dtype=torch.bfloat16: each bucket is cast to bf16, summed by RCCL in bf16 (half the
        # xGMI bytes: 652 MB instead of 1.30 GB per step at WavLM-Large) and cast back into the
        # f32 gradient after the wait. None keeps the exact f32 sum.
        self.wire_dtype = wire_dtype
        self._works = []
        self.issued_elems = 0

    def active(self) -> bool:
        return dist.is_initialized() and (self.force or dist.get_world_size(self.group) > 1)

    def start(self) -> None:
        self._works = []
        self.issued_elems = 0

    def _to_wire(self, dst: torch.Tensor) -> torch.Tensor:
        """The bucket in the wire dtype: nrse_cast on the GPU (no ATen kernel in the step); CPU
        tensors (the gloo tests) through torch."""
        if not dst.is_cuda:
            return dst.to(self.wire_dtype)
        from . import kernels as K
        buf = torch.empty(dst.shape, device=dst.device, dtype=self.wire_dtype)
        K.cast(dst, buf)
        return buf

    @staticmethod
    def _from_wire(buf: torch.Tensor, dst: torch.Tensor) -> None:
        if not dst.is_cuda:
            dst.copy_(buf)
            return
        from . import kernels as K
        K.cast(buf, dst)

    def issue(self, view: torch.Tensor) -> None:
        """Asynchronously all-reduce one contiguous gradient range (split into buckets)."""
        if not self.active() or view.numel() == 0:
            return
        esize = view.element_size() if self.wire_dtype is None else torch.empty((), dtype=self.wire_dtype).element_size()
        step = max(1, self.bucket_bytes // esize)
        n = view.numel()
        end = n
        while end > 0:
            start = max(0, end - step)
            dst = view[start:end]
            buf = dst if self.wire_dtype is None else self._to_wire(dst)
            work = dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            self._works.append((work, buf, dst))
            end = start
        self.issued_elems += n

    def finish(self) -> None:
        for work, buf, dst in self._works:
            work.wait()
            if buf is not dst:
                self._from_wire(buf, dst)
                if buf.is_cuda:  # the wire copy is freed after this; keep it until the cast-back ran
                    buf.record_stream(torch.cuda.current_stream(buf.device))
        self._works = []

    def __call__(self, flat: torch.Tensor) -> None:
        self.start()
        self.issue(flat)
        self.finish()


class SyncBN:
    """SyncBatchNorm for the heads' BatchNorm1d layers (engine.sync_bn): the per-column batch
    statistics (forward) and the (sum dy, sum dy*xhat) terms (backward) are summed over the
    ranks with one small all-reduce each, so N ranks x B rows normalise like one B*N batch
    (torch.nn.SyncBatchNorm semantics). Off by default: the reference is single-process, and
    plain per-replica BatchNorm is what its modules would do under DDP."""

    def __init__(self, group=None):
        self.group = group

    def world(self) -> int:
        return dist.get_world_size(self.group)

    def all_reduce(self, t: torch.Tensor) -> None:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)


def all_reduce_sum(t: torch.Tensor, group=None) -> None:
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)


def world_size() -> int:
    return dist.get_world_size() if dist.is_initialized() else 1
