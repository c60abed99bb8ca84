"""Health checks of the training loop (train_byol.py:52-59, src/utils/debugging_utils.py:4-30).

The reference runs check_audio_tensor on clean / noisy inputs and on online_pred / target_proj
every step: four reductions and up to eight host syncs, logging a warning per bad tensor (it
never stops training). Here one device kernel (nrse_health) reduces each tensor into a stats row
[nan count, inf count, sum|x|, max|x|] inside the fused step, and HealthMonitor reads the rows
back a few steps later from pinned memory, so the warnings appear with a lag of `lag` steps and
no host sync is added to the step. The decision order and messages follow check_audio_tensor.
"""
from __future__ import annotations

import logging
from collections import deque

import torch

from . import kernels as K

logger = logging.getLogger("nrse")

HEALTH_NAMES = ("clean_input_values", "noisy_input_values", "online_pred", "target_proj")


def interpret(stats, name: str, max_threshold: float = 1e6, min_threshold: float = 1e-6):
    """(ok, warning message or None) for one stats row, in check_audio_tensor's order:
    NaN, Inf, sum|x| < min_threshold, max|x| > max_threshold (debugging_utils.py:6-22)."""
    nan, inf, sabs, mabs = (float(v) for v in stats[:4])
    if nan > 0:
        return False, f"WARNING: {name} contains NaN values!"
    if inf > 0:
        return False, f"WARNING: {name} contains Inf values!"
    if sabs < min_threshold:
        return False, f"WARNING: {name} contains very small values!"
    if mabs > max_threshold:
        return False, f"WARNING: {name} contains very large values! Max abs value: {mabs}"
    return True, None


def tensor_stats(tensor: torch.Tensor) -> torch.Tensor:
    """Device stats row of one tensor via nrse_health (f32/bf16 device tensors)."""
    t = tensor.contiguous()
    stats = torch.zeros(4, device=t.device, dtype=torch.float32)
    K.health(t, stats)
    return stats


def check_audio_tensor(tensor, name, config, max_threshold=1e6, min_threshold=1e-6) -> bool:
    """Drop-in for src/utils/debugging_utils.py:4-30 (synchronous, like the reference)."""
    ok, msg = interpret(tensor_stats(tensor).cpu(), name, max_threshold, min_threshold)
    if not ok:
        logger.warning(msg)
        return False
    if config.get("logging", {}).get("level") == "DEBUG":
        x = tensor.float()
        logger.debug(f"Stats for {name}: mean={x.mean().item():.4f}, std={x.std().item():.4f}, "
                     f"min={x.min().item():.4f}, max={x.max().item():.4f}")
    return True


SAT_NAMES = ("layer-weight fp8 correction planes", "conv-stack fp8 planes", "layer-activation fp8 copies")


class HealthMonitor:
    """Deferred reader of the engine's per-step health rows (engine.health_buf [4, 4]) and, with
    an engine, of its fp8 saturation counters (engine.sat_buf, ABI 10): a count that moved since
    the engine's last re-derivation makes the monitor call engine.rederive_split_exponents() (the
    split-weight mode's exponents follow weights that grew in training), with the same lag."""

    def __init__(self, lag: int = 2, names=HEALTH_NAMES):
        self.lag = lag
        self.names = names
        self._pending = deque()
        self.warnings = []       # (step, message), for tests and logs
        self.rederived = []      # (step, engine.rederive_split_exponents() result)

    def record(self, step: int, health_buf: torch.Tensor, engine=None) -> None:
        host = torch.empty(health_buf.shape, dtype=health_buf.dtype, pin_memory=True)
        host.copy_(health_buf, non_blocking=True)
        sat = None
        if engine is not None and getattr(engine, "sat_buf", None) is not None:
            sat = torch.empty(engine.sat_buf.shape, dtype=engine.sat_buf.dtype, pin_memory=True)
            sat.copy_(engine.sat_buf, non_blocking=True)
            sat = (sat, engine, engine.sat_epoch)
        ev = torch.cuda.Event()
        ev.record()
        self._pending.append((step, host, ev, sat))
        while len(self._pending) > self.lag:
            self._drain_one()

    def _drain_one(self) -> None:
        step, host, ev, sat = self._pending.popleft()
        ev.synchronize()
        for row, name in zip(host, self.names):
            ok, msg = interpret(row, name)
            if not ok:
                logger.warning(f"step {step}: {msg}")
                self.warnings.append((step, msg))
        if sat is not None:
            counts, engine, epoch = sat
            # a copy taken before the last re-derivation reports counts that are already handled
            if epoch == engine.sat_epoch and int(counts.abs().sum()) > 0:
                what = ", ".join(f"{n}: {int(c)}" for n, c in zip(SAT_NAMES, counts) if int(c))
                msg = f"fp8 correction conversions saturated ({what}); re-deriving the split-weight exponents"
                logger.warning(f"step {step}: {msg}")
                self.warnings.append((step, msg))
                self.rederived.append((step, engine.rederive_split_exponents()))

    def flush(self) -> None:
        while self._pending:
            self._drain_one()
