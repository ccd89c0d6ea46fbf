"""FedAvg over the data plane: RCCL (backend ``nccl``) over xGMI, or gloo on CPU.

Reference semantics (src/server.py:155-179): uniform average of EVERY
state-dict entry of the participating clients (params, BN running stats and
the int64 ``num_batches_tracked``, which becomes float and is truncated back on
load).  The reference does it on the coordinator's CPU after a gRPC gather of
base64 checkpoints; fedmi does it as ONE all-reduce of the client's flat fp32
state (:meth:`LocalTrainer.float_state`) — the result is already resident on
every client, so the reference's broadcast (SendModel, src/server.py:144-153)
disappears from the steady state.

``-c Y`` (compression) switches to :mod:`fedmi.parallel.compress`.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Optional

import torch
import torch.distributed as dist

from ..engine.base import LocalTrainer


def _world(group) -> int:
    if not dist.is_available() or not dist.is_initialized():
        return 1
    return dist.get_world_size(group)


def _supports_avg(group) -> bool:
    try:
        return dist.get_backend(group) == "nccl"
    except Exception:
        return False


def allreduce_mean_(t: torch.Tensor, group=None) -> torch.Tensor:
    """In-place mean over the group (RCCL ncclAvg; SUM+scale on gloo)."""
    w = _world(group)
    if w == 1:
        return t
    if _supports_avg(group):
        dist.all_reduce(t, op=dist.ReduceOp.AVG, group=group)
    else:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        t.div_(w)
    return t


def allreduce_int_mean_(t: torch.Tensor, group=None) -> torch.Tensor:
    """Integer buffers: sum then floor-divide (== reference float mean + int64 truncation)."""
    w = _world(group)
    if w == 1:
        return t
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    t.div_(w, rounding_mode="floor")
    return t


def broadcast_state_(trainer: LocalTrainer, src: int = 0, group=None) -> None:
    """Give every client rank ``src``'s model (fixes reference quirk A7: independent random inits)."""
    if _world(group) == 1:
        return
    dist.broadcast(trainer.float_state(), src=src, group=group)
    for b in trainer.int_state():
        dist.broadcast(b, src=src, group=group)
    trainer.after_aggregate()


@dataclass
class AggregationTimer:
    last_ms: float = 0.0
    total_ms: float = 0.0
    calls: int = 0


@dataclass
class FedAvg:
    """Dense or compressed FedAvg of a LocalTrainer's state across the group."""

    group: Optional[object] = None
    compressor: Optional[object] = None      # fedmi.parallel.compress.Compressor
    timer: AggregationTimer = field(default_factory=AggregationTimer)

    def world(self) -> int:
        return _world(self.group)

    def average(self, trainer: LocalTrainer) -> None:
        t0 = time.perf_counter()
        if self.world() > 1:
            if self.compressor is not None:
                self.compressor.aggregate(trainer, self.group)
            else:
                allreduce_mean_(trainer.float_state(), self.group)
            for b in trainer.int_state():
                allreduce_int_mean_(b, self.group)
        trainer.after_aggregate()
        dt = (time.perf_counter() - t0) * 1e3
        self.timer.last_ms = dt
        self.timer.total_ms += dt
        self.timer.calls += 1
