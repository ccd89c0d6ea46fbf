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

import threading
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


def _run(fn, t: torch.Tensor, group, abort: Optional[threading.Event], **kw) -> None:
    """One collective.  RCCL is stream-ordered (an abort is ncclCommAbort from the watchdog); a host-blocking
    backend (gloo) runs it ``async_op`` and stops waiting when ``abort`` is set
    (:func:`fedmi.parallel.group.wait_work`)."""
    if abort is None or _supports_avg(group):
        fn(t, group=group, **kw)
        return
    from .group import wait_work

    wait_work(fn(t, group=group, async_op=True, **kw), abort, fn.__name__)


def allreduce_mean_(t: torch.Tensor, group=None, abort: Optional[threading.Event] = None) -> torch.Tensor:
    """In-place mean over the group (RCCL ncclAvg; SUM+scale on gloo)."""
    w = _world(group)
    if w == 1:
        return t
    if _supports_avg(group):
        dist.all_reduce(t, op=dist.ReduceOp.AVG, group=group)
    else:
        _run(dist.all_reduce, t, group, abort, op=dist.ReduceOp.SUM)
        t.div_(w)
    return t


def allreduce_int_mean_(t: torch.Tensor, group=None, abort: Optional[threading.Event] = None) -> torch.Tensor:
    """Integer buffers: sum then floor-divide (== reference float mean + int64 truncation)."""
    w = _world(group)
    if w == 1:
        return t
    _run(dist.all_reduce, t, group, abort, op=dist.ReduceOp.SUM)
    t.div_(w, rounding_mode="floor")
    return t


def broadcast_state_(trainer: LocalTrainer, src: int = 0, group=None, abort: Optional[threading.Event] = None) -> None:
    """Give every client rank ``src``'s model (fixes reference quirk A7: independent random inits)."""
    if _world(group) == 1:
        return
    _run(dist.broadcast, trainer.float_state(), group, abort, src=src)
    for b in trainer.int_state():
        _run(dist.broadcast, b, group, abort, src=src)
    trainer.after_aggregate()


@dataclass
class AggregationTimer:
    last_ms: float = 0.0
    total_ms: float = 0.0
    calls: int = 0


@dataclass
class FedAvg:
    """Dense or compressed FedAvg of a LocalTrainer's state across the group.

    ``transport``: a :class:`fedmi.parallel.peer.PeerAllReduce` — the hand-written
    hipIpc peer kernels carry the aggregation instead of ``torch.distributed``
    collectives (RCCL on GPUs, gloo on CPU).
    """

    group: Optional[object] = None
    compressor: Optional[object] = None      # fedmi.parallel.compress.Compressor
    transport: Optional[object] = None       # fedmi.parallel.peer.PeerAllReduce
    timer: AggregationTimer = field(default_factory=AggregationTimer)
    abort: Optional[threading.Event] = None  # the generation's loss flag (GroupManager.abort_event)

    def world(self) -> int:
        if self.transport is not None:
            return self.transport.world
        return _world(self.group)

    def label(self) -> str:
        """What actually carries the aggregation (reported by the benches)."""
        if self.world() == 1:
            base = "none (single client)"
        elif self.transport is not None:
            base = f"peer-{self.transport.algo}-hipipc"
        else:
            be = dist.get_backend(self.group)
            base = "rccl-allreduce" if be == "nccl" else f"{be}-allreduce"
        if self.compressor is not None and self.world() > 1:
            base += "+" + type(self.compressor).__name__.replace("Compressor", "").lower()
        return base

    def average(self, trainer: LocalTrainer) -> None:
        t0 = time.perf_counter()
        if self.world() > 1:
            if self.compressor is not None:
                self.compressor.aggregate(trainer, self.group, transport=self.transport)
            elif self.transport is not None:
                self.transport.allreduce_mean_(trainer.float_state())
            else:
                allreduce_mean_(trainer.float_state(), self.group, self.abort)
            for b in trainer.int_state():
                if self.transport is not None:
                    self.transport.allreduce_mean_(b)
                else:
                    allreduce_int_mean_(b, self.group, self.abort)
        elif self.compressor is not None:
            # a client training alone holds the global model: it becomes the new anchor
            self.compressor.reset(trainer)
        trainer.after_aggregate()
        dt = (time.perf_counter() - t0) * 1e3
        self.timer.last_ms = dt
        self.timer.total_ms += dt
        self.timer.calls += 1

    def resync(self, trainer: LocalTrainer, src: int = 0) -> None:
        """Everyone adopts rank ``src``'s model (init, or after an aborted round) and re-anchors."""
        if self.transport is not None:
            if self.transport.world > 1:
                self.transport.broadcast_(trainer.float_state(), src)
                for b in trainer.int_state():
                    self.transport.broadcast_(b, src)
            trainer.after_aggregate()
        else:
            broadcast_state_(trainer, src, self.group, self.abort)
        if self.compressor is not None:
            self.compressor.reset(trainer)


def eval_shard(test, rank: int, world: int):
    """Contiguous 1/world slice of the test set for data-parallel evaluation.

    After FedAvg every client holds the same global model, so the reference's
    "every client evaluates the full test set" (src/client.py:30 ->
    src/main.py:167-191) computes the same numbers ``world`` times; splitting
    the set and summing the (loss, correct, count) accumulators over the clients
    gives the identical global result with 1/world of the work per client.
    """
    n = len(test)
    lo, hi = n * rank // world, n * (rank + 1) // world
    return type(test)(test.x[lo:hi], test.y[lo:hi])


class EvalHistory:
    """Per-round eval accumulators kept on device; one collective when read.

    ``record()`` after each :meth:`LocalTrainer.evaluate` is a 16-byte
    device-to-device copy (no host sync, no collective on the round's critical
    path); ``reduce()`` sums every round's (loss_sum, correct, count) over the
    group in ONE all-reduce and returns the global per-round EpochStats.
    """

    def __init__(self, trainer: LocalTrainer, max_rounds: int):
        raw = trainer.eval_stats_raw()
        self.trainer = trainer
        self.buf = torch.zeros((max_rounds,) + tuple(raw.shape), dtype=raw.dtype, device=raw.device)
        self.n = 0

    def record(self) -> None:
        if self.n >= self.buf.shape[0]:
            raise IndexError("EvalHistory full")
        es = self.trainer.eval_stream()
        if es is None:
            self.buf[self.n].copy_(self.trainer.eval_stats_raw(), non_blocking=True)
        else:                                  # the eval runs overlapped on its own stream: copy there
            with torch.cuda.stream(es):
                self.buf[self.n].copy_(self.trainer.eval_stats_raw(), non_blocking=True)
        self.n += 1

    def reduce(self, group=None):
        from ..engine.base import EpochStats

        es = self.trainer.eval_stream()
        if es is not None:
            torch.cuda.current_stream(self.buf.device).wait_stream(es)
        rows = self.buf[: self.n].cpu()
        vals = [self.trainer.decode_stats(rows[i]) for i in range(self.n)]
        t = torch.tensor([[s.loss_sum, s.correct, s.count] for s in vals], dtype=torch.float64).reshape(-1, 3)
        if _world(group) > 1:
            if _supports_avg(group):           # RCCL reduces device tensors
                t = t.to(self.buf.device)
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
            t = t.cpu()
        return [EpochStats(float(a), int(round(b)), int(round(c))) for a, b, c in t.tolist()]
