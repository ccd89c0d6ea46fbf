"""``-c Y``: compressed FedAvg updates on the data plane.

Reference -c Y = gRPC gzip of base64 fp32 checkpoints (src/server.py:103-107,
src/client.py:39-43): 0.98-0.99x of the raw size at 16 ms-3 s of CPU per
message.  fedmi keeps the flag (and gzip on the gRPC control
channel) and compresses the *update* instead:

* ``topk``  — each client sends the k largest-magnitude entries of
  d = (w_local - w_global) + e (error feedback e carries the rest to the next
  round); selection is exact, on the GPU in 4 launches and 2 passes over the
  state (csrc/kernels/compress.hip ``launch_topk_ef``: fused delta + 11-bit
  histogram, bin pick, wave-aggregated compaction of the certain winners and the
  boundary-bin candidates, exact candidate select); (idx, val) pairs are all-gathered (RCCL, or the
  hipIpc peer kernels of :mod:`fedmi.parallel.peer`) and applied to the global
  model in rank order without atomics, so every client holds a bit-identical
  global model.  Payload per client: 8k bytes.
* ``int8``  — per-256-element absmax int8 quantisation with error feedback;
  payload n + 4n/256 bytes (~3.9x smaller than fp32).

After aggregation every client holds w_global' = w_global + mean(sparse d),
exactly like dense FedAvg when k = n.

Every client must hold the same anchor ``global_ref``.  It is re-anchored
(:meth:`reset`) whenever the model is replaced from outside — a rank-0 init
broadcast, a SendModel resync, a new membership generation — and a client
that trains alone (world 1) simply adopts its local model.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from .. import native


def _world(group) -> int:
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


PROBE = None          # diagnostics hook (client agent, FEDMI_DEBUG_STATS=1): called with a phase tag


def _probe(tag: str) -> None:
    if PROBE is not None:
        PROBE(tag)


def _all_gather_flat(t: torch.Tensor, group, transport=None) -> torch.Tensor:
    if transport is not None:
        return transport.all_gather(t)
    w = _world(group)
    if w == 1:
        return t.clone().unsqueeze(0)
    out = torch.empty((w,) + tuple(t.shape), dtype=t.dtype, device=t.device)
    if t.is_cuda:
        dist.all_gather_into_tensor(out.view(-1), t.contiguous().view(-1), group=group)
    else:
        dist.all_gather(list(out.unbind(0)), t.contiguous(), group=group)
    return out


class _EFCompressor:
    """``warmup``: the first ``warmup`` aggregations are dense FedAvg (the largest updates of a run come
    first, when a 1 % selection defers most of them); compression starts from the dense global model
    with an empty residual."""

    def __init__(self, trainer, warmup: int = 0):
        self.warmup = int(warmup)
        self.dense_rounds = 0
        x = trainer.float_state()
        self.n = x.numel()
        self.dev = x.device
        self.global_ref = x.detach().clone()
        self.residual = torch.zeros_like(self.global_ref)
        self.d = torch.empty_like(self.global_ref)
        self._nat = native.require() if x.is_cuda else None
        self.bytes_sent = 0          # this client's compressed payload bytes, summed over rounds
        self.dense_bytes = 0         # what dense fp32 FedAvg would have sent
        self.rounds = 0

    def reset(self, trainer) -> None:
        """Re-anchor on the trainer's current model (after a resync/load)."""
        self.global_ref.copy_(trainer.float_state())
        self.residual.zero_()

    def _dense(self, x: torch.Tensor, group, transport) -> bool:
        """Dense FedAvg of ``x`` while in warm-up; True if it ran (the anchor follows, residual empty)."""
        if self.dense_rounds >= self.warmup:
            return False
        if transport is not None:
            transport.allreduce_mean_(x)
        else:
            from .fedavg import allreduce_mean_

            allreduce_mean_(x, group)
        self.global_ref.copy_(x)
        self.residual.zero_()
        self.dense_rounds += 1
        self.bytes_sent += 4 * self.n
        self.dense_bytes += 4 * self.n
        self.rounds += 1
        return True

    def _delta(self, x: torch.Tensor) -> None:
        if self._nat is not None:
            self._nat.ef_delta(native.stream_handle(self.dev), x.data_ptr(), self.global_ref.data_ptr(),
                               self.residual.data_ptr(), self.d.data_ptr(), self.n)
        else:
            torch.sub(x, self.global_ref, out=self.d)
            self.d.add_(self.residual)


class TopKCompressor(_EFCompressor):
    def __init__(self, trainer, ratio: float = 0.01, warmup: int = 0):
        super().__init__(trainer, warmup)
        self.k = max(1, min(self.n, int(round(self.n * ratio))))
        self.idx = torch.empty(self.k, dtype=torch.int32, device=self.dev)
        self.val = torch.empty(self.k, dtype=torch.float32, device=self.dev)
        if self._nat is not None:
            self.state = torch.zeros(self._nat.topk_state_bytes(), dtype=torch.uint8, device=self.dev)
            # boundary-bin candidates (index, key) + the level-3 list: sized for the worst case (every
            # entry in one bin)
            self.cidx = torch.empty(2 * self.n, dtype=torch.int32, device=self.dev)
            self.ckey = torch.empty(2 * self.n, dtype=torch.int32, device=self.dev)

    def overflowed(self, clear: bool = True) -> bool:
        """True if a select ever produced more than k entries (the excess was dropped, never written
        past the payload; a kernel bug, not a data condition).  Synchronous; read at end of run."""
        if self._nat is None:
            return False
        off = int(self._nat.topk_overflow_offset())
        word = self.state[off:off + 4].view(torch.int32)
        hit = bool(word.item())
        if clear and hit:
            word.zero_()
        return hit

    def compress(self, x: torch.Tensor) -> None:
        if self._nat is not None:
            # d = x - global + residual is built IN the residual buffer; the winners are zeroed there
            self._nat.topk_ef(native.stream_handle(self.dev), x.data_ptr(), self.global_ref.data_ptr(),
                              self.residual.data_ptr(), self.n, self.k, self.state.data_ptr(), self.cidx.data_ptr(),
                              self.ckey.data_ptr(), self.idx.data_ptr(), self.val.data_ptr())
            return
        self._delta(x)
        sel = self.d.abs().topk(self.k, sorted=False).indices
        self.idx.copy_(sel.to(torch.int32))
        self.val.copy_(self.d[sel])
        self.residual.copy_(self.d)
        self.residual[sel] = 0.0

    def aggregate(self, trainer, group=None, transport=None) -> None:
        x = trainer.float_state()
        if self._dense(x, group, transport):
            return
        self.compress(x)
        _probe("topk")
        w = transport.world if transport is not None else _world(group)
        idx_all = _all_gather_flat(self.idx, group, transport)
        _probe("gather-idx")
        val_all = _all_gather_flat(self.val, group, transport)
        _probe("gather-val")
        self.bytes_sent += 8 * self.k
        self.dense_bytes += 4 * self.n
        self.rounds += 1
        if self._nat is not None:
            self._nat.scatter_add_ranked(native.stream_handle(self.dev), self.global_ref.data_ptr(),
                                         idx_all.data_ptr(), val_all.data_ptr(), w, self.k, 1.0 / w, self.n)
        else:
            for r in range(w):                 # rank order, like the GPU path
                self.global_ref.index_add_(0, idx_all[r].long(), val_all[r] * (1.0 / w))
        x.copy_(self.global_ref)
        _probe("scatter")


class Int8Compressor(_EFCompressor):
    CHUNK = 256

    def __init__(self, trainer, warmup: int = 0):
        super().__init__(trainer, warmup)
        self.nchunks = (self.n + self.CHUNK - 1) // self.CHUNK
        self.q = torch.empty(self.n, dtype=torch.int8, device=self.dev)
        self.scales = torch.empty(self.nchunks, dtype=torch.float32, device=self.dev)

    def compress(self, x: torch.Tensor) -> None:
        self._delta(x)
        if self._nat is not None:
            self._nat.quant_int8(native.stream_handle(self.dev), self.d.data_ptr(), self.n, self.q.data_ptr(),
                                 self.scales.data_ptr(), self.residual.data_ptr())
        else:
            pad = torch.zeros(self.nchunks * self.CHUNK, device=self.dev)
            pad[:self.n] = self.d
            blocks = pad.view(self.nchunks, self.CHUNK)
            amax = blocks.abs().amax(1)
            s = torch.where(amax > 0, amax / 127.0, torch.ones_like(amax))
            q = torch.round(blocks / s[:, None]).clamp_(-127, 127)
            self.q.copy_(q.view(-1)[:self.n].to(torch.int8))
            self.scales.copy_(s)
            self.residual.copy_(self.d - (q * s[:, None]).view(-1)[:self.n])

    # the fused peer kernel (quantise + exchange + dequantise-average in one launch); False: the unfused
    # reference path (tests compare the two bit for bit)
    fused = True

    def aggregate(self, trainer, group=None, transport=None) -> None:
        x = trainer.float_state()
        if self._dense(x, group, transport):
            return
        if self.fused and transport is not None and hasattr(transport, "int8_ef_allreduce_"):
            transport.int8_ef_allreduce_(x, self.global_ref, self.residual)
            self.bytes_sent += self.n + 4 * self.nchunks
            self.dense_bytes += 4 * self.n
            self.rounds += 1
            return
        self.compress(x)
        w = transport.world if transport is not None else _world(group)
        q_all = _all_gather_flat(self.q, group, transport)
        s_all = _all_gather_flat(self.scales, group, transport)
        self.bytes_sent += self.n + 4 * self.nchunks
        self.dense_bytes += 4 * self.n
        self.rounds += 1
        if self._nat is not None:
            self._nat.dequant_accum(native.stream_handle(self.dev), q_all.data_ptr(), s_all.data_ptr(), w, self.n,
                                    self.global_ref.data_ptr(), 1.0 / w)
        else:
            idx = torch.arange(self.n, device=self.dev) // self.CHUNK
            deq = q_all.float() * s_all[:, idx]
            self.global_ref.add_(deq.sum(0) / w)
        x.copy_(self.global_ref)


# What ``-c Y`` selects: the compressor that stays within 3 points of dense FedAvg at the fewest bytes on the
# 8-rank rehearsal (profiles/r5_dataplane/: 3 seeds x 23 rounds) -- int8 + error feedback, a quarter of the dense
# bytes; top-k needs ~20 % of the entries (40 % of the dense bytes: 8 B per kept entry) to get as close.
DEFAULT_Y = "int8"
DEFAULT_TOPK_RATIO = 0.2


def make_compressor(kind: Optional[str], ratio: float, trainer, warmup: int = 0):
    if kind in (None, "", "none", "n", "N"):
        return None
    if kind in ("Y", "y"):
        kind = DEFAULT_Y
    if kind == "topk":
        return TopKCompressor(trainer, ratio, warmup)
    if kind == "int8":
        return Int8Compressor(trainer, warmup)
    raise ValueError(f"unknown compression {kind!r}")
