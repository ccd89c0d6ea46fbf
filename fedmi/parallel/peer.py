"""Peer-to-peer (hipIpc over xGMI) collectives for small FedAvg payloads.

The reference averages client models on the coordinator's CPU after a gRPC
gather of base64 checkpoints and broadcasts the result back
(src/server.py:51-75, 155-179).  fedmi's data plane does it on the GPUs:
:class:`PeerAllReduce` maps every client's staging buffer into every other
client's address space once (IPC handles exchanged through the rendezvous
store) and then runs each all-reduce as ONE kernel (csrc/comm/peer_comm.hip):
a flag barrier, then direct loads from all peers over all xGMI links.  For the
248 KB LeNet model that beats a ring collective, whose latency floor dominates
at that size.

Works with any ``torch.distributed`` store (TCPStore of torchrun, the
coordinator's generation store, or a FileStore) and with several ranks on ONE
GPU (same-device IPC), which is how it is tested on a single-GPU box.
"""
from __future__ import annotations

import os
import time
from typing import Optional

import torch
import torch.distributed as dist

from .. import native

ALGOS = {"oneshot": 0, "twoshot": 1}


def agree_any(store, key: str, rank: int, world: int, mine: bool) -> bool:
    """OR of a per-rank flag over all ranks, through the rendezvous store (blocks until all have set it)."""
    store.set(f"{key}/{rank}", b"1" if mine else b"0")
    return any(store.get(f"{key}/{r}") == b"1" for r in range(world))


class PeerAllReduce:
    """IPC-mapped all-reduce / all-gather among ``world`` ranks of one node."""

    def __init__(self, rank: int, world: int, capacity_bytes: int, store, tag: str = "default",
                 algo: str = "oneshot", timeout_ms: float = 30000.0, device: Optional[torch.device] = None):
        if algo not in ALGOS:
            raise ValueError(f"algo must be one of {sorted(ALGOS)}")
        self.nat = native.require()
        self.rank, self.world = rank, world
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.algo = algo
        self.store = store
        self.tag = tag
        with torch.cuda.device(self.device):
            self.comm = self.nat.PeerComm(rank, world, int(capacity_bytes))
            self.comm.set_timeout_ms(float(timeout_ms))
            key = f"fedmi/peer/{tag}"
            store.set(f"{key}/h{rank}", self.comm.handle())
            handles = [store.get(f"{key}/h{r}") for r in range(world)]
            self.comm.connect(handles)
        self._closed = False
        self.calls = 0
        self.timeout_ms = float(timeout_ms)
        # ranks sharing a GPU (one-GPU rehearsals / drills): a collective kernel spinning in its barrier
        # can keep a co-located peer's queued kernels from being scheduled until the barrier times out, so
        # each collective is gated by a host barrier once this rank's stream has drained.  The gate waits
        # for all ``world`` ranks, so the decision must be the same on every rank: it is taken if ANY rank
        # shares its GPU (e.g. 3 ranks on 2 GPUs gate all three).  Never taken with one rank per GPU (the
        # production layout).
        self.colocated = agree_any(store, f"{key}/coloc", rank, world, bool(self.comm.colocated)) and world > 1
        # diagnostics only (tools/bench_peer.py --no-gate): the kernels' own cost without the host gate, as
        # round 2 measured it before the gate existed -- the barrier timeout still bounds a non-co-scheduled peer
        if os.environ.get("FEDMI_PEER_GATE", "1") == "0":
            self.colocated = False
        self._gate_n = 0
        self._gate_failed = False
        self._abort = False

    def request_abort(self) -> None:
        """Called from a watchdog thread when the coordinator reports a lost client: every barrier of this
        communicator -- the kernel's (host-pinned abort word) and the co-located host gate -- fails at its
        next poll instead of waiting out ``timeout_ms``.  Sticky for this generation's communicator."""
        self._abort = True
        self.comm.request_abort()

    def _gate(self) -> bool:
        """False: a peer never reached this collective (its kernel must not be launched; ``error()`` is set)."""
        if self._abort:
            self._gate_failed = True
            return False
        if not self.colocated:
            return True
        if self._gate_failed:
            return False
        torch.cuda.current_stream(self.device).synchronize()
        self._gate_n += 1
        key = f"fedmi/peer/{self.tag}/gate{self._gate_n}"
        self.store.add(key, 1)
        deadline = time.monotonic() + self.timeout_ms / 1e3
        while int(self.store.add(key, 0)) < self.world:
            if self._abort or time.monotonic() > deadline:
                self._gate_failed = True
                return False
            time.sleep(0.0002)
        return True

    @property
    def capacity(self) -> int:
        return int(self.comm.capacity)

    def _stream(self) -> int:
        return native.stream_handle(self.device)

    def allreduce_mean_(self, t: torch.Tensor) -> torch.Tensor:
        """In place: t <- mean over ranks (fp32, rank-ordered sum: bit-identical on every rank)."""
        if not self._gate():
            return t
        if t.dtype == torch.float32:
            if not t.is_contiguous() or t.data_ptr() % 16:
                raise ValueError("peer all-reduce needs a contiguous, 16-byte aligned fp32 tensor")
            self.comm.allreduce_f32(self._stream(), t.data_ptr(), t.data_ptr(), t.numel(), 1.0 / self.world,
                                    ALGOS[self.algo], 0)
        elif t.dtype == torch.int64:
            self.comm.allreduce_i64_mean_floor(self._stream(), t.data_ptr(), t.data_ptr(), t.numel())
        else:
            raise TypeError(f"peer all-reduce: unsupported dtype {t.dtype}")
        self.calls += 1
        return t

    def allreduce_sum(self, src: torch.Tensor, dst: torch.Tensor, scale: float = 1.0) -> torch.Tensor:
        if not self._gate():
            return dst
        self.comm.allreduce_f32(self._stream(), src.data_ptr(), dst.data_ptr(), src.numel(), float(scale),
                                ALGOS[self.algo], 0)
        self.calls += 1
        return dst

    def int8_ef_allreduce_(self, x: torch.Tensor, g: torch.Tensor, r: torch.Tensor) -> None:
        """-c Y fused into the collective (one launch): x - g + r is quantised to int8 per 256-entry chunk with the
        quantisation error kept in ``r``, every rank's int8 payload is dequantised and averaged in rank order into
        ``g``, and ``x`` becomes the new global model ``g`` (fp32, contiguous, same length)."""
        if not self._gate():
            return
        self.comm.allreduce_int8_ef(self._stream(), x.data_ptr(), g.data_ptr(), r.data_ptr(), x.numel(),
                                    1.0 / self.world)
        self.calls += 1

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """[world, *t.shape] with rank r's tensor in row r."""
        t = t.contiguous()
        nbytes = t.numel() * t.element_size()
        pad = (-nbytes) % 16
        if pad:
            flat = torch.zeros(nbytes + pad, dtype=torch.uint8, device=t.device)
            flat[:nbytes].copy_(t.view(-1).view(torch.uint8))
            src = flat
        else:
            src = t.view(-1).view(torch.uint8)
        out = torch.empty(self.world * (nbytes + pad), dtype=torch.uint8, device=t.device)
        if not self._gate():
            return out.view(self.world, nbytes + pad)[:, :nbytes].contiguous().view(t.dtype).view((self.world,) + tuple(t.shape))
        self.comm.allgather(self._stream(), src.data_ptr(), out.data_ptr(), nbytes + pad, 0)
        self.calls += 1
        rows = out.view(self.world, nbytes + pad)[:, :nbytes].contiguous()
        return rows.view(t.dtype).view((self.world,) + tuple(t.shape))

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        """In place: every rank gets rank ``src``'s ``t`` (an all-gather, row ``src`` kept)."""
        t.copy_(self.all_gather(t)[src])
        return t

    def error(self) -> int:
        """Nonzero if a barrier timed out (a peer died or never arrived); synchronous."""
        return int(self.comm.error()) or int(self._gate_failed)

    def close(self, barrier: bool = True) -> None:
        """Unmap peers.  With ``barrier`` every rank first drains its stream and waits for the
        others through the store, so no rank frees memory a peer may still read."""
        if self._closed:
            return
        self._closed = True
        torch.cuda.synchronize(self.device)
        if barrier and self.world > 1:
            key = f"fedmi/peer/{self.tag}/closing"
            self.store.add(key, 1)
            deadline = time.monotonic() + 60.0
            while int(self.store.add(key, 0)) < self.world and time.monotonic() < deadline:
                time.sleep(0.002)
        self.comm.disconnect()


def make_peer_allreduce(t: torch.Tensor, store=None, tag: str = "fedavg", algo: str = "oneshot",
                        group=None, headroom: float = 1.0) -> PeerAllReduce:
    """PeerAllReduce sized for ``t`` among the ranks of the default (or given) process group."""
    if store is None:
        store = dist.distributed_c10d._get_default_store()
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    cap = max(4096, int(t.numel() * t.element_size() * headroom))
    return PeerAllReduce(rank, world, cap, store, tag=tag, algo=algo, device=t.device)
