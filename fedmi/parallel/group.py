"""Elastic data-plane membership for gRPC-driven clients.

The coordinator tells each live client its (rank, world) in ``TrainRequest``
(reference semantics, src/server.py:54) plus, in gRPC metadata, a membership
*generation* and the address of a rendezvous ``TCPStore`` it hosts.  A client
whose (generation, rank, world) changed drops its data plane and joins a fresh
one under a generation-prefixed store namespace, so a dead or rejoining client
never wedges the survivors (reference quirks A5/A6: world counted dead clients,
stale files were averaged).

Two data planes:

* ``peer`` (GPU clients of one node): the hipIpc peer kernels of
  :mod:`fedmi.parallel.peer`.  No communicator at all -- the store only carries
  the IPC handles.  A peer that dies mid-collective makes the survivors' barrier
  time out (bounded, sets an error flag) instead of hanging; the next generation
  maps fresh buffers.
* ``dist``: a ``torch.distributed`` process group (``nccl`` = RCCL over xGMI on
  GPUs, ``gloo`` on CPU hosts).  A broken RCCL communicator is ABORTED
  (``ncclCommAbort`` via the process group), never destroyed: destroy would
  block on the dead peer.  The collective timeout is short (``timeout_s``).
* ``auto`` (GPU clients' default): at the first generation with world > 1 the
  client forms BOTH, verifies the peer kernels against the process group's
  all-reduce on random data and times both on a model-sized buffer
  (:func:`fedmi.parallel.select.verify_and_select`, the same check bench.py
  runs); the faster verified plane is kept for every later generation.  Ranks
  sharing a GPU cannot run RCCL: they verify against gloo and keep the peer.
"""
from __future__ import annotations

import datetime
import threading
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass(frozen=True)
class Membership:
    generation: int
    rank: int
    world: int
    store_host: str
    store_port: int


def abort_default_group() -> None:
    """Tear down the default process group without talking to (possibly dead) peers."""
    if not dist.is_initialized():
        return
    try:
        if dist.get_backend() == "nccl":
            dist.distributed_c10d._abort_process_group()     # ncclCommAbort: never blocks on a dead peer
        else:
            dist.destroy_process_group()
    except Exception:  # pragma: no cover - best effort on a broken communicator
        try:
            dist.destroy_process_group()
        except Exception:
            pass


class GroupManager:
    def __init__(self, backend: str, device: Optional[torch.device] = None, timeout_s: float = 20.0,
                 transport: str = "dist", peer_capacity: int = 0, peer_timeout_ms: float = 10000.0,
                 init_world1: bool = False, model_numel: int = 0):
        """``init_world1``: form a process group even for a client alone (world 1); by default a
        lone client has no data plane at all, since FedAvg of one model is the identity."""
        if transport not in ("dist", "peer", "auto"):
            raise ValueError("transport must be 'dist', 'peer' or 'auto'")
        self.backend = backend
        self.device = device
        self.timeout = datetime.timedelta(seconds=timeout_s)
        self.transport_kind = transport
        self.peer_capacity = peer_capacity
        self.peer_timeout_ms = peer_timeout_ms
        self.init_world1 = init_world1
        self.model_numel = model_numel       # auto: size of the buffer the candidates are timed on
        self.current: Optional[Membership] = None
        self.transport = None               # PeerAllReduce of the current generation (peer mode)
        self._retired: list = []            # previous generations' buffers, kept mapped a while: a peer that
                                            # has not noticed the regroup yet may still touch them
        self._lock = threading.Lock()
        self.generations_joined = 0
        self.selected: Optional[str] = None   # auto: "peer" | "dist" once decided
        self.select_info: dict = {}

    def _drop(self) -> None:
        if self.transport is not None:
            try:
                self.transport.close(barrier=False)
            except Exception:  # pragma: no cover
                pass
            self._retired = (self._retired + [self.transport])[-4:]
            self.transport = None
        abort_default_group()
        self.current = None

    def ensure(self, m: Membership) -> bool:
        """Join (or re-join) the data-plane group described by ``m``; True if it changed."""
        with self._lock:
            if self.current == m and ((m.world == 1 and not self.init_world1) or self.transport is not None
                                      or dist.is_initialized()):
                return False
            self._drop()
            kind = self.transport_kind if self.transport_kind != "auto" else (self.selected or "auto")
            if m.world > 1 or (self.init_world1 and kind == "dist"):
                store = dist.TCPStore(m.store_host, m.store_port, world_size=None, is_master=False,
                                      timeout=self.timeout, wait_for_workers=False)
                pstore = dist.PrefixStore(f"fedmi/gen{m.generation}", store)
                if kind == "auto":
                    self._select(m, pstore)
                elif kind == "peer":
                    self.transport = self._peer(m, pstore)
                else:
                    self._init_group(self.backend, m, pstore)
            self.current = m
            self.generations_joined += 1
            return True

    def _peer(self, m: Membership, pstore):
        from .peer import PeerAllReduce

        if self.peer_capacity <= 0:
            raise ValueError("peer transport needs peer_capacity > 0")
        peer = PeerAllReduce(m.rank, m.world, self.peer_capacity, pstore, tag=f"gen{m.generation}",
                             timeout_ms=self.peer_timeout_ms, device=self.device)
        if self.selected == "peer" and self.select_info.get("chosen"):
            peer.algo = self.select_info["chosen"]
        return peer

    def _init_group(self, backend: str, m: Membership, store) -> None:
        kw = {}
        if backend == "nccl" and self.device is not None:
            kw["device_id"] = self.device
        dist.init_process_group(backend, store=store, rank=m.rank, world_size=m.world, timeout=self.timeout, **kw)

    def _select(self, m: Membership, pstore) -> None:
        """First multi-client generation of an ``auto`` client: verify + time peer vs the process group."""
        from .select import verify_and_select

        peer = self._peer(m, pstore)
        backend = "gloo" if (peer.colocated or self.device is None or self.device.type != "cuda") else self.backend
        self._init_group(backend, m, dist.PrefixStore("select", pstore))
        numel = self.model_numel or max(1, self.peer_capacity // 4)
        try:
            choice, info = verify_and_select(peer, numel, self.device)
        except Exception:
            peer.close(barrier=False)
            raise
        info["group_backend"] = backend
        self.select_info = info
        if choice is None:                   # RCCL won: it carries FedAvg from now on
            peer.close(barrier=True)
            self.selected = "dist"
        else:
            self.transport = peer
            self.selected = "peer"
            dist.destroy_process_group()       # healthy group, all ranks here: a plain destroy

    def interrupt(self) -> None:
        """Called WITHOUT the agent lock when a newer generation arrives while an old round is
        still blocked in a collective: abort the RCCL communicator so that round fails fast.
        (Peer collectives need nothing: their barriers time out on their own.)"""
        if self.transport is None and dist.is_initialized() and self.backend == "nccl":
            abort_default_group()

    def shutdown(self) -> None:
        with self._lock:
            self._drop()


class StoreHost:
    """Rendezvous TCPStore hosted by the (acting) coordinator."""

    def __init__(self, host: str = "127.0.0.1", port: int = 0, timeout_s: float = 60.0):
        self.store = dist.TCPStore(host, port, world_size=None, is_master=True,
                                   timeout=datetime.timedelta(seconds=timeout_s), wait_for_workers=False)
        self.host = host
        self.port = self.store.port
