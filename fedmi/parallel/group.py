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
                 init_world1: bool = False):
        """``init_world1``: form a process group even for a client alone (world 1); by default a
        lone client has no data plane at all, since FedAvg of one model is the identity."""
        if transport not in ("dist", "peer"):
            raise ValueError("transport must be 'dist' or 'peer'")
        self.backend = backend
        self.device = device
        self.timeout = datetime.timedelta(seconds=timeout_s)
        self.transport_kind = transport
        self.peer_capacity = peer_capacity
        self.peer_timeout_ms = peer_timeout_ms
        self.init_world1 = init_world1
        self.current: Optional[Membership] = None
        self.transport = None               # PeerAllReduce of the current generation (peer mode)
        self._retired: list = []            # previous generations' buffers, kept mapped a while: a peer that
                                            # has not noticed the regroup yet may still touch them
        self._lock = threading.Lock()
        self.generations_joined = 0

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
            if m.world > 1 or (self.init_world1 and self.transport_kind == "dist"):
                store = dist.TCPStore(m.store_host, m.store_port, world_size=None, is_master=False,
                                      timeout=self.timeout, wait_for_workers=False)
                pstore = dist.PrefixStore(f"fedmi/gen{m.generation}", store)
                if self.transport_kind == "peer":
                    from .peer import PeerAllReduce

                    if self.peer_capacity <= 0:
                        raise ValueError("peer transport needs peer_capacity > 0")
                    self.transport = PeerAllReduce(m.rank, m.world, self.peer_capacity, pstore,
                                                   tag=f"gen{m.generation}", timeout_ms=self.peer_timeout_ms,
                                                   device=self.device)
                else:
                    kw = {}
                    if self.backend == "nccl" and self.device is not None:
                        kw["device_id"] = self.device
                    dist.init_process_group(self.backend, store=pstore, rank=m.rank, world_size=m.world,
                                            timeout=self.timeout, **kw)
            self.current = m
            self.generations_joined += 1
            return True

    def interrupt(self) -> None:
        """Called WITHOUT the agent lock when a newer generation arrives while an old round is
        still blocked in a collective: abort the RCCL communicator so that round fails fast.
        (Peer collectives need nothing: their barriers time out on their own.)"""
        if self.transport_kind == "dist" and dist.is_initialized() and self.backend == "nccl":
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
