"""Elastic data-plane membership for gRPC-driven clients.

The coordinator tells each live client its (rank, world) in ``TrainRequest``
(reference semantics, src/server.py:54) plus, in gRPC metadata, a membership
*generation* and the address of a rendezvous ``TCPStore`` it hosts.  A client
whose (generation, rank, world) changed tears down its communicator and joins
a fresh one under a generation-prefixed store namespace, so a dead or
rejoining client never wedges the survivors' all-reduce (reference quirks
A5/A6: world counted dead clients, stale files were averaged).

On GPUs the backend is ``nccl`` (RCCL over xGMI); on CPU hosts ``gloo``.
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


class GroupManager:
    def __init__(self, backend: str, device: Optional[torch.device] = None, timeout_s: float = 60.0):
        self.backend = backend
        self.device = device
        self.timeout = datetime.timedelta(seconds=timeout_s)
        self.current: Optional[Membership] = None
        self._lock = threading.Lock()

    def _destroy(self) -> None:
        if dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:  # pragma: no cover - best effort on a broken communicator
                pass
        self.current = None

    def ensure(self, m: Membership) -> None:
        """Join (or re-join) the data-plane group described by ``m``."""
        with self._lock:
            if self.current == m and (m.world == 1 or dist.is_initialized()):
                return
            self._destroy()
            if m.world > 1:
                store = dist.TCPStore(m.store_host, m.store_port, world_size=None, is_master=False,
                                      timeout=self.timeout, wait_for_workers=False)
                pstore = dist.PrefixStore(f"fedmi/gen{m.generation}", store)
                kw = {}
                if self.backend == "nccl" and self.device is not None:
                    kw["device_id"] = self.device
                dist.init_process_group(self.backend, store=pstore, rank=m.rank, world_size=m.world,
                                        timeout=self.timeout, **kw)
            self.current = m

    def shutdown(self) -> None:
        with self._lock:
            self._destroy()


class StoreHost:
    """Rendezvous TCPStore hosted by the (acting) coordinator."""

    def __init__(self, host: str = "127.0.0.1", port: int = 0, timeout_s: float = 60.0):
        self.store = dist.TCPStore(host, port, world_size=None, is_master=True,
                                   timeout=datetime.timedelta(seconds=timeout_s), wait_for_workers=False)
        self.host = host
        self.port = self.store.port
