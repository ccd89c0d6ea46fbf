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
* Loss propagation: the coordinator learns of a dead client within milliseconds (its StartTrain fails with
  UNAVAILABLE) and sets ``abort`` in the generation's store namespace.  Every member runs a watchdog
  thread on that key; on it, the peer barriers fail at their next poll (host-pinned abort word), an RCCL
  communicator is aborted (``ncclCommAbort``) and a gloo collective stops waiting -- the survivors leave
  the collective at once instead of after ``timeout_s`` (reference: a dead client is dropped at its next
  failed RPC, src/server.py:59-62, 72-75).
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
import time
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


ABORT_KEY = "abort"          # per generation, under the client's "fedmi/gen<g>" store prefix
ABORT_POLL_S = 0.02


class CollectiveAborted(RuntimeError):
    """A collective was abandoned because the coordinator reported a lost client."""


def wait_work(work, abort: Optional[threading.Event], what: str = "collective") -> None:
    """Wait for an ``async_op`` collective, giving up as soon as ``abort`` is set.  Used for host-blocking
    backends (gloo): an abandoned gloo work keeps its worker thread until its own timeout, so the group
    it belongs to is detached, not destroyed (:func:`_detach_default_group`)."""
    if abort is None:
        work.wait()
        return
    while not work.is_completed():
        if abort.is_set():
            raise CollectiveAborted(f"{what} abandoned: the coordinator reported a lost client")
        time.sleep(0.0002)
    work.wait()               # completed: surfaces its error, if any


def _detach_default_group() -> bool:
    """Forget the default gloo group WITHOUT shutting it down (its destructor would join a worker thread
    still blocked on the dead peer until the gloo timeout).  The object stays referenced by the caller's
    retired list.  Private c10d state: returns False (caller destroys normally) if the layout differs."""
    c = dist.distributed_c10d
    w = getattr(c, "_world", None)
    pg = getattr(w, "default_pg", None) if w is not None else None
    if pg is None:
        return False
    try:
        for name in ("pg_map", "pg_names", "pg_group_ranks", "pg_backend_config", "pg_to_tag",
                     "pg_coalesce_state", "pg_default_device"):
            d = getattr(w, name, None)
            if isinstance(d, dict):
                d.pop(pg, None)
        tags = getattr(w, "tags_to_pg", None)
        if isinstance(tags, dict):
            for k in list(tags):
                tags[k] = [g for g in tags[k] if g is not pg]
        w.default_pg = None
    except Exception:  # pragma: no cover - torch internals moved
        return False
    return True


def abort_default_group(pending: bool = False) -> object:
    """Tear down the default process group without talking to (possibly dead) peers.  ``pending``: a gloo
    collective was abandoned on it -- detach instead of destroy.  Returns the detached group (keep it
    referenced) or None."""
    if not dist.is_initialized():
        return None
    if pending and dist.get_backend() == "gloo":
        pg = dist.distributed_c10d._get_default_group()
        if _detach_default_group():
            return pg
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
    return None


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
        # loss propagation: set by the watchdog when the coordinator reports a lost client for the current
        # generation (a fresh Event per generation; FedAvg polls it around host-blocking collectives)
        self.abort_event = threading.Event()
        self.aborts_seen = 0
        self._watch_stop: Optional[threading.Event] = None
        self._detached: list = []            # gloo groups left with an abandoned collective (never destroyed)

    def _drop(self) -> None:
        if self._watch_stop is not None:
            self._watch_stop.set()
            self._watch_stop = None
        if self.transport is not None:
            try:
                self.transport.close(barrier=False)
            except Exception:  # pragma: no cover
                pass
            self._retired = (self._retired + [self.transport])[-4:]
            self.transport = None
        pg = abort_default_group(pending=self.abort_event.is_set())
        if pg is not None:
            self._detached.append(pg)
        self.current = None
        self.abort_event = threading.Event()

    def _watch(self, m: Membership, stop: threading.Event, ev: threading.Event) -> None:
        """Watchdog of generation ``m``: its own store connection (the main thread's is not shared across
        threads), one ``check`` of the abort key every ABORT_POLL_S."""
        try:
            store = dist.TCPStore(m.store_host, m.store_port, world_size=None, is_master=False,
                                  timeout=self.timeout, wait_for_workers=False)
            pstore = dist.PrefixStore(f"fedmi/gen{m.generation}", store)
        except Exception:  # pragma: no cover - the coordinator is gone; the collective timeout still bounds us
            return
        while not stop.wait(ABORT_POLL_S):
            try:
                hit = pstore.check([ABORT_KEY])
            except Exception:
                return
            if hit:
                self._on_abort(ev)
                return

    def _on_abort(self, ev: threading.Event) -> None:
        if ev is not self.abort_event or ev.is_set():
            return                              # a later generation already replaced this one
        ev.set()
        self.aborts_seen += 1
        tp = self.transport
        if tp is not None:
            tp.request_abort()
        elif dist.is_initialized() and self.backend == "nccl":
            abort_default_group()               # ncclCommAbort: the spinning RCCL kernel exits
        # gloo: FedAvg's wait_work() sees the event and abandons the work

    def request_abort(self) -> None:
        """Abort the current generation's collectives locally (tests; the watchdog's action)."""
        self._on_abort(self.abort_event)

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
                self._watch_stop = threading.Event()
                threading.Thread(target=self._watch, args=(m, self._watch_stop, self.abort_event),
                                 name=f"fedmi-abort-watch-g{m.generation}", daemon=True).start()
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
        still blocked in a collective: that round fails fast (the same action as the abort watchdog)."""
        self._on_abort(self.abort_event)

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
        self._lock = threading.Lock()

    def abort_generation(self, generation: int, reason: str = "") -> None:
        """Tell every member of ``generation`` that a client was lost (their watchdogs abort the collective)."""
        with self._lock:
            self.store.set(f"fedmi/gen{generation}/{ABORT_KEY}", (reason or "lost").encode()[:200])
