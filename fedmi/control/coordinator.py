"""Coordinator: drives federated rounds over the ``federated.Trainer`` RPCs.

Reference: ``run()`` / ``trainThreadFunc`` / ``allreduce()`` /
``sendOptimizedModel`` / ``checkClientStatus`` in src/server.py:51-179.

Per round (synchronous, one local epoch per client, like the reference):
  live clients get StartTrain(rank=i, world=#live) in parallel, with a deadline;
  * ``agg="collective"``: clients all-reduce among themselves (RCCL); the
    coordinator persists rank 0's averaged checkpoint;
  * ``agg="grpc"``: reference parameter-server path — replies are written to
    ``<mount>/test_<rank>.pth``, averaged (only the replies of THIS round), the
    result saved and SendModel'ed back.
  ``<mount>/optimizedModel.pth`` is written and replicated to the backup by a
  background thread (in order), off the round's critical path.  In collective
  mode rank 0's upload is pipelined by one round except on the final round.
  A collective round that lost a client is aborted: the survivors are rolled
  back to the last committed global model (SendModel) before regrouping.

Fixes vs the reference: deadlines on every RPC (A3),
world = live clients only and no stale-file averaging (A5/A6), the round is
persisted in the checkpoint's ``epoch`` and resumed (A8), a lock-guarded
membership table (races in §5.2), a monotonic *term* sent as metadata so
clients fence off a stale coordinator (split brain), and the rejoin tracker
is a daemon thread that stops with the coordinator.
"""
from __future__ import annotations

import concurrent.futures as cf
import json
import threading
import time
from collections import OrderedDict
from dataclasses import dataclass, field
from pathlib import Path
from typing import Dict, List, Optional

import grpc
import torch

from .. import ckpt as ck
from ..parallel.group import StoreHost
from ..utils.metrics import MetricsLog, Timer, log
from ..utils.trace import phase
from ..wire import proto as P
from .client_agent import (META_FETCH, META_GEN, META_HAVE, META_LEASE, META_ROUND, META_STORE, META_SYNC, META_TERM,
                           META_UPLOAD)


@dataclass
class CoordinatorConfig:
    clients: List[str] = field(default_factory=lambda: ["localhost:50051", "localhost:50052"])
    rounds: int = 20                     # src/server.py:120
    agg: str = "collective"              # "collective" (RCCL among clients) | "grpc" (reference)
    gzip: bool = False                   # -c Y on the control channel (src/server.py:103-107)
    root: str = "."
    primary: bool = True                 # mount dir Primary/ vs Backup/
    train_timeout_s: float = 600.0
    rpc_timeout_s: float = 30.0
    heartbeat_s: float = 1.0             # rejoin probe period (src/server.py:81)
    store_host: str = "127.0.0.1"
    store_port: int = 0
    backup_address: Optional[str] = None
    min_clients: int = 1
    round_pause_s: float = 0.0
    ckpt_sync_every: int = 0             # >0: rank 0 uploads THAT round's checkpoint every k rounds (always the last)
    # collective mode with fedmi clients: the per-round model upload leaves the StartTrain reply and a
    # background fetcher pulls rank 0's newest checkpoint at most this often (<= 0: upload every reply)
    ckpt_fetch_interval_s: float = 0.05
    # collective mode: one StartTrain runs up to this many consecutive rounds on the clients (x-fedmi-lease), so
    # the fan-out / gather round trip is paid once per lease; 1 = one RPC per round (the reference's cadence;
    # always the case for agg="grpc")
    lease_rounds: int = 64
    # target duration of one lease (s): the lease length follows the measured round time, so fast rounds
    # (LeNet, ~10 ms) amortise the round trip over ~25 rounds while slow rounds (ResNet-18, ~0.9 s) keep one
    # StartTrain per round and the coordinator reacts to joins / failures at that cadence.  The first lease is
    # one round (the round time is not known yet).  0: always lease_rounds
    lease_s: float = 0.25


def fedavg_state_dicts(sds: List[dict], weights: Optional[List[float]] = None) -> "OrderedDict[str, torch.Tensor]":
    """Uniform (or weighted) average of every entry (reference src/server.py:163-171).

    Integer buffers stay integer: floor of the mean, which equals the
    reference's float mean truncated back to int64 on load.
    """
    if not sds:
        raise ValueError("no state dicts to average")
    n = len(sds)
    w = weights or [1.0 / n] * n
    out = OrderedDict()
    for k in sds[0]:
        vals = [sd[k] for sd in sds]
        if vals[0].is_floating_point():
            acc = torch.zeros_like(vals[0], dtype=torch.float32)
            for wi, v in zip(w, vals):
                acc.add_(v.float(), alpha=wi)
            out[k] = acc.to(vals[0].dtype)
        else:
            out[k] = torch.div(sum(v.long() for v in vals), n, rounding_mode="floor").to(vals[0].dtype)
    return out


class _Member:
    __slots__ = ("address", "active", "channel", "stub", "fedmi")

    def __init__(self, address: str, gzip: bool):
        self.address = address
        self.active = True
        self.fedmi = False          # answered with fedmi trailing metadata: understands upload/fetch
        self.channel = P.make_channel(address, gzip=gzip)
        self.stub = P.TrainerStub(self.channel)

    def reconnect(self, gzip: bool) -> None:
        try:
            self.channel.close()
        except Exception:
            pass
        self.channel = P.make_channel(self.address, gzip=gzip)
        self.stub = P.TrainerStub(self.channel)


class Coordinator:
    def __init__(self, cfg: CoordinatorConfig, metrics: Optional[MetricsLog] = None, role: str = "primary",
                 term: Optional[int] = None):
        self.cfg = cfg
        self.role = role
        self.metrics = metrics or MetricsLog()
        self.term = term if term is not None else time.time_ns()
        self.mount = ck.mount_dir(cfg.root, cfg.primary)
        self.model_path = self.mount / ck.OPTIMIZED_MODEL
        self._lock = threading.Lock()
        self.members: "OrderedDict[str, _Member]" = OrderedDict((a, _Member(a, cfg.gzip)) for a in cfg.clients)
        self.stop_event = threading.Event()
        self.generation = 0
        self._last_live: Optional[tuple] = None
        self.round = ck.read_epoch(self.model_path) or 0          # resume (quirk A8)
        self.latest_model: Optional[bytes] = self.model_path.read_bytes() if self.model_path.exists() else None
        self.store = StoreHost(cfg.store_host, cfg.store_port) if cfg.agg == "collective" else None
        self._pool = cf.ThreadPoolExecutor(max_workers=max(4, 2 * len(self.members)), thread_name_prefix="fedmi-rpc")
        self._backup = None
        if cfg.backup_address:
            self._backup = P.TrainerStub(P.make_channel(cfg.backup_address))
        self._tracker: Optional[threading.Thread] = None
        self.round_times: List[float] = []
        self._round_s: Optional[float] = None     # smoothed seconds per round (sizes the lease, cfg.lease_s)
        self.installed_epoch = ck.read_epoch(self.model_path) or -1
        self._persist_cv = threading.Condition()
        self._to_persist: Optional[bytes] = None
        self._persist_seq = 0
        self._persisted_seq = 0
        self._persist_stop = False
        self._persist_thread = threading.Thread(target=self._persister, name="fedmi-persist", daemon=True)
        self._persist_thread.start()
        self._fetch_thread: Optional[threading.Thread] = None
        self._fetches = 0
        self._lease_end = 0                  # last round of the StartTrain lease in flight (0: none)
        if cfg.agg == "collective" and cfg.ckpt_fetch_interval_s > 0:
            self._fetch_thread = threading.Thread(target=self._fetcher, name="fedmi-fetch", daemon=True)
            self._fetch_thread.start()

    # ---- logging / membership -------------------------------------------------
    def _log(self, msg: str) -> None:
        log(f"{self.role} coordinator", msg)

    def live(self) -> List[str]:
        with self._lock:
            return [a for a, m in self.members.items() if m.active]

    def _mark(self, address: str, active: bool) -> None:
        with self._lock:
            m = self.members.get(address)
            if m is not None and m.active != active:
                m.active = active
                self._log(f"client {address} -> {'active' if active else 'INACTIVE'}")

    def client_status(self) -> Dict[str, bool]:
        with self._lock:
            return {a: m.active for a, m in self.members.items()}

    def _lease(self, rnd: int) -> int:
        """Rounds the next StartTrain covers: the configured lease, never past the last round, and ending on
        a ``ckpt_sync_every`` boundary (those rounds upload their own checkpoint)."""
        if self.cfg.agg != "collective":
            return 1
        k = int(self.cfg.lease_rounds)
        if self.cfg.lease_s > 0:
            k = 1 if self._round_s is None else min(k, max(1, int(self.cfg.lease_s / max(self._round_s, 1e-6))))
        k = max(1, min(k, self.cfg.rounds - rnd + 1))
        if self.cfg.ckpt_sync_every > 0:
            k = min(k, self.cfg.ckpt_sync_every - (rnd - 1) % self.cfg.ckpt_sync_every)
        return k

    def _meta(self, round_no: int, live: List[str], lease: int = 1):
        md = [(META_TERM, str(self.term)), (META_ROUND, str(round_no)), (META_GEN, str(self.generation))]
        if lease > 1:
            md.append((META_LEASE, str(lease)))
        k = self.cfg.ckpt_sync_every
        end = round_no + lease - 1
        sync = end >= self.cfg.rounds or (k > 0 and end % k == 0)
        if sync:
            md.append((META_SYNC, "1"))
        elif (self._fetch_thread is not None and live and self.members[live[0]].fedmi):
            md.append((META_UPLOAD, "0"))           # rank 0's model is fetched off the critical path
        if self.store is not None:
            md.append((META_STORE, f"{self.store.host}:{self.store.port}"))
        return md

    # ---- model persistence / replication --------------------------------------
    def _install_global(self, data: bytes, epoch: Optional[int] = None) -> None:
        if epoch is not None and epoch <= self.installed_epoch:
            return
        self.latest_model = data
        if epoch is not None:
            self.installed_epoch = epoch
        with self._persist_cv:
            self._to_persist = data            # coalesced: only the newest model is written/replicated
            self._persist_seq += 1
            self._persist_cv.notify()

    def _persister(self) -> None:
        """Writes ``<mount>/optimizedModel.pth`` and replicates it to the backup, newest model first.

        Rounds can outpace a slow disk or backup link: intermediate models are skipped
        (bounded memory, minimal lag) instead of queueing every round's checkpoint."""
        while True:
            with self._persist_cv:
                while self._to_persist is None and not self._persist_stop:
                    self._persist_cv.wait()
                if self._to_persist is None:
                    return
                data, seq = self._to_persist, self._persist_seq
                self._to_persist = None
            ck.atomic_write(self.model_path, data)
            if self._backup is not None:
                try:
                    self._backup.SendModel(P.SendModelRequest(model=ck.to_b64(data)),
                                           timeout=self.cfg.rpc_timeout_s, metadata=[(META_TERM, str(self.term))])
                except grpc.RpcError as e:
                    self._log(f"backup replication failed: {e.code().name}")
            with self._persist_cv:
                self._persisted_seq = seq
                self._persist_cv.notify_all()

    def _fetcher(self) -> None:
        """Pull rank 0's newest checkpoint (SendModel + x-fedmi-fetch) whenever rounds moved past the
        installed model, at most every ``ckpt_fetch_interval_s``: persistence and backup replication
        without a model upload inside each StartTrain reply."""
        while not self.stop_event.wait(self.cfg.ckpt_fetch_interval_s):
            live = self.live()
            behind = self.round > self.installed_epoch or self._lease_end > max(self.round, self.installed_epoch)
            if not live or not behind or not self.members[live[0]].fedmi:
                continue
            m = self.members[live[0]]
            try:
                call = m.stub.SendModel.with_call(P.SendModelRequest(model=""), timeout=self.cfg.rpc_timeout_s,
                                                  metadata=[(META_TERM, str(self.term)), (META_FETCH, "1"),
                                                            (META_HAVE, str(self.installed_epoch))])
            except grpc.RpcError:
                continue                     # membership changes are the round loop's business
            reply, call = call
            epoch = int(dict(call.trailing_metadata() or ()).get("x-fedmi-ckpt-epoch", "-1"))
            if reply.reply and epoch > self.installed_epoch:
                self._fetches += 1
                self._install_global(ck.from_b64(reply.reply), epoch)

    def _catch_up_committed(self, addr: str, target: Optional[int] = None, wait_s: float = 2.0) -> None:
        """Synchronously pull the newest COMMITTED global model from ``addr`` (the aborted round's rank 0,
        which keeps the checkpoint of its last successful round) until it covers ``target`` (the round rank 0
        reported as committed in its ABORTED trailer; default ``self.round``): the background fetcher may be
        several rounds behind.  A model newer than ``self.round`` -- rounds of a lease that completed their
        all-reduce before the failure, or an aborted round whose all-reduce had finished on rank 0 -- is a
        full FedAvg result and becomes the committed round: the round counter follows it (otherwise the next
        round would report that epoch again and _install_global would drop it as not newer).  Best effort:
        an unreachable rank 0 leaves ``latest_model`` as it is."""
        m = self.members.get(addr)
        if m is None or not m.fedmi or self.cfg.agg != "collective":
            return
        want = self.round if target is None else max(self.round, int(target))
        deadline = time.monotonic() + wait_s
        while self.installed_epoch < want and time.monotonic() < deadline:
            try:
                reply, call = m.stub.SendModel.with_call(
                    P.SendModelRequest(model=""), timeout=self.cfg.rpc_timeout_s,
                    metadata=[(META_TERM, str(self.term)), (META_FETCH, "1"), (META_HAVE, str(self.installed_epoch))])
            except grpc.RpcError:
                break
            epoch = int(dict(call.trailing_metadata() or ()).get("x-fedmi-ckpt-epoch", "-1"))
            if reply.reply and epoch > self.installed_epoch:
                self._install_global(ck.from_b64(reply.reply), epoch)
            else:
                time.sleep(0.02)             # its writer is still serialising the committed round
        if self.installed_epoch > self.round:
            self._log(f"rank 0 committed round {self.installed_epoch} before the abort: advancing the round counter")
            self.round = self.installed_epoch

    def flush(self) -> None:
        """Wait until the newest installed model is on disk (and offered to the backup)."""
        with self._persist_cv:
            target = self._persist_seq
            while self._persisted_seq < target and self._persist_thread.is_alive():
                self._persist_cv.wait(timeout=1.0)

    def _send_model(self, address: str, data_b64: str) -> bool:
        m = self.members[address]
        try:
            m.stub.SendModel(P.SendModelRequest(model=data_b64), timeout=self.cfg.train_timeout_s,
                             metadata=[(META_TERM, str(self.term))])
            return True
        except grpc.RpcError as e:
            self._log(f"SendModel to {address} failed: {e.code().name}")
            self._mark(address, False)
            return False

    # ---- one round ------------------------------------------------------------------
    def run_round(self) -> bool:
        with phase("coordinator-round"):
            return self._run_round()

    def _run_round(self) -> bool:
        live = self.live()
        if len(live) < max(1, self.cfg.min_clients):
            time.sleep(self.cfg.heartbeat_s)
            return False
        if tuple(live) != self._last_live:
            self.generation += 1                      # new data-plane group for a new member set
            self._last_live = tuple(live)
        world = len(live)
        rnd = self.round + 1
        lease = self._lease(rnd)
        end = rnd + lease - 1
        self._log(f"Starting round {rnd}" + (f"-{end}" if lease > 1 else "")
                  + f" with {world} client(s) (gen {self.generation})")
        t = Timer()
        md = self._meta(rnd, live, lease)
        t_send = time.time()
        self._lease_end = end
        futs = {}
        timeout = self._train_deadline(lease)
        gen = self.generation
        # blocking unary calls on the coordinator's pool (a grpc ``.future()`` call starts a channel spin thread
        # per call: ~1 ms per client per round on the control plane)
        for rank, addr in enumerate(live):
            stub = self.members[addr].stub
            f = self._pool.submit(stub.StartTrain.with_call, P.TrainRequest(rank=rank, world=world),
                                  timeout=timeout, metadata=md)
            if world > 1 and self.store is not None:
                f.add_done_callback(lambda f_, a_=addr: self._propagate_loss(f_, a_, gen))
            futs[addr] = (rank, f)
        replies, failed, client_rounds, ckpt_epochs, lease_stats, committed, ok_rounds = {}, [], [], {}, None, {}, {}
        for addr, (rank, f) in futs.items():
            try:
                reply, call = f.result()
                replies[rank] = reply.message
                tm = dict(call.trailing_metadata() or ())
                if "x-fedmi-client-round" in tm:
                    client_rounds.append(int(tm["x-fedmi-client-round"]))
                    ok_rounds[rank] = int(tm["x-fedmi-client-round"])
                    self.members[addr].fedmi = True
                if "x-fedmi-ckpt-epoch" in tm:
                    ckpt_epochs[rank] = int(tm["x-fedmi-ckpt-epoch"])
                if rank == 0 and "x-fedmi-lease-stats" in tm:
                    lease_stats = tm["x-fedmi-lease-stats"]
            except grpc.RpcError as e:
                self._log(f"StartTrain on {addr} failed: {e.code().name} {e.details() or ''}".strip())
                failed.append(addr)
                try:   # an aborted lease reports the rounds it committed before the failure
                    tm = dict(e.trailing_metadata() or ())
                    if "x-fedmi-client-round" in tm:
                        committed[rank] = int(tm["x-fedmi-client-round"])
                        self.members[addr].fedmi = True      # a fedmi client (it serves the fetch path)
                    if rank == 0 and "x-fedmi-lease-stats" in tm:
                        lease_stats = tm["x-fedmi-lease-stats"]
                except Exception:
                    pass
                # ABORTED / FAILED_PRECONDITION: the client answered (its collective lost a peer, or it
                # fenced us); only an unreachable or silent client leaves the membership
                if e.code() not in (grpc.StatusCode.ABORTED, grpc.StatusCode.FAILED_PRECONDITION):
                    self._mark(addr, False)
        self._lease_end = 0
        t_train = t.ms()
        t_recv = time.time()
        ok = False
        if self.cfg.agg == "collective":
            if failed:
                # the survivors' all-reduce for this round is not trustworthy: roll them back to the
                # last committed global model, then regroup (new generation) next round.  Lease rounds that
                # completed before the failure stay committed (rank 0 checkpointed them).
                self._log(f"round {rnd} aborted ({len(failed)} client(s) lost); rolling back survivors, regrouping")
                self._last_live = None           # force a new generation even if every member answered ABORTED
                target = committed.get(0)
                if 0 in replies:
                    # rank 0 finished the whole call: every round it ran completed its all-reduce (all members
                    # contributed), so they are committed even though another rank failed afterwards
                    target = ok_rounds.get(0, end)
                    if replies[0]:
                        self._install_global(ck.from_b64(replies[0]), ckpt_epochs.get(0, target))
                self._catch_up_committed(live[0], target)
                if self.latest_model is not None:
                    if self.installed_epoch >= 0 and self.installed_epoch < self.round:
                        # rank 0's newest committed round was not reachable: the round counter follows
                        # the model the survivors are rolled back to
                        self._log(f"rewinding round {self.round} -> {self.installed_epoch} (newest committed model)")
                        self.round = self.installed_epoch
                    b64 = ck.to_b64(self.latest_model)
                    # EVERY member still active -- the ones that answered ABORTED too: their model may be
                    # partially averaged (peer blocks past the barrier wrote the mean in place)
                    with self._lock:
                        targets = [a for a in live if self.members[a].active]
                    self.metrics.write(role=self.role, event="rollback", round=rnd, epoch=self.installed_epoch,
                                       targets=targets, state_sum=ck.state_digest(ck.from_bytes(self.latest_model)["net"]))
                    sends = [self._pool.submit(self._send_model, a, b64) for a in targets]
                    for s_ in sends:
                        s_.result()
            else:
                msg = replies.get(0, "")
                if msg:
                    self._install_global(ck.from_b64(msg), ckpt_epochs.get(0, end))
                ok = True
        else:
            good = {r: ck.from_b64(m) for r, m in replies.items() if m}
            if good:
                for r, data in good.items():
                    ck.atomic_write(self.mount / f"test_{r}.pth", data)
                sds = [ck.from_bytes(d)["net"] for d in good.values()]
                avg = fedavg_state_dicts(sds)
                data = ck.to_bytes(ck.make_checkpoint(avg, acc=1, epoch=rnd))
                self._install_global(data, rnd)
                b64 = ck.to_b64(data)
                sends = [self._pool.submit(self._send_model, a, b64) for a in live if a not in failed]
                for s_ in sends:
                    s_.result()
                ok = True
        if ok:
            self.round = max([end] + client_rounds)
        dt = t.ms()
        self.round_times.append(dt / lease)
        if ok:   # per-round wall time (the lease length follows it): a faster round is taken at once (the first
            # rounds carry group setup and warm-up), a slower one is smoothed in
            per_s = dt / lease / 1e3
            self._round_s = (per_s if self._round_s is None or per_s < self._round_s
                             else 0.7 * self._round_s + 0.3 * per_s)
        t_done = time.time()
        if ok:
            per = [(r_, True, lo, ac, tr_) for r_, lo, ac, tr_ in self._lease_rows(lease_stats, rnd, end)]
        else:
            # an aborted lease: the rounds before the failure are committed (the round counter now covers them),
            # the failing round is the one after them
            # (rows with rank 0's stats only: a committed round this call did not run -- a client fencing a new
            # term off rounds it committed under the previous one -- is not this coordinator's round)
            done = [row for row in self._lease_rows(lease_stats, rnd, self.round)
                    if row[0] <= self.round and row[1] is not None]
            per = [(r_, True, lo, ac, tr_) for r_, lo, ac, tr_ in done]
            per.append((max(rnd, self.round + 1), False, None, None, t_done))
        for r_, ok_r, loss, acc, t_r in per:
            self.metrics.write(role=self.role, event="round", round=r_, ok=ok_r, world=world, generation=self.generation,
                               failed=[] if ok_r else failed, train_ms=t_train / lease, round_ms=dt / lease,
                               term=self.term, t_send=t_send, t_recv=t_recv, t_done=t_done, lease=lease, t_round=t_r,
                               **({"train_loss": loss, "test_acc": acc} if loss is not None else {}))
        if self.cfg.round_pause_s:
            time.sleep(self.cfg.round_pause_s)
        return ok

    @staticmethod
    def _lease_rows(raw: Optional[str], rnd: int, end: int):
        """(round, train_loss, test_acc, t_done) per round of a lease from rank 0's x-fedmi-lease-stats
        trailer (reference peers send none: one row per round with no stats)."""
        rows = []
        if raw:
            try:
                rows = [(int(r[0]), float(r[1]), float(r[2]), float(r[3])) for r in json.loads(raw)]
            except (ValueError, TypeError, IndexError):
                rows = []
        have = {r[0] for r in rows}
        now = time.time()
        rows += [(r, None, None, now) for r in range(rnd, end + 1) if r not in have]
        return sorted(rows)

    def _train_deadline(self, lease: int) -> float:
        """StartTrain deadline: the per-round timeout plus the lease's expected run time with headroom (a
        multiple of the per-round timeout would let a stuck-but-alive client hold a lease for hours)."""
        if lease <= 1:
            return self.cfg.train_timeout_s
        if self._round_s is None:
            return self.cfg.train_timeout_s * lease
        return self.cfg.train_timeout_s + 4.0 * lease * self._round_s

    def _propagate_loss(self, f, addr: str, gen: int) -> None:
        """Done-callback of a StartTrain future: an unreachable client (not ABORTED / FAILED_PRECONDITION,
        which are answers from a live client) aborts its generation's collective on every survivor at once
        -- they would otherwise wait out the collective timeout inside the barrier (reference: the dead client
        is marked inactive at its failed RPC, src/server.py:59-62)."""
        if f.cancelled():
            return
        e = f.exception()
        if not isinstance(e, grpc.RpcError):
            return
        code = e.code() if callable(getattr(e, "code", None)) else None
        if code in (grpc.StatusCode.ABORTED, grpc.StatusCode.FAILED_PRECONDITION):
            return
        try:
            self.store.abort_generation(gen, addr)
            self.metrics.write(role=self.role, event="loss_propagated", generation=gen, client=addr,
                               code=getattr(code, "name", str(code)))
        except Exception as err:  # pragma: no cover - the store is ours; best effort
            self._log(f"could not propagate the loss of {addr}: {err!r}")

    # ---- rejoin tracker (src/server.py:78-101) --------------------------------------
    def _track(self) -> None:
        while not self.stop_event.wait(self.cfg.heartbeat_s):
            with self._lock:
                inactive = [a for a, m in self.members.items() if not m.active]
            for addr in inactive:
                m = self.members[addr]
                m.reconnect(self.cfg.gzip)
                try:
                    r = m.stub.HeartBeat(P.Request(), timeout=self.cfg.rpc_timeout_s)
                except grpc.RpcError:
                    continue
                if r.status == 1:
                    if self.latest_model is not None:
                        if not self._send_model(addr, ck.to_b64(self.latest_model)):
                            continue
                    self._mark(addr, True)

    def start_tracker(self) -> None:
        if self._tracker is None:
            self._tracker = threading.Thread(target=self._track, name="fedmi-tracker", daemon=True)
            self._tracker.start()

    # ---- lifecycle ------------------------------------------------------------------
    def run(self) -> None:
        self.start_tracker()
        self._log(f"term {self.term}, resuming at round {self.round}, clients {list(self.members)}")
        while self.round < self.cfg.rounds and not self.stop_event.is_set():
            self.run_round()
        live = self.live()
        if live and self.installed_epoch < self.round:
            # a lease ended without uploading its last round (pipelined upload, fetcher stopped): pull rank 0's
            # newest committed model so Primary/optimizedModel.pth and the backup replica cover every round run
            self._catch_up_committed(live[0], self.round)
        self._log(f"finished at round {self.round}")

    def stop(self) -> None:
        self.stop_event.set()

    def close(self) -> None:
        self.stop()
        if self._fetch_thread is not None:
            self._fetch_thread.join(timeout=self.cfg.rpc_timeout_s)
        self.flush()
        with self._persist_cv:
            self._persist_stop = True
            self._persist_cv.notify_all()
        self._persist_thread.join(timeout=30)
        self._pool.shutdown(wait=False, cancel_futures=True)
        for m in self.members.values():
            try:
                m.channel.close()
            except Exception:
                pass
