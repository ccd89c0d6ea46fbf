"""Primary / backup coordinator roles and failover.

Reference (src/server.py:181-264):
  * primary pings the backup every 1 s with CheckIfPrimaryUp(req=recovering),
  * backup serves SendModel (replica -> Backup/optimizedModel.pth) and
    CheckIfPrimaryUp; a 10 s watchdog SIGUSR1s itself and runs ``run()`` INSIDE
    the signal handler when pings stop (13.7 s measured takeover);
  * a recovering primary's first ping carries "1" and the backup demotes —
    which crashes in the reference (``Thread.terminate``, quirk A2) and leaves
    the restarted primary hung on an RPC without deadline (A3).

fedmi keeps the same RPCs and message contents but runs the role switch as an
explicit state machine on a thread: promotion starts a Coordinator (mount
Backup/, resuming from the replicated round), demotion stops it cleanly and
goes back to serving the replica.  Deadline-based watchdog (default 3 s) and
term fencing (the newer coordinator wins at the clients).
"""
from __future__ import annotations

import threading
import time
from dataclasses import replace
from typing import Optional

import grpc

from .. import ckpt as ck
from ..utils.metrics import MetricsLog, log
from ..wire import proto as P
from .coordinator import Coordinator, CoordinatorConfig


class BackupServer(P.TrainerServicer):
    """Hot standby: replica store + primary watchdog + promotion/demotion."""

    def __init__(self, cfg: CoordinatorConfig, watchdog_s: float = 3.0, metrics: Optional[MetricsLog] = None,
                 startup_grace_s: Optional[float] = None):
        self.cfg = replace(cfg, primary=False, backup_address=None)
        self.watchdog_s = watchdog_s
        # Until the first ping of a primary arrives, silence only means "not started yet" (a primary
        # process can take seconds to come up): promote only after this longer grace period.
        self.startup_grace_s = startup_grace_s if startup_grace_s is not None else max(10.0, 5 * watchdog_s)
        self.metrics = metrics or MetricsLog()
        self.mount = ck.mount_dir(cfg.root, primary=False)
        self._lock = threading.Lock()
        self.last_ping = time.monotonic()
        self.primary_seen = False
        self.coordinator: Optional[Coordinator] = None
        self._coord_thread: Optional[threading.Thread] = None
        self.promotions = 0
        self.demotions = 0
        self.promoted_at: Optional[float] = None
        self._stop = threading.Event()
        self._watch = threading.Thread(target=self._watchdog, name="fedmi-watchdog", daemon=True)

    def start(self) -> None:
        self._watch.start()

    def _log(self, msg: str) -> None:
        log("backup", msg)

    @property
    def is_acting_primary(self) -> bool:
        return self.coordinator is not None

    # ---- RPCs -----------------------------------------------------------------------
    def SendModel(self, request, context):
        data = ck.from_b64(request.model)
        ck.atomic_write(self.mount / ck.OPTIMIZED_MODEL, data)
        return P.SendModelReply(reply="success")

    def CheckIfPrimaryUp(self, request, context):
        with self._lock:
            self.last_ping = time.monotonic()
            first = not self.primary_seen
            self.primary_seen = True
            demote = request.req == "1" and self.coordinator is not None
        if first:
            self.metrics.write(role="backup", event="primary_seen")
        if demote:
            self._log("primary is back (recovering=1): stepping down")
            threading.Thread(target=self.demote, name="fedmi-demote", daemon=True).start()
        return P.PingResponse(value=1)

    def HeartBeat(self, request, context):
        return P.HeartBeatResponse(status=1)

    # ---- role state machine ------------------------------------------------------------
    def _watchdog(self) -> None:
        period = max(0.05, self.watchdog_s / 10)
        while not self._stop.wait(period):
            with self._lock:
                silent = time.monotonic() - self.last_ping
                limit = self.watchdog_s if self.primary_seen else self.startup_grace_s
                should = self.coordinator is None and silent > limit
            if should:
                self._log(f"no ping from primary for {silent:.2f}s: promoting to primary")
                self.promote()

    def promote(self) -> None:
        with self._lock:
            if self.coordinator is not None:
                return
            coord = Coordinator(self.cfg, metrics=self.metrics, role="backup-as-primary")
            self.coordinator = coord
            self.promotions += 1
            self.promoted_at = time.time()
        self.metrics.write(role="backup", event="promoted", round=coord.round)
        self._coord_thread = threading.Thread(target=coord.run, name="fedmi-backup-coordinator", daemon=True)
        self._coord_thread.start()

    def demote(self) -> None:
        with self._lock:
            coord, self.coordinator = self.coordinator, None
            self.last_ping = time.monotonic()
        if coord is None:
            return
        coord.stop()
        if self._coord_thread is not None:
            self._coord_thread.join(timeout=self.cfg.train_timeout_s)
        coord.close()
        self.demotions += 1
        self.metrics.write(role="backup", event="demoted", round=coord.round)
        self._log("back to standby")

    def stop(self) -> None:
        self._stop.set()
        self.demote()


class PrimaryPinger:
    """Primary -> backup liveness pings (src/server.py:188-200), with deadlines.

    ``recovering`` is "1" until the first SUCCESSFUL ping after (re)start, so a
    promoted backup always learns that the primary is back.
    """

    def __init__(self, backup_address: str, interval_s: float = 1.0, timeout_s: float = 2.0):
        self.stub = P.TrainerStub(P.make_channel(backup_address))
        self.interval = interval_s
        self.timeout = timeout_s
        self.recovering = 1
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, name="fedmi-pinger", daemon=True)

    def start(self) -> None:
        self._t.start()

    def _run(self) -> None:
        while not self._stop.is_set():
            try:
                self.stub.CheckIfPrimaryUp(P.PingRequest(req=str(self.recovering)), timeout=self.timeout)
                self.recovering = 0
            except grpc.RpcError:
                pass
            self._stop.wait(self.interval)

    def stop(self) -> None:
        self._stop.set()


def serve_backup(backup: BackupServer, port: int | str, max_workers: int = 10):
    server = P.make_server(max_workers=max_workers)
    P.add_TrainerServicer_to_server(backup, server)
    bound = server.add_insecure_port(f"[::]:{port}")
    if bound == 0:
        raise RuntimeError(f"backup could not bind port {port}")
    server.start()
    backup.start()
    return server, bound
