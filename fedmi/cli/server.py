"""Coordinator process: ``python -m fedmi.cli.server --p y|n ...``.

Reference-compatible flags (src/server.py:268-301): ``-c/--compressFlag Y``,
``--p y`` (primary; anything else = backup), ``--backupAddress``,
``--backupPort``.  The reference hard-codes the client list, 20 rounds, the
heartbeat periods and the mount dirs; here they are flags with the
reference's values as defaults.
"""
from __future__ import annotations

import argparse
import signal
import sys
import threading

from ..control.coordinator import Coordinator, CoordinatorConfig
from ..control.roles import BackupServer, PrimaryPinger, serve_backup
from ..utils.metrics import MetricsLog, log


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description="fedmi coordinator (primary or hot-standby backup)")
    ap.add_argument("-c", "--compressFlag", help="'Y': gzip the gRPC control channel (+ clients compress updates)")
    ap.add_argument("--p", default="n", help="'y' = primary, otherwise backup")
    ap.add_argument("--backupAddress", default="localhost")
    ap.add_argument("--backupPort", default="8080")
    ap.add_argument("--clients", default="localhost:50051,localhost:50052",
                    help="comma-separated client addresses (reference: hard-coded two)")
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--agg", default="collective", choices=["collective", "grpc"],
                    help="collective = RCCL all-reduce among clients; grpc = reference parameter server")
    ap.add_argument("--root", default=".", help="directory holding Primary/ and Backup/")
    ap.add_argument("--heartbeat", type=float, default=1.0, help="ping / rejoin-probe period (s)")
    ap.add_argument("--watchdog", type=float, default=3.0, help="backup promotes after this much ping silence (s)")
    ap.add_argument("--startup-grace", type=float, default=None,
                    help="before the first primary ping: promote only after this much silence (default max(10, 5*watchdog))")
    ap.add_argument("--train-timeout", type=float, default=600.0)
    ap.add_argument("--rpc-timeout", type=float, default=30.0)
    ap.add_argument("--store-host", default="127.0.0.1")
    ap.add_argument("--store-port", type=int, default=0)
    ap.add_argument("--min-clients", type=int, default=1)
    ap.add_argument("--metrics", default=None, help="JSONL metrics file")
    ap.add_argument("--ckpt-fetch-interval", type=float, default=0.05,
                    help="collective mode: pull rank 0's newest checkpoint in the background at most this often "
                         "(s) instead of inside every StartTrain reply; <= 0: upload in every reply")
    ap.add_argument("--ckpt-sync-every", type=int, default=0,
                    help="rank 0 uploads THAT round's checkpoint every k rounds (0: pipelined by one round, "
                         "synchronous on the final round)")
    ap.add_argument("--lease", type=int, default=64,
                    help="collective mode: at most this many rounds per StartTrain (round lease; the gRPC round trip "
                         "is paid once per lease); 1 = one StartTrain per round like the reference")
    ap.add_argument("--lease-s", type=float, default=0.25,
                    help="target duration of one lease (s): the lease length follows the measured round time "
                         "(fast rounds: long leases; rounds slower than this: one round per StartTrain); 0 = always "
                         "--lease rounds")
    return ap


def main(argv=None) -> int:
    a = build_parser().parse_args(argv)
    gzip = a.compressFlag == "Y"
    log("server", f"Compression {a.compressFlag} enabled")
    cfg = CoordinatorConfig(clients=[c for c in a.clients.split(",") if c], rounds=a.rounds, agg=a.agg, gzip=gzip,
                            root=a.root, primary=(a.p == "y"), train_timeout_s=a.train_timeout,
                            rpc_timeout_s=a.rpc_timeout, heartbeat_s=a.heartbeat, store_host=a.store_host,
                            store_port=a.store_port, min_clients=a.min_clients, ckpt_sync_every=a.ckpt_sync_every,
                            ckpt_fetch_interval_s=a.ckpt_fetch_interval, lease_rounds=max(1, a.lease),
                            lease_s=max(0.0, a.lease_s),
                            backup_address=f"{a.backupAddress}:{a.backupPort}")
    metrics = MetricsLog(a.metrics)
    stop = threading.Event()

    def _sig(signum, frame):
        stop.set()

    signal.signal(signal.SIGTERM, _sig)
    signal.signal(signal.SIGINT, _sig)

    if a.p == "y":
        log("server", "Primary triggered")
        pinger = PrimaryPinger(cfg.backup_address, interval_s=a.heartbeat, timeout_s=max(1.0, 2 * a.heartbeat))
        pinger.start()
        coord = Coordinator(cfg, metrics=metrics, role="primary")
        t = threading.Thread(target=coord.run, name="fedmi-primary", daemon=True)
        t.start()
        while t.is_alive() and not stop.is_set():
            t.join(timeout=0.5)
        coord.stop()
        t.join(timeout=cfg.train_timeout_s)
        coord.close()
        pinger.stop()
        return 0
    log("server", "Backup triggered")
    backup = BackupServer(cfg, watchdog_s=a.watchdog, metrics=metrics, startup_grace_s=a.startup_grace)
    server, port = serve_backup(backup, a.backupPort)
    log("server", f"backup serving on :{port}")
    while not stop.is_set():
        stop.wait(0.5)
    backup.stop()
    server.stop(grace=1.0)
    return 0


if __name__ == "__main__":
    sys.exit(main())
