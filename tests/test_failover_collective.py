"""Primary/backup failover with COLLECTIVE FedAvg (BASELINE.json config 5): the
primary drives rounds of client processes whose FedAvg is a collective among
themselves; the primary dies mid-run, the backup promotes itself, rebuilds the
client process group under its own rendezvous store and continues from the
replicated round; the clients' checkpoints keep advancing.  The CPU variant
runs MLP clients on gloo; the GPU variant runs native-LeNet clients on the
MI355X (sharing its one GPU; their FedAvg runs through the hipIpc peer kernels)."""
import threading
import time

import pytest

from fedmi import ckpt as ck
from fedmi.control.coordinator import Coordinator, CoordinatorConfig
from fedmi.control.roles import BackupServer, PrimaryPinger, serve_backup

from helpers import free_port, spawn_client, stop_proc, wait_heartbeat


def _wait(pred, timeout=60.0, step=0.05):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if pred():
            return time.time() - t0
        time.sleep(step)
    raise TimeoutError("condition not reached")


def _run(tmp_path, device: str, model_args):
    addrs = [f"127.0.0.1:{free_port()}" for _ in range(2)]
    transport = ("--transport", "peer") if device.startswith("cuda") else ("--backend", "gloo")
    procs = [spawn_client(a, tmp_path, "--agg", "collective", *transport, *model_args,
                          log_path=tmp_path / f"client{i}.log", device=device) for i, a in enumerate(addrs)]
    try:
        for a in addrs:
            wait_heartbeat(a, timeout=100)
        bport = free_port()
        cfg = CoordinatorConfig(clients=addrs, rounds=10_000, agg="collective", root=str(tmp_path / "srv"),
                                heartbeat_s=0.1, train_timeout_s=60, rpc_timeout_s=10,
                                backup_address=f"127.0.0.1:{bport}", round_pause_s=0.05)
        backup = BackupServer(cfg, watchdog_s=1.0)
        bserver, _ = serve_backup(backup, bport)
        pinger = PrimaryPinger(cfg.backup_address, interval_s=0.1, timeout_s=2.0)
        pinger.start()
        primary = Coordinator(cfg, role="primary")
        t = threading.Thread(target=primary.run, daemon=True)
        t.start()
        _wait(lambda: primary.round >= 3)
        _wait(lambda: (tmp_path / "srv" / "Backup" / "optimizedModel.pth").exists())
        # ---- the primary dies mid-run
        pinger.stop()
        primary.stop()
        t.join(timeout=60)
        primary.close()
        r_dead = primary.round
        _wait(lambda: backup.is_acting_primary, timeout=20)
        acting = backup.coordinator
        assert acting.round >= r_dead - 1                 # resumed from the replicated round
        _wait(lambda: acting.round >= r_dead + 2, timeout=120)
        # clients followed the new coordinator: their checkpoints carry its rounds
        for a in addrs:
            _wait(lambda: (ck.read_epoch(tmp_path / "checkpoint" / f"{a}.pth") or 0) >= r_dead + 1, timeout=30)
        backup.stop()
        bserver.stop(None)
    finally:
        for p in procs:
            stop_proc(p)


@pytest.mark.slow
def test_collective_failover_cpu(tmp_path):
    _run(tmp_path, "cpu", ("--model", "mlp", "--data", "synthetic-mnist", "--n-train", "512", "--n-test", "256",
                           "--lr", "0.05"))


@pytest.mark.gpu
def test_collective_failover_gpu(tmp_path):
    _run(tmp_path, "cuda:0", ("--model", "lenet", "--n-train", "2560", "--n-test", "1000"))
