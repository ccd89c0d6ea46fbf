"""Failover with REAL process deaths (SIGKILL), the reference's scenario
(src/server.py:219-264 backup watchdog + promotion; src/server.py:59-62,78-101
client loss and rejoin), driven through the reference-compatible entry points
``server.py`` / ``client.py`` as separate processes.

* primary SIGKILLed in the middle of the round loop -> the backup process
  promotes itself within its watchdog window and continues from the replicated
  round (reference: 13.7 s takeover, restart at round 0); the primary process is
  restarted -> the backup steps down cleanly (reference: crash, quirk A2) and the
  restarted primary resumes from its own persisted round.
* one client SIGKILLed while the other clients wait INSIDE the FedAvg collective
  (fault-injection stall right before the collective) -> the survivors' collective
  fails within the collective timeout, the round is aborted and rolled back, and
  the survivors finish the next round as a smaller group within a bounded time.

CPU variants use MLP clients over gloo; GPU variants run native-LeNet clients on
the MI355X whose FedAvg uses the hipIpc peer kernels.
"""
import os
import time

import pytest

from fedmi import ckpt as ck

from helpers import (free_port, kill9, read_jsonl, spawn_client, spawn_server, stop_proc, wait_for,
                     wait_heartbeat)

pytestmark = [pytest.mark.slow, pytest.mark.timeout(300)]

RECOVERY_S = 2.0      # kill -> first committed round of the survivors, default collective timeout
CPU_MODEL = ("--model", "mlp", "--data", "synthetic-mnist", "--n-train", "512", "--n-test", "256", "--lr", "0.05")
GPU_MODEL = ("--model", "lenet", "--n-train", "2560", "--n-test", "1000")


def _report(**rec):
    """FEDMI_FAILOVER_REPORT=<jsonl>: append the measured drill numbers (profiles/)."""
    path = os.environ.get("FEDMI_FAILOVER_REPORT")
    if path:
        import json
        from pathlib import Path

        Path(path).parent.mkdir(parents=True, exist_ok=True)
        with open(path, "a") as f:
            f.write(json.dumps(rec) + "\n")


def _keep_logs(tmp_path, tag):
    """On failure, copy the drill's logs next to FEDMI_FAILOVER_REPORT (read back from the GPU box), and print each
    client log's tail into the captured output (a suite run without the report path still records them)."""
    for f in sorted(tmp_path.glob("client*.log")):
        lines = f.read_text(errors="replace").splitlines()
        print(f"----- {tag}: {f.name} (last 15 of {len(lines)} lines)")
        print("\n".join(lines[-15:]))
    path = os.environ.get("FEDMI_FAILOVER_REPORT")
    if path:
        import shutil
        from pathlib import Path

        dst = Path(path).parent / f"logs_{tag}"
        dst.mkdir(parents=True, exist_ok=True)
        for f in list(tmp_path.glob("*.log")) + list(tmp_path.glob("*.jsonl")):
            shutil.copy(f, dst / f.name)


def _rounds(path, ok_only=True):
    return [r for r in read_jsonl(path) if r.get("event") == "round" and (r.get("ok") or not ok_only)]


def _client_args(device, collective_timeout=None):
    """``collective_timeout`` None: the client CLI's default (20 s) -- the client-loss drills rely on the
    coordinator's loss propagation (abort key -> watchdog), not on the timeout."""
    ct = () if collective_timeout is None else ("--collective-timeout", str(collective_timeout))
    if device.startswith("cuda"):
        return ("--transport", "peer") + ct + GPU_MODEL
    return ("--backend", "gloo") + ct + CPU_MODEL


def _primary_sigkill_and_recover(tmp_path, device, n_clients=2):
    addrs = [f"127.0.0.1:{free_port()}" for _ in range(n_clients)]
    procs = [spawn_client(a, tmp_path, "--agg", "collective", *_client_args(device, 3),
                          "--metrics", str(tmp_path / f"client{i}.jsonl"),
                          log_path=tmp_path / f"client{i}.log", device=device) for i, a in enumerate(addrs)]
    bport = free_port()
    common = ("--backupPort", str(bport), "--clients", ",".join(addrs), "--rounds", "100000", "--root",
              str(tmp_path / "srv"), "--heartbeat", "0.1", "--watchdog", "1.0", "--train-timeout", "60",
              "--rpc-timeout", "5")
    try:
        for a in addrs:
            wait_heartbeat(a, timeout=120)
        backup = spawn_server(tmp_path, *common, "--metrics", str(tmp_path / "backup.jsonl"),
                              log_path=tmp_path / "backup.log")
        primary = spawn_server(tmp_path, "--p", "y", *common, "--metrics", str(tmp_path / "primary.jsonl"),
                               log_path=tmp_path / "primary.log")
        wait_for(lambda: len(_rounds(tmp_path / "primary.jsonl")) >= 4, timeout=120)
        # the backup's watchdog is armed (it has had a ping) before the kill
        wait_for(lambda: [r for r in read_jsonl(tmp_path / "backup.jsonl") if r.get("event") == "primary_seen"],
                 timeout=15)
        # the backup saw the primary (its watchdog is armed) and never acted as primary before the kill
        assert not [r for r in read_jsonl(tmp_path / "backup.jsonl") if r.get("event") == "promoted"]
        wait_for(lambda: (tmp_path / "srv" / "Backup" / ck.OPTIMIZED_MODEL).exists(), timeout=30)
        # ---- the primary process dies mid-run (the round loop runs back to back: mid-round)
        t_kill = kill9(primary)
        r_dead = max(r["round"] for r in _rounds(tmp_path / "primary.jsonl"))
        promoted = wait_for(lambda: [r for r in read_jsonl(tmp_path / "backup.jsonl") if r.get("event") == "promoted"],
                            timeout=30)
        takeover = promoted[0]["ts"] - t_kill
        assert takeover < 5.0, takeover                       # watchdog 1 s (reference: 13.7 s)
        # the acting backup resumes from the replicated round (not round 0, quirk A8) and keeps going
        first = wait_for(lambda: [r for r in _rounds(tmp_path / "backup.jsonl") if r["ts"] > t_kill], timeout=120)[0]
        # Replication is asynchronous and coalesced (fetch every 50 ms), so the replica trails the dead
        # primary by a bounded TIME, not a bounded round count: GPU rounds of this drill take a few ms.
        # It must hold at least what the primary had finished 1 s before the kill.
        prim = _rounds(tmp_path / "primary.jsonl")
        r_floor = max([r["round"] for r in prim if r["ts"] <= t_kill - 1.0] + [1])
        # Round leases: the clients keep running the dead primary's lease until the backup's newer term
        # reaches them (they stop at the next round boundary), and the primary records a lease's rounds only
        # when it ends.  So the backup resumes right after the clients' last COMMITTED round, which can be
        # past the primary's last recorded round: no round is skipped or repeated.
        committed = set()
        for i in range(n_clients):
            committed |= {r["round"] for r in read_jsonl(tmp_path / f"client{i}.jsonl")
                          if "train_ms" in r and "round" in r and r["ts"] < first["ts"]}
        assert r_floor <= first["round"], (first["round"], r_floor)
        assert first["round"] - 1 in committed and first["round"] - 1 >= r_dead, (first["round"], r_dead,
                                                                                 sorted(committed)[-5:])
        r_dead = first["round"] - 1
        wait_for(lambda: max([r["round"] for r in _rounds(tmp_path / "backup.jsonl")] + [0]) >= r_dead + 2,
                 timeout=120)
        # ---- the primary process is restarted: the backup demotes itself cleanly (quirk A2)
        primary2 = spawn_server(tmp_path, "--p", "y", *common, "--metrics", str(tmp_path / "primary2.jsonl"),
                                log_path=tmp_path / "primary2.log")
        procs.append(primary2)
        wait_for(lambda: [r for r in read_jsonl(tmp_path / "backup.jsonl") if r.get("event") == "demoted"],
                 timeout=60)
        r2 = wait_for(lambda: _rounds(tmp_path / "primary2.jsonl"), timeout=120)
        assert r2[0]["round"] >= r_floor                     # resumed from Primary/optimizedModel.pth's epoch
        assert backup.poll() is None                         # the demoted backup is alive and serving
        wait_heartbeat(f"127.0.0.1:{bport}", timeout=10)
        demoted = [r for r in read_jsonl(tmp_path / "backup.jsonl") if r.get("event") == "demoted"][0]
        _report(drill="primary_sigkill", device=device, clients=n_clients, takeover_s=round(takeover, 3),
                primary_last_round=r_dead,
                backup_first_round=first["round"], restarted_primary_first_round=r2[0]["round"],
                demote_after_restart_s=round(demoted["ts"] - promoted[0]["ts"], 3))
        stop_proc(primary2)
        stop_proc(backup)
        return takeover
    finally:
        for p in procs:
            stop_proc(p)


def _client_killed_mid_collective(tmp_path, device, n_clients=3):
    from fedmi.control.coordinator import Coordinator, CoordinatorConfig

    addrs = [f"127.0.0.1:{free_port()}" for _ in range(n_clients)]
    victim = n_clients - 1
    surv = n_clients - 1
    procs = [spawn_client(a, tmp_path, "--agg", "collective", *_client_args(device),
                          "--metrics", str(tmp_path / f"client{i}.jsonl"),
                          log_path=tmp_path / f"client{i}.log", device=device,
                          env_extra={"FEDMI_FAULT_STALL_AVG_S": "4", "FEDMI_FAULT_STALL_FROM_ROUND": "3"}
                          if i == victim else None)
             for i, a in enumerate(addrs)]
    import threading

    try:
        for a in addrs:
            wait_heartbeat(a, timeout=120)
        cfg = CoordinatorConfig(clients=addrs, rounds=100000, agg="collective", root=str(tmp_path / "srv"),
                                heartbeat_s=0.2, train_timeout_s=60, rpc_timeout_s=5)
        from fedmi.utils.metrics import MetricsLog

        coord = Coordinator(cfg, metrics=MetricsLog(tmp_path / "coord.jsonl"))
        t = threading.Thread(target=coord.run, daemon=True)
        t.start()
        # rounds 1-2 commit; from round 3 on the victim stalls 4 s before the collective: the survivors
        # are inside it when it dies.  The coordinator runs round leases (one StartTrain for many rounds), so
        # committed rounds are read off the clients' own per-round records.
        def client_rounds(i=0):
            return [r for r in read_jsonl(tmp_path / f"client{i}.jsonl") if "train_ms" in r and "round" in r]

        wait_for(lambda: len(client_rounds()) >= 2, timeout=60)
        time.sleep(2.0)
        t_kill = kill9(procs[victim])
        committed = max(r["round"] for r in client_rounds() if r["ts"] < t_kill)
        # survivors fail fast, the round is aborted; the next round runs with the survivors only
        ok2 = wait_for(lambda: [r for r in _rounds(tmp_path / "coord.jsonl") if r["world"] == surv], timeout=90)
        recovery = ok2[0]["ts"] - t_kill
        aborted = [r for r in _rounds(tmp_path / "coord.jsonl", ok_only=False) if not r.get("ok")]
        assert aborted and addrs[victim] in aborted[0]["failed"], aborted   # no spurious abort before the kill
        # the survivors sit in the collective with the default 20 s timeout: only the coordinator's loss
        # propagation (abort key -> each survivor's watchdog) gets them out this fast
        assert recovery <= RECOVERY_S, recovery
        prop = [r for r in read_jsonl(tmp_path / "coord.jsonl") if r.get("event") == "loss_propagated"]
        assert prop and prop[0]["client"] == addrs[victim], prop
        # every survivor -- each answered ABORTED -- was rolled back to the committed global model
        rb = wait_for(lambda: [r for r in read_jsonl(tmp_path / "coord.jsonl") if r.get("event") == "rollback"],
                      timeout=10)[0]
        assert sorted(rb["targets"]) == sorted(addrs[:surv]), rb
        assert rb["epoch"] == committed, (rb, committed)          # not a stale fetch: the newest committed round
        for i in range(surv):
            got = [r for r in read_jsonl(tmp_path / f"client{i}.jsonl")
                   if r.get("event") == "send_model" and r["ts"] > t_kill]
            assert got and got[0]["epoch"] == rb["epoch"] and got[0]["state_sum"] == rb["state_sum"], (i, got[:1], rb)
            # the client restored the round's starting (= committed) model itself, before the coordinator did
            ab = [r for r in read_jsonl(tmp_path / f"client{i}.jsonl") if r.get("event") == "round_aborted"]
            assert ab and ab[0]["restored_sum"] == rb["state_sum"], (i, ab[:1], rb)
        wait_for(lambda: len([r for r in _rounds(tmp_path / "coord.jsonl") if r["world"] == surv]) >= 2, timeout=60)
        coord.stop()
        t.join(timeout=60)
        coord.close()
        # the survivors hold the same global model
        for a in addrs[:surv]:
            wait_for(lambda a=a: (ck.read_epoch(tmp_path / "checkpoint" / f"{a}.pth") or 0) >= coord.round, timeout=30)
        m0 = ck.load(tmp_path / "checkpoint" / f"{addrs[0]}.pth")["net"]
        import torch

        for a in addrs[1:surv]:
            m1 = ck.load(tmp_path / "checkpoint" / f"{a}.pth")["net"]
            for k in m0:
                assert torch.allclose(m0[k], m1[k], atol=1e-6), (a, k)
        _report(drill="client_sigkill_mid_collective", device=device, clients=n_clients, recovery_s=round(recovery, 3),
                aborted_round=aborted[0]["round"], next_ok_round=ok2[0]["round"], collective_timeout_s=20,
                loss_propagated_s=round(prop[0]["ts"] - t_kill, 3))
        return recovery
    finally:
        for p in procs:
            stop_proc(p)


def _drill(fn, tmp_path, device, tag):
    try:
        return fn(tmp_path, device)
    except BaseException:
        _keep_logs(tmp_path, tag)
        raise


def test_primary_sigkill_backup_promotes_then_demotes_cpu(tmp_path):
    _drill(_primary_sigkill_and_recover, tmp_path, "cpu", "primary_cpu")


def test_client_sigkill_mid_collective_cpu(tmp_path):
    _drill(_client_killed_mid_collective, tmp_path, "cpu", "client_cpu")


@pytest.mark.gpu
def test_primary_sigkill_backup_promotes_then_demotes_gpu(tmp_path):
    _drill(_primary_sigkill_and_recover, tmp_path, "cuda:0", "primary_gpu")


@pytest.mark.gpu
def test_client_sigkill_mid_collective_gpu(tmp_path):
    _drill(_client_killed_mid_collective, tmp_path, "cuda:0", "client_gpu")


# BASELINE config 5 at its stated scale: 8 client processes (all on the one GPU of the test box, peer
# transport over same-device hipIpc), primary + backup coordinators.
@pytest.mark.gpu
@pytest.mark.timeout(420)
def test_primary_sigkill_8_clients_gpu(tmp_path):
    _drill(lambda t, d: _primary_sigkill_and_recover(t, d, n_clients=8), tmp_path, "cuda:0", "primary_gpu8")


@pytest.mark.gpu
@pytest.mark.timeout(420)
def test_client_sigkill_mid_collective_8_clients_gpu(tmp_path):
    _drill(lambda t, d: _client_killed_mid_collective(t, d, n_clients=8), tmp_path, "cuda:0", "client_gpu8")


def test_client_sigkill_mid_collective_8_clients_cpu(tmp_path):
    _drill(lambda t, d: _client_killed_mid_collective(t, d, n_clients=8), tmp_path, "cpu", "client_cpu8")
