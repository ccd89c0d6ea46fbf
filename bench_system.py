#!/usr/bin/env python
"""System benchmark: the reference's PROCESS layout, timed end to end.

Where ``bench.py`` times the federated round inside torchrun ranks, this
launches what a user of the reference launches (README.md:6-16 of the
reference): a backup ``server.py``, N ``client.py`` processes (one GPU each,
or several on one GPU) and a primary ``server.py --p y`` that drives the rounds
over ``federated.proto`` (src/server.py:113-153).  Every round in the timed
region therefore includes the StartTrain fan-out, the local epochs, the
clients' FedAvg (hipIpc peer kernels or RCCL), per-round evaluation, the
clients' checkpoint writes, rank 0's checkpoint upload, the primary's
``Primary/optimizedModel.pth`` write and its replication to the backup.

Rounds/s is measured from the primary's own per-round JSONL timestamps
(steady state, after ``--warmup`` rounds); the per-phase split comes from the
clients' and the primary's JSONL records.

  python bench_system.py --clients 1 --rounds 30 --warmup 5
  python bench_system.py --clients 4 --rounds 20          # 4 client processes (one GPU each if present)
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
N_TRAIN = 50000


def _port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn(args, cwd: Path, log: Path, env: dict) -> subprocess.Popen:
    return subprocess.Popen([sys.executable, *args], cwd=str(cwd), env=env, stdout=open(log, "w"),
                            stderr=subprocess.STDOUT, start_new_session=True)


def _stop(p: subprocess.Popen) -> None:
    if p.poll() is None:
        try:
            os.killpg(p.pid, 15)
            p.wait(timeout=15)
        except (ProcessLookupError, subprocess.TimeoutExpired):
            try:
                os.killpg(p.pid, 9)
            except ProcessLookupError:
                pass


def _wait_heartbeat(addr: str, timeout: float, procs) -> None:
    sys.path.insert(0, str(ROOT))
    from fedmi.wire import proto as P

    stub = P.TrainerStub(P.make_channel(addr))
    t0 = time.time()
    while time.time() - t0 < timeout:
        if any(p.poll() is not None for p in procs):
            raise RuntimeError("a client process exited during start-up")
        try:
            if stub.HeartBeat(P.Request(), timeout=1.0).status == 1:
                return
        except Exception:
            time.sleep(0.25)
    raise TimeoutError(f"client {addr} did not come up in {timeout:.0f}s")


def _jsonl(path: Path):
    if not path.exists():
        return []
    return [json.loads(line) for line in path.read_text().splitlines() if line.strip()]


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--clients", type=int, default=1)
    ap.add_argument("--rounds", type=int, default=30, help="timed rounds")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="lenet")
    ap.add_argument("-c", "--compressFlag", default=None, help="'Y': gzip control channel + int8 error-feedback updates")
    ap.add_argument("--transport", default="auto", choices=["auto", "peer", "dist"])
    ap.add_argument("--agg", default="collective", choices=["collective", "grpc"])
    ap.add_argument("--gpus", type=int, default=None, help="GPUs to spread clients over (default: all visible)")
    ap.add_argument("--no-backup", action="store_true")
    ap.add_argument("--ckpt-sync-every", type=int, default=0)
    ap.add_argument("--lease", type=int, default=64,
                    help="at most this many rounds per StartTrain (round lease); 1 = one StartTrain per round "
                         "(reference cadence)")
    ap.add_argument("--lease-s", type=float, default=0.25,
                    help="target lease duration (s); 0 = always --lease rounds (server.py --lease-s)")
    ap.add_argument("--keep", default=None, help="keep the run directory here")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--startup-timeout", type=float, default=300.0)
    a = ap.parse_args()

    import torch

    ngpu = a.gpus if a.gpus is not None else (torch.cuda.device_count() if torch.cuda.is_available() else 0)
    run = Path(a.keep) if a.keep else Path(tempfile.mkdtemp(prefix="fedmi_sys_"))
    run.mkdir(parents=True, exist_ok=True)
    env = dict(os.environ)
    env["PYTHONPATH"] = str(ROOT) + os.pathsep + env.get("PYTHONPATH", "")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "2")
    procs = []
    comp = ["-c", a.compressFlag] if a.compressFlag else []
    total = a.warmup + a.rounds
    try:
        bport = _port()
        if not a.no_backup:
            procs.append(_spawn([str(ROOT / "server.py"), "--backupPort", str(bport), "--root", str(run / "srv"),
                                 "--metrics", str(run / "backup.jsonl"), "--watchdog", "30", *comp],
                                run, run / "backup.log", env))
        addrs = [f"127.0.0.1:{_port()}" for _ in range(a.clients)]
        for i, addr in enumerate(addrs):
            dev = f"cuda:{i % ngpu}" if ngpu else "cpu"
            procs.append(_spawn([str(ROOT / "client.py"), "-a", addr, "--device", dev, "--model", a.model,
                                 "--agg", a.agg, "--transport", a.transport, "--root", str(run),
                                 "--metrics", str(run / f"client{i}.jsonl"), "--quiet", *comp],
                                run, run / f"client{i}.log", env))
        for addr in addrs:
            _wait_heartbeat(addr, a.startup_timeout, procs)
        prim = _spawn([str(ROOT / "server.py"), "--p", "y", "--backupPort", str(bport), "--clients", ",".join(addrs),
                       "--rounds", str(total), "--agg", a.agg, "--root", str(run / "srv"), "--train-timeout", "600",
                       "--metrics", str(run / "primary.jsonl"), "--ckpt-sync-every", str(a.ckpt_sync_every),
                       "--lease", str(a.lease), "--lease-s", str(a.lease_s), *comp],
                      run, run / "primary.log", env)
        procs.append(prim)
        deadline = time.time() + 600 + 60 * total
        last = 0
        while prim.poll() is None and time.time() < deadline:
            time.sleep(0.5)
            n = sum(1 for r in _jsonl(run / "primary.jsonl") if r.get("event") == "round")
            if n >= last + 10:
                print(f"[bench_system] {n}/{total} rounds", file=sys.stderr, flush=True)
                last = n
        if prim.poll() is None:
            raise TimeoutError("primary did not finish")
        if prim.returncode != 0:
            raise RuntimeError(f"primary exited with {prim.returncode}; see {run / 'primary.log'}")
    finally:
        for p in procs:
            _stop(p)

    rounds = [r for r in _jsonl(run / "primary.jsonl") if r.get("event") == "round" and r.get("ok")]
    if len(rounds) < total:
        print(f"[bench_system] only {len(rounds)} ok rounds of {total}; see {run}", file=sys.stderr)
        return 1
    # per-round completion time: the client-reported end of each leased round (t_round), else the event time
    tk = "t_round" if all("t_round" in r for r in rounds) else "ts"
    t0, t1 = rounds[a.warmup - 1][tk], rounds[total - 1][tk]
    rps = a.rounds / (t1 - t0)
    timed = {r["round"] for r in rounds[a.warmup:total]}

    def mean(xs):
        return round(statistics.fmean(xs), 4) if xs else None

    phases = {}
    for key in ("group_ms", "train_ms", "allreduce_ms", "eval_ms", "ckpt_ms", "round_ms"):
        per_client = []
        for i in range(a.clients):
            recs = [r for r in _jsonl(run / f"client{i}.jsonl") if r.get("round") in timed and key in r]
            per_client.append(mean([r[key] for r in recs]))
        vals = [v for v in per_client if v is not None]
        phases[f"client_{key}"] = max(vals) if vals else None
    coord_round = mean([r["round_ms"] for r in rounds[a.warmup:total]])
    phases["coordinator_round_ms"] = coord_round
    if coord_round is not None and phases.get("client_round_ms") is not None:
        phases["rpc_and_coordinator_overhead_ms"] = round(coord_round - phases["client_round_ms"], 4)
    # the overhead split (one host clock): request latency (coordinator send -> client handler entry),
    # client handler work outside its timed round, reply latency (handler exit -> coordinator has the
    # reply), coordinator bookkeeping after the replies, and the gap to the next round's send
    by_round = {r["round"]: r for r in rounds}
    # request / reply latency only where a StartTrain begins or ends (the first / last round of a lease)
    c0 = {r["round"]: r for r in _jsonl(run / "client0.jsonl") if r.get("round") in timed and "t_enter" in r
          and r.get("lease_index", 0) == 0 and r.get("lease", 1) == 1}
    req, rep, post, gap, hnd = [], [], [], [], []
    for rnd_, cr in c0.items():
        pr = by_round.get(rnd_)
        if pr is None or "t_send" not in pr:
            continue
        req.append((cr["t_enter"] - pr["t_send"]) * 1e3)
        rep.append((pr["t_recv"] - cr["t_exit"]) * 1e3)
        hnd.append((cr["t_exit"] - cr["t_enter"]) * 1e3 - cr["round_ms"])
        post.append((pr["t_done"] - pr["t_recv"]) * 1e3)
        nxt = by_round.get(rnd_ + 1)
        if nxt is not None and "t_send" in nxt:
            gap.append((nxt["t_send"] - pr["t_done"]) * 1e3)
    if req:
        phases.update(request_latency_ms=mean(req), client_handler_untimed_ms=mean(hnd), reply_latency_ms=mean(rep),
                      coordinator_post_ms=mean(post), coordinator_loop_gap_ms=mean(gap))
    last_rec = [r for r in _jsonl(run / "client0.jsonl") if r.get("round") == total]
    out = {
        "metric": f"system rounds/sec (primary+backup+{a.clients} client processes over gRPC), {a.model} FedAvg",
        "value": round(rps, 4),
        "unit": "rounds/s",
        "samples_per_sec": round(rps * N_TRAIN, 1),
        "samples_per_sec_per_client": round(rps * N_TRAIN / a.clients, 1),
        "n_clients": a.clients,
        "gpus": ngpu,
        "rounds": a.rounds,
        "warmup": a.warmup,
        "ms_per_round": round(1e3 / rps, 4),
        "config": {"model": a.model, "agg": a.agg, "transport": a.transport, "compress": a.compressFlag,
                   "backup": not a.no_backup, "ckpt_sync_every": a.ckpt_sync_every, "lease": a.lease,
                   "lease_s": a.lease_s,
                   "batch": 128, "eval_per_round": True, "data": "synthetic CIFAR-shaped 50k/10k"},
        "phases_ms": phases,
        "last_round": {k: last_rec[0].get(k) for k in ("train_loss", "train_acc", "test_loss", "test_acc")}
        if last_rec else None,
        "primary_model_epoch": None,
        "run_dir": str(run),
    }
    try:
        sys.path.insert(0, str(ROOT))
        from fedmi import ckpt as ck

        out["primary_model_epoch"] = ck.read_epoch(run / "srv" / "Primary" / ck.OPTIMIZED_MODEL)
        out["backup_model_epoch"] = ck.read_epoch(run / "srv" / "Backup" / ck.OPTIMIZED_MODEL)
    except Exception:
        pass
    line = json.dumps(out)
    print(line, flush=True)
    if a.json_out:
        Path(a.json_out).write_text(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
