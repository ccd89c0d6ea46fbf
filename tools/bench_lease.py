#!/usr/bin/env python
"""Control-plane cost per round of the coordinator's StartTrain fan-out, one RPC per round (lease 1, the
reference's cadence, src/server.py:120-153) vs round leases (x-fedmi-lease: one StartTrain runs K rounds),
against 1..8 fake client PROCESSES that train instantly (tests/fake_client.py): everything timed is control
plane.  CPU only.  One JSON line per (clients, lease).

    python tools/bench_lease.py [--leases 1 4 16 64] [--clients 1 2 4 8] [--rounds 256]
"""
from __future__ import annotations

import argparse
import contextlib
import io
import json
import subprocess
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--leases", type=int, nargs="+", default=[1, 4, 16, 64])
    ap.add_argument("--clients", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--rounds", type=int, default=256)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from fedmi.control.coordinator import Coordinator, CoordinatorConfig

    tmp = Path(tempfile.mkdtemp(prefix="fedmi_lease_"))
    procs, addrs = [], []
    for i in range(max(a.clients)):
        procs.append(subprocess.Popen([sys.executable, str(ROOT / "tests" / "fake_client.py"), str(tmp / f"p{i}")],
                                      stdout=subprocess.DEVNULL, stderr=subprocess.STDOUT))
    try:
        for i in range(len(procs)):
            while not (tmp / f"p{i}").exists():
                time.sleep(0.05)
            addrs.append(f"127.0.0.1:{(tmp / f'p{i}').read_text()}")
        lines = []
        for n in a.clients:
            for lease in a.leases:
                cfg = CoordinatorConfig(clients=addrs[:n], rounds=a.rounds, agg="collective",
                                        root=str(tmp / f"s{n}_{lease}"), lease_rounds=lease, lease_s=0, ckpt_fetch_interval_s=0,
                                        heartbeat_s=5.0, rpc_timeout_s=10, train_timeout_s=30)
                with contextlib.redirect_stdout(io.StringIO()):
                    c = Coordinator(cfg)
                    c.run_round()                     # connection setup outside the timed part
                    r0, t0 = c.round, time.perf_counter()
                    while c.round < a.rounds:
                        c.run_round()
                    ms = (time.perf_counter() - t0) / (c.round - r0) * 1e3
                    c.close()
                rec = {"bench": "lease_control_plane", "clients": n, "lease": lease,
                       "control_ms_per_round": round(ms, 4), "rounds": a.rounds}
                print(json.dumps(rec), flush=True)
                lines.append(rec)
        if a.out:
            Path(a.out).write_text("".join(json.dumps(r) + "\n" for r in lines))
    finally:
        for p in procs:
            p.kill()
    return 0


if __name__ == "__main__":
    sys.exit(main())
