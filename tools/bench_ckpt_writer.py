#!/usr/bin/env python
"""Sustained-rate microbench of AsyncCheckpointWriter at the N=8 LeNet round cadence.

At 8 clients a LeNet round is ~1.3 ms of local compute (49 SGD steps), so the
per-round checkpoint (Primary/optimizedModel.pth + checkpoint/<client>.pth,
bench.py one_round) must not back-pressure the loop.  This drives ``submit`` at
a fixed cadence with the LeNet flat state on the GPU (views into one fp32
buffer, like the engine's state_dict) and reports the achieved round cadence,
submit latency percentiles, files written and rounds coalesced -- for the
coalescing writer (default) and the write-every-round writer.
"""
from __future__ import annotations

import argparse
import json
import sys
import tempfile
import time
from collections import OrderedDict
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def lenet_state(device):
    shapes = [("conv1.weight", (6, 3, 5, 5)), ("conv1.bias", (6,)), ("conv2.weight", (16, 6, 5, 5)),
              ("conv2.bias", (16,)), ("fc1.weight", (120, 400)), ("fc1.bias", (120,)), ("fc2.weight", (84, 120)),
              ("fc2.bias", (84,)), ("fc3.weight", (10, 84)), ("fc3.bias", (10,))]
    n = sum(torch.Size(s).numel() for _, s in shapes)
    flat = torch.randn(n, device=device)
    sd, o = OrderedDict(), 0
    for k, s in shapes:
        m = torch.Size(s).numel()
        sd[k] = flat[o:o + m].view(s)
        o += m
    return flat, sd


def run(coalesce, rounds: int, cadence_ms: float, device) -> dict:
    from fedmi.ckpt import AsyncCheckpointWriter, RoundCheckpointWriter

    flat, sd = lenet_state(device)
    root = Path(tempfile.mkdtemp(prefix="ckw_"))
    paths = [root / "Primary" / "optimizedModel.pth", root / "checkpoint" / "client0.pth"]
    for p in paths:
        p.parent.mkdir(parents=True, exist_ok=True)
    native = isinstance(coalesce, str)
    w = RoundCheckpointWriter(coalesce=coalesce == "native-coalesce") if native else AsyncCheckpointWriter(coalesce=coalesce)
    lat = []
    t0 = time.perf_counter()
    nxt = t0
    for r in range(rounds):
        flat.add_(1e-3)                         # the "round": model changes on the GPU
        nxt += cadence_ms * 1e-3
        while time.perf_counter() < nxt:        # the rest of the round (launches, waits)
            time.sleep(0)
        a = time.perf_counter()
        w.submit(paths, sd, acc=1, epoch=r + 1)
        lat.append((time.perf_counter() - a) * 1e3)
    t_loop = time.perf_counter() - t0
    w.flush()
    t_all = time.perf_counter() - t0
    from fedmi.ckpt import load
    last = load(paths[0])["epoch"]
    w.close()
    lat.sort()
    return {"writer": "native-cxx" if native else "python-thread",
            "coalesce": coalesce == "native-coalesce" if native else coalesce, "rounds": rounds, "target_cadence_ms": cadence_ms,
            "achieved_cadence_ms": round(t_loop / rounds * 1e3, 4), "flush_ms": round((t_all - t_loop) * 1e3, 3),
            "submit_ms_p50": round(lat[len(lat) // 2], 4), "submit_ms_p99": round(lat[int(len(lat) * 0.99)], 4),
            "submit_ms_max": round(lat[-1], 4), "files_written": w.written, "rounds_coalesced": w.coalesced,
            "last_epoch_on_disk": last, "device": str(device)}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=1000)
    ap.add_argument("--cadence-ms", type=float, default=1.3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    rows = [run("native", a.rounds, a.cadence_ms, dev), run("native-coalesce", a.rounds, a.cadence_ms, dev),
            run(True, a.rounds, a.cadence_ms, dev),
            run(False, a.rounds, a.cadence_ms, dev)]
    for r in rows:
        print(json.dumps(r), flush=True)
    if a.out:
        Path(a.out).write_text("".join(json.dumps(r) + "\n" for r in rows))
    return 0


if __name__ == "__main__":
    sys.exit(main())
