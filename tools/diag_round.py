#!/usr/bin/env python
"""Per-phase cost of one federated round on ONE GPU, as rank 0 of a simulated
world of W clients (strided 1/W shard, no collective): shows which fixed
per-round costs limit strong scaling of bench.py at 2/4/8 GPUs.

    python tools/diag_round.py [--model lenet] [--worlds 1,2,4,8] [--rounds 20]

Phases (each bracketed by torch.cuda.synchronize in the *phased* pass):
train (graph replay of the local epoch), aggregate (after_aggregate: repack),
eval, ckpt (state_dict snapshot + async writer submit x2).  A second pass runs
the same rounds without intermediate syncs = the bench's per-round time.
"""
from __future__ import annotations

import argparse
import json
import sys
import tempfile
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="lenet")
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--eval-shard", action="store_true", help="evaluate only this rank's 1/W of the test set")
    args = ap.parse_args()

    from fedmi.ckpt import AsyncCheckpointWriter, OPTIMIZED_MODEL, client_ckpt_path, mount_dir
    from fedmi.engine import build_trainer
    from fedmi.engine.base import TrainerConfig
    from fedmi.engine.data import make_dataset, strided_schedule
    from fedmi.parallel.fedavg import eval_shard

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    data = make_dataset("synthetic-cifar10", device=dev, n_train=50000, n_test=10000, seed=0)
    tr = build_trainer(args.model, data, dev, TrainerConfig(seed=17))
    root = Path(tempfile.mkdtemp(prefix="fedmi_diag_"))
    prim = mount_dir(root, primary=True)
    cpath = client_ckpt_path(root, "client0")
    writer = AsyncCheckpointWriter()

    def sync():
        torch.cuda.synchronize(dev)

    for W in [int(w) for w in args.worlds.split(",")]:
        tr.set_schedule(*strided_schedule(50000, 128, W - 1, W))   # slowest rank (owns the partial batch)
        tr.set_test_data(eval_shard(data.test, 0, W) if args.eval_shard else data.test)
        ph = {"train": 0.0, "aggregate": 0.0, "eval": 0.0, "ckpt": 0.0}
        for r in range(3):                       # warm-up (graph capture)
            tr.train_epoch(); tr.after_aggregate(); tr.evaluate()
            writer.submit([prim / OPTIMIZED_MODEL, cpath], tr.state_dict(), epoch=r)
        writer.flush(); sync()
        for r in range(args.rounds):
            t = time.perf_counter(); tr.train_epoch(); sync(); ph["train"] += time.perf_counter() - t
            t = time.perf_counter(); tr.after_aggregate(); sync(); ph["aggregate"] += time.perf_counter() - t
            t = time.perf_counter(); tr.evaluate(); sync(); ph["eval"] += time.perf_counter() - t
            t = time.perf_counter()
            writer.submit([prim / OPTIMIZED_MODEL, cpath], tr.state_dict(), epoch=r)
            writer.flush(); sync()
            ph["ckpt"] += time.perf_counter() - t
        t0 = time.perf_counter()
        for r in range(args.rounds):
            tr.train_epoch(); tr.after_aggregate(); tr.evaluate()
            writer.submit([prim / OPTIMIZED_MODEL, cpath], tr.state_dict(), epoch=r)
        writer.flush(); sync()
        t_round = (time.perf_counter() - t0) / args.rounds
        out = {"world": W, "batches": len(strided_schedule(50000, 128, W - 1, W)[0]),
               "round_ms": round(t_round * 1e3, 3), "rounds_per_s": round(1 / t_round, 2)}
        out.update({f"{k}_ms": round(v / args.rounds * 1e3, 3) for k, v in ph.items()})
        print(json.dumps(out), flush=True)
    writer.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
