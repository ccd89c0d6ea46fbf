#!/usr/bin/env python
"""A/B the LeNet fc1 placement (own kernel vs inside the FC tail) in ONE process,
interleaved rounds (cdna_hip_programming.md rule 24): full 50k-sample rounds
with eval, like bench.py, median ms per round per variant.

    python tools/ab_lenet.py [--rounds 6] [--reps 3]
"""
import argparse
import json
import statistics
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    from fedmi.engine import build_trainer
    from fedmi.engine.base import TrainerConfig
    from fedmi.engine.data import make_dataset, strided_schedule

    dev = torch.device("cuda", 0)
    data = make_dataset("synthetic-cifar10", device=dev, n_train=50000, n_test=10000, seed=0)
    tr = build_trainer("lenet", data, dev, TrainerConfig(seed=17))
    tr.set_schedule(*strided_schedule(50000, 128, 0, 1))
    res = {False: [], True: []}
    for rep in range(a.reps):
        for v in (False, True):
            tr.set_fuse_fc1(v)
            tr.train_epoch(); tr.evaluate()            # capture + warm
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.rounds):
                tr.train_epoch(); tr.after_aggregate(); tr.evaluate()
            torch.cuda.synchronize()
            res[v].append((time.perf_counter() - t0) / a.rounds * 1e3)
    ev = tr.eval_stats()
    print(json.dumps({"fc1_kernel_ms": [round(x, 3) for x in res[False]],
                      "fc1_in_tail_ms": [round(x, 3) for x in res[True]],
                      "median_kernel": round(statistics.median(res[False]), 3),
                      "median_fused": round(statistics.median(res[True]), 3),
                      "test_acc": round(ev.acc, 2)}))


if __name__ == "__main__":
    main()
