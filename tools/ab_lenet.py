#!/usr/bin/env python
"""A/B an engine knob of the fused LeNet step in ONE process, interleaved rounds
(cdna_hip_programming.md rule 24): full 50k-sample rounds with eval, like
bench.py, median ms per round per variant.

    python tools/ab_lenet.py --knob fuse_fc1 [--rounds 6] [--reps 3]   # fc1 inside the FC tail vs own kernel
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
    ap.add_argument("--knob", default="fuse_fc1", choices=["fuse_fc1"])
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from fedmi.engine import build_trainer
    from fedmi.engine.base import TrainerConfig
    from fedmi.engine.data import make_dataset, strided_schedule

    dev = torch.device("cuda", 0)
    data = make_dataset("synthetic-cifar10", device=dev, n_train=50000, n_test=10000, seed=0)
    tr = build_trainer("lenet", data, dev, TrainerConfig(seed=17))
    tr.set_schedule(*strided_schedule(50000, 128, 0, 1))

    def setv(v):
        tr.set_fuse_fc1(v)

    res = {False: [], True: []}
    for rep in range(a.reps):
        for v in (False, True):
            setv(v)
            tr.train_epoch(); tr.evaluate()            # capture + warm
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.rounds):
                tr.train_epoch(); tr.after_aggregate(); tr.evaluate()
            torch.cuda.synchronize()
            res[v].append((time.perf_counter() - t0) / a.rounds * 1e3)
    ev = tr.eval_stats()
    out = {"knob": a.knob, "off_ms": [round(x, 3) for x in res[False]], "on_ms": [round(x, 3) for x in res[True]],
           "median_off": round(statistics.median(res[False]), 3), "median_on": round(statistics.median(res[True]), 3),
           "test_acc": round(ev.acc, 2)}
    print(json.dumps(out))
    if a.out:
        Path(a.out).write_text(json.dumps(out) + "\n")


if __name__ == "__main__":
    main()
