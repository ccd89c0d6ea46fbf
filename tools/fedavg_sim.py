#!/usr/bin/env python
"""In-process FedAvg simulator: N clients on ONE device, one process, same data split and
round semantics as bench.py / the client agents -- for engine-vs-engine parity runs.

Every client is a full :class:`LocalTrainer` (own model, momentum, data shard); a round
is: each client trains one local epoch on its shard -> the uniform mean of every
float state entry and the floor mean of the int64 BN counters (reference
src/server.py:155-179, fedmi.parallel.fedavg semantics) is loaded into every client
-> the global model is evaluated on the full test set.  ``--engine native`` uses
the fedmi HIP engines (bf16 activations, fp32 master), ``--engine fp32`` plain
PyTorch fp32 (FEDMI_TORCH_PATH=1), both from the same initial weights.

  python tools/fedavg_sim.py --model resnet18 --clients 2 --noniid 2 --rounds 8 --engine fp32
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

N_TRAIN, N_TEST, BATCH = 50000, 10000, 128


def _eval_batch_bn(tr) -> None:
    """Diagnostic (PyTorch engines): evaluate the global model with batch-statistics BN instead of the averaged
    running statistics (train-mode BN at momentum 0, so the running buffers are left as they are)."""
    from torch.nn.modules.batchnorm import _BatchNorm

    m = tr.model
    bns = [b for b in m.modules() if isinstance(b, _BatchNorm)]
    mom = [b.momentum for b in bns]
    for b in bns:
        b.momentum = 0.0
    orig_eval = m.eval
    m.eval = lambda: m.train()
    try:
        with torch.no_grad():
            tr.evaluate()
    finally:
        m.eval = orig_eval
        for b, v in zip(bns, mom):
            b.momentum = v
        m.eval()


def _run_seed(a, seed, data, dev, out) -> None:
    from fedmi.engine import build_trainer
    from fedmi.engine.base import TrainerConfig
    from fedmi.engine.data import contiguous_schedule, label_shard_indices, strided_schedule

    cfg = TrainerConfig(seed=seed, lr=a.lr, augment=not a.no_augment, use_graph=not a.no_graph)
    W = a.clients
    clients = []
    init = None
    for r in range(W):
        tr = build_trainer(a.model, data, dev, cfg, init_state=init)
        if a.engine == "bf16":
            def run(x, m=tr.model):
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    return m(x).float()
            tr._run = run
        if init is None:        # one shared init (rank-0 broadcast, reference quirk A7 fixed)
            init = {k: v.detach().cpu().clone() for k, v in tr.state_dict().items()}
        if a.noniid > 0:
            shards = label_shard_indices(data.train.y.cpu().numpy(), W, a.noniid, seed=0)
            tr.set_train_data(data.train.subset(shards[r]))
            tr.set_schedule(*contiguous_schedule(len(shards[r]), BATCH))
        else:
            tr.set_schedule(*strided_schedule(a.n_train, BATCH, r, W))
        clients.append(tr)
    for rnd in range(1, a.rounds + 1):
        t0 = time.perf_counter()
        tstats = []
        for tr in clients:
            tr.train_epoch()
            tstats.append(tr.train_stats())
        with torch.no_grad():
            mean = torch.stack([tr.float_state() for tr in clients]).mean(0)
            ints = [torch.div(sum(bs), W, rounding_mode="floor")
                    for bs in zip(*[[b.clone() for b in tr.int_state()] for tr in clients])]
            for tr in clients:
                tr.float_state().copy_(mean)
                for b, v in zip(tr.int_state(), ints):
                    b.copy_(v)
                tr.after_aggregate()
        if a.bn_eval == "batch":
            _eval_batch_bn(clients[0])
        else:
            clients[0].evaluate()
        ev = clients[0].eval_stats()
        torch.cuda.synchronize() if dev.type == "cuda" else None
        rec = {"round": rnd, "engine": a.engine, "model": a.model, "clients": W, "lr": a.lr, "seed": seed,
               "data": a.data,
               "deterministic": bool(a.deterministic),
               "augment": not a.no_augment, "graph": not a.no_graph,
               "split": f"noniid-{a.noniid}" if a.noniid else "strided-iid", "bn_eval": a.bn_eval,
               "train_loss": [round(s.loss, 4) for s in tstats], "train_acc": [round(s.acc, 2) for s in tstats],
               "test_loss": round(ev.loss, 4), "test_acc": round(ev.acc, 2),
               "finite": bool(torch.isfinite(mean).all()), "round_s": round(time.perf_counter() - t0, 3)}
        line = json.dumps(rec)
        print(line, flush=True)
        if out:
            out.write(line + "\n")
            out.flush()


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--clients", type=int, default=2)
    ap.add_argument("--noniid", type=int, default=0, help="label shards per client (0 = strided IID)")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--engine", choices=["native", "fp32", "bf16"], default="native",
                    help="bf16: PyTorch autocast bf16 (torch's own mixed precision of the same model)")
    ap.add_argument("--data", default="synthetic-cifar10",
                    help="dataset spec (fedmi.engine.data.make_dataset): synthetic-cifar10 | synthetic-cifar10-easy | ...")
    ap.add_argument("--n-train", type=int, default=N_TRAIN)
    ap.add_argument("--n-test", type=int, default=N_TEST)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--seed", type=int, default=17)
    ap.add_argument("--seeds", default="", help="comma list: run each seed in turn (one process)")
    ap.add_argument("--out", default=None, help="JSONL, one record per round")
    ap.add_argument("--no-augment", action="store_true", help="no crop/flip (diagnostics)")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of graph replay (diagnostics)")
    ap.add_argument("--deterministic", action="store_true",
                    help="PyTorch engines: deterministic algorithms (MIOpen / rocBLAS deterministic kernels), so two "
                         "runs of the fp32 reference agree and a parity gap is the engine's, not reference noise")
    ap.add_argument("--bn-eval", choices=["running", "batch"], default="running",
                    help="batch: evaluate the global model with batch-statistics BN (diagnostic, PyTorch engines)")
    a = ap.parse_args()
    if a.bn_eval == "batch" and a.engine == "native":
        ap.error("--bn-eval batch needs a PyTorch engine (fp32 / bf16)")
    if a.engine in ("fp32", "bf16"):
        os.environ["FEDMI_TORCH_PATH"] = "1"
    if a.deterministic:
        from fedmi.utils.stats import make_deterministic

        make_deterministic()

    from fedmi.engine.data import make_dataset

    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    data = make_dataset(a.data, device=dev, n_train=a.n_train, n_test=a.n_test, seed=0)
    seeds = [int(v) for v in a.seeds.split(",")] if a.seeds else [a.seed]
    out = open(a.out, "w") if a.out else None
    for seed in seeds:
        _run_seed(a, seed, data, dev, out)
        torch.cuda.empty_cache() if dev.type == "cuda" else None
    return 0


if __name__ == "__main__":
    sys.exit(main())
