#!/usr/bin/env python
"""Where do the native engine and fp32 PyTorch first part ways at the reference lr (non-IID, round 1)?

VERDICT r3 "next round" 2: at lr 0.1 on the 2-label-shard split the native ResNet-18 engine dies (test
accuracy 10 %) in more seeds than fp32.  This steps THE SAME client (client ``--client`` of the
``--clients`` x ``--noniid`` split) through round 1 one batch at a time with several engines from one
init, no augmentation (identical batches), and records after every step:

  * the batch loss and accuracy of each engine;
  * per parameter tensor: ||w_e - w_fp32|| / ||w_fp32 - w_init|| (how far engine e has drifted from the
    fp32 trajectory, relative to how far fp32 itself moved), and the gradient cosine vs fp32;
  * per BatchNorm: running_mean / running_var relative difference vs fp32.

Engines: ``native`` (fedmi HIP, bf16 activations), ``fp32`` (PyTorch fp32), ``bf16`` (PyTorch autocast
bf16 -- the same model in torch's own mixed precision: is the fragility bf16's, or the kernels'?).
One JSON line per step; a summary line at the end names the first step / tensor where the native
engine's drift exceeds ``--thr`` and where torch-bf16's does.

  python tools/diag_noniid_bisect.py --steps 120 --out profiles/r4_noniid/bisect_s17.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def _cos(a, b):
    return float(F.cosine_similarity(a.flatten().double(), b.flatten().double(), dim=0, eps=1e-30))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--clients", type=int, default=2)
    ap.add_argument("--noniid", type=int, default=2)
    ap.add_argument("--client", type=int, default=0)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--seed", type=int, default=17)
    ap.add_argument("--steps", type=int, default=120)
    ap.add_argument("--engines", nargs="+", default=["native", "fp32", "bf16"])
    ap.add_argument("--thr", type=float, default=0.5)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()

    from fedmi.engine.base import TrainerConfig
    from fedmi.engine.cnn_native import CNNNativeTrainer
    from fedmi.engine.data import contiguous_schedule, label_shard_indices, make_dataset
    from fedmi.engine.torch_engine import TorchTrainer
    from fedmi.models import build_model

    dev = torch.device("cuda", 0)
    data = make_dataset("synthetic-cifar10", device=dev, n_train=50000, n_test=1000, seed=0)
    shards = label_shard_indices(data.train.y.cpu().numpy(), a.clients, a.noniid, seed=0)
    shard = data.train.subset(shards[a.client])
    starts, sizes = contiguous_schedule(len(shard), 128)
    cfg = TrainerConfig(seed=a.seed, lr=a.lr, augment=False, use_graph=False)
    torch.manual_seed(a.seed)
    init = {k: v.detach().clone() for k, v in build_model(a.model).state_dict().items()}
    eng = {}
    for e in a.engines:
        if e == "native":
            tr = CNNNativeTrainer(a.model, data, dev, cfg, init_state=init)
        else:
            tr = TorchTrainer(a.model, data, dev, cfg, init_state=init, hybrid=False)
            if e == "bf16":
                m = tr.model

                def run(x, m=m):
                    with torch.autocast("cuda", dtype=torch.bfloat16):
                        return m(x).float()
                tr._run = run
        tr.set_train_data(shard)
        eng[e] = tr
    w0 = {k: v.detach().float().clone() for k, v in eng["fp32"].state_dict().items()}
    out = open(a.out, "w") if a.out else None
    first = {}
    for step in range(min(a.steps, len(starts))):
        rec = {"step": step, "start": starts[step], "nb": sizes[step]}
        for e, tr in eng.items():
            tr.set_schedule([starts[step]], [sizes[step]])
            tr.train_epoch()
            st = tr.train_stats()
            rec[f"loss_{e}"] = round(st.loss, 5)
            rec[f"acc_{e}"] = round(st.acc, 2)
        torch.cuda.synchronize()
        sd = {e: {k: v.detach().float() for k, v in tr.state_dict().items()} for e, tr in eng.items()}
        gr = {e: {k: p.grad.detach().float() for k, p in tr.model.named_parameters() if p.grad is not None}
              for e, tr in eng.items()}
        ref = sd["fp32"]
        for e in eng:
            if e == "fp32":
                continue
            drift, gcos, bn = {}, {}, {}
            for k, v in sd[e].items():
                if not v.is_floating_point() or v.numel() == 0:
                    continue
                if k.endswith("running_mean") or k.endswith("running_var"):
                    bn[k] = round(float((v - ref[k]).norm() / (ref[k].norm() + 1e-12)), 5)
                    continue
                moved = float((ref[k] - w0[k]).norm())
                drift[k] = round(float((v - ref[k]).norm()) / max(moved, 1e-12), 5)
                if k in gr[e] and k in gr["fp32"]:
                    gcos[k] = round(_cos(gr[e][k], gr["fp32"][k]), 4)
            worst = max(drift, key=drift.get)
            rec[f"{e}_worst_drift"] = [worst, drift[worst]]
            rec[f"{e}_drift"] = drift
            rec[f"{e}_gcos"] = gcos
            rec[f"{e}_bn"] = bn
            if e not in first and drift[worst] > a.thr and step > 0:
                first[e] = {"step": step, "tensor": worst, "drift": drift[worst],
                            "first_layers_over": [k for k in drift if drift[k] > a.thr][:8]}
        line = json.dumps(rec)
        if out:
            out.write(line + "\n")
            out.flush()
        short = {k: v for k, v in rec.items() if not isinstance(v, dict)}
        print(json.dumps(short), flush=True)
    summ = {"summary": True, "args": vars(a), "first_over_thr": first}
    print(json.dumps(summ), flush=True)
    if out:
        out.write(json.dumps(summ) + "\n")
        out.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
