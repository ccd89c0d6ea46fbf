#!/usr/bin/env python
"""Per-tensor gradient cosines of the native CNN engine at random init (one batch of 64):

  native vs emulated   -- same engine schedule and bf16 buffers, kernels vs their PyTorch twins
                          (tests/emulate.py); both round activations to bf16 at the same points, so
                          what differs is only fp32 reduction order inside the kernels
  native vs fp32       -- plain PyTorch fp32 autograd of the reference model
  emulated vs fp32     -- the same, for the twins (the bf16-storage floor)
  torch-bf16 vs fp32   -- PyTorch's own bf16 (autocast) model: how ill-conditioned the net is

Writes one JSON object per model (tensor -> the four cosines) for the per-tensor bounds of
tests/test_cnn_native_gpu.py::test_native_matches_emulated_kernels_on_gpu.

  python tools/diag_grad_cosines.py --models ResNet18 MobileNetV2 --out profiles/r4_tests/grad_cosines.jsonl
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def _cos(a, b):
    return float(F.cosine_similarity(a.flatten().double(), b.flatten().double(), dim=0))


def main() -> int:
    from fedmi.engine.base import TrainerConfig
    from fedmi.engine.cnn_native import CNNNativeTrainer
    from fedmi.engine.data import augment_normalize, make_dataset
    from fedmi.models import build_model
    from emulate import emulated

    ap = argparse.ArgumentParser()
    ap.add_argument("--models", nargs="+", default=["ResNet18", "MobileNetV2"])
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    nb = 64
    data = make_dataset("synthetic-cifar10", device=dev, n_train=128, n_test=64, seed=0)
    lines = []
    for name in a.models:
        torch.manual_seed(0)
        init = build_model(name).state_dict()
        g = {}
        for kind in ("native", "emulated"):
            cfg = TrainerConfig(batch_size=nb, augment=False, use_graph=False)
            if kind == "native":
                tr = CNNNativeTrainer(name, data, dev, cfg, init_state=init)
                tr.grads_for_batch(0, nb)
            else:
                with emulated():
                    tr = CNNNativeTrainer(name, data, dev, cfg, init_state=init)
                    tr.grads_for_batch(0, nb)
            torch.cuda.synchronize()
            g[kind] = {k: p.grad.detach().float().clone() for k, p in tr.model.named_parameters()}
        x = augment_normalize(data.train.x[:nb], None, 0, 0)
        y = data.train.y[:nb].long()
        for kind in ("fp32", "torch-bf16"):
            ref = build_model(name).to(dev)
            ref.load_state_dict(init)
            ref.train()
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=kind == "torch-bf16"):
                loss = F.cross_entropy(ref(x), y)
            loss.backward()
            g[kind] = {k: p.grad.detach().float().clone() for k, p in ref.named_parameters()}
        rows = {}
        for k in g["native"]:
            rows[k] = {"native_vs_emulated": round(_cos(g["native"][k], g["emulated"][k]), 4),
                       "native_vs_fp32": round(_cos(g["native"][k], g["fp32"][k]), 4),
                       "emulated_vs_fp32": round(_cos(g["emulated"][k], g["fp32"][k]), 4),
                       "torch_bf16_vs_fp32": round(_cos(g["torch-bf16"][k], g["fp32"][k]), 4)}
        vals = [r["native_vs_emulated"] for r in rows.values()]
        rec = {"model": name, "batch": nb, "tensors": len(rows),
               "native_vs_emulated_min": min(vals), "native_vs_emulated_mean": round(sum(vals) / len(vals), 4),
               "below_0.99": sum(v < 0.99 for v in vals), "per_tensor": rows}
        print(json.dumps({k: v for k, v in rec.items() if k != "per_tensor"}), flush=True)
        lines.append(json.dumps(rec))
    if a.out:
        Path(a.out).parent.mkdir(parents=True, exist_ok=True)
        Path(a.out).write_text("\n".join(lines) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
