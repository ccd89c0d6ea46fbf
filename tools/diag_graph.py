"""Run-to-run spread of the native CNN engine: eager vs eager, graph vs graph,
eager vs graph after the same SGD steps from one init.

    python tools/diag_graph.py [ResNet18] [steps]
"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from fedmi.engine.base import TrainerConfig  # noqa: E402
from fedmi.engine.cnn_native import CNNNativeTrainer  # noqa: E402
from fedmi.engine.data import make_dataset  # noqa: E402
from fedmi.models import build_model  # noqa: E402


def run(name, data, init, graph, steps, dev):
    tr = CNNNativeTrainer(name, data, dev, TrainerConfig(batch_size=128, lr=0.05, use_graph=graph, seed=3),
                          init_state=init)
    tr.set_schedule([128 * i for i in range(steps)], [128] * steps)
    before = tr.float_state().clone()
    tr.train_epoch()
    torch.cuda.synchronize()
    return tr.float_state().clone(), tr.momentum_state().clone(), tr.train_stats().loss, before


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "ResNet18"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    dev = torch.device("cuda", 0)
    data = make_dataset("synthetic-cifar10", device=dev, n_train=128 * steps, n_test=500, seed=0)
    init = build_model(name).state_dict()
    r = {k: run(name, data, init, g, steps, dev) for k, g in (("e1", False), ("e2", False), ("g1", True),
                                                              ("g2", True))}
    upd = float((r["e1"][0] - r["e1"][3]).norm())
    for a, b in (("e1", "e2"), ("g1", "g2"), ("e1", "g1")):
        dp = float((r[a][0] - r[b][0]).norm())
        dm = float((r[a][1] - r[b][1]).norm() / r[a][1].norm())
        print(f"{name} steps {steps} {a} vs {b}: |dparam| {dp:.4e} (update norm {upd:.4e}) rel dmom {dm:.3e} "
              f"loss {r[a][2]:.5f} / {r[b][2]:.5f}")


if __name__ == "__main__":
    main()
