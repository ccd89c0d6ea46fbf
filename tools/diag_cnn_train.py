"""Train a zoo CNN with the native engine and with the PyTorch engine on the same
synthetic data / init / lr and print per-epoch losses + final accuracy.

    python tools/diag_cnn_train.py ResNet18 [lr] [epochs] [n_train]
"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from fedmi.engine.base import TrainerConfig  # noqa: E402
from fedmi.engine.cnn_native import CNNNativeTrainer  # noqa: E402
from fedmi.engine.data import contiguous_schedule, make_dataset  # noqa: E402
from fedmi.engine.torch_engine import TorchTrainer  # noqa: E402
from fedmi.models import build_model  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "ResNet18"
    lr = float(sys.argv[2]) if len(sys.argv) > 2 else 0.1
    epochs = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    n = int(sys.argv[4]) if len(sys.argv) > 4 else 10240
    dev = torch.device("cuda", 0)
    data = make_dataset("synthetic-cifar10", device=dev, n_train=n, n_test=2000, seed=0)
    init = build_model(name).state_dict()
    for kind in ("native", "torch"):
        cfg = TrainerConfig(batch_size=128, lr=lr, seed=7)
        tr = (CNNNativeTrainer if kind == "native" else TorchTrainer)(name, data, dev, cfg, init_state=init)
        tr.set_schedule(*contiguous_schedule(n, 128))
        for e in range(epochs):
            tr.train_epoch()
            tr.evaluate()
            s, v = tr.train_stats(), tr.eval_stats()
            print(f"{name} {kind:6s} lr {lr} epoch {e}: train loss {s.loss:.4f} acc {s.acc:.2f} | "
                  f"test loss {v.loss:.4f} acc {v.acc:.2f}", flush=True)


if __name__ == "__main__":
    main()
