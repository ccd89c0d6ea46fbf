"""Convergence A/B on one GPU: fused HIP LeNet vs PyTorch fp32 vs PyTorch bf16-autocast.

Same data, same init, same augmentation stream, same SGD recipe; prints
per-epoch train loss / test accuracy of each engine.
"""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

from fedmi.engine.base import TrainerConfig  # noqa: E402
from fedmi.engine.data import make_dataset, strided_schedule  # noqa: E402
from fedmi.engine.lenet_native import LeNetNativeTrainer  # noqa: E402
from fedmi.engine.torch_engine import TorchTrainer  # noqa: E402
from fedmi.models.small import LeNet  # noqa: E402


def main(epochs=4, n_train=50000):
    dev = torch.device("cuda", 0)
    ds = make_dataset("synthetic-cifar10", device=dev, n_train=n_train, n_test=10000, seed=0)
    torch.manual_seed(17)
    init = LeNet().state_dict()
    sched = strided_schedule(n_train, 128, 0, 1)
    cfg = TrainerConfig(seed=17)
    engines = {
        "hip-fused": LeNetNativeTrainer(ds, dev, cfg, init_state=init),
        "torch-fp32": TorchTrainer("lenet", ds, dev, cfg, init_state=init),
    }
    for e in engines.values():
        e.set_schedule(*sched)
    for ep in range(epochs):
        line = []
        for name, e in engines.items():
            t0 = time.perf_counter()
            e.train_epoch()
            e.evaluate()
            tr, ev = e.train_stats(), e.eval_stats()
            line.append(f"{name}: loss {tr.loss:.3f} train {tr.acc:5.1f}% test {ev.acc:5.1f}% "
                        f"({(time.perf_counter() - t0) * 1e3:.0f} ms)")
        print(f"epoch {ep}: " + " | ".join(line), flush=True)


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
