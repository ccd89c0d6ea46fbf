"""Standalone (non-federated) training: ``python -m fedmi.cli.train``.

The reference's ``main.py`` doubles as a standalone CIFAR trainer
(``train(epoch)`` src/main.py:104-125, ``test(epoch)`` :193-228): full-dataset
shuffled epochs at batch 128, SGD(lr, 0.9, 5e-4), a CosineAnnealingLR(T_max=200)
that is created but never stepped (:101, :242), evaluation after each epoch and
a ``{'net','acc','epoch'}`` checkpoint written to ``./checkpoint/<address>.pth``
whenever the test accuracy improves; ``--resume`` restarts from it (:87-96).

Here the same loop runs on the device-resident engines (fused HIP LeNet, or
the generic engine for the zoo).  ``--cosine`` actually steps the schedule
(the reference's is dead code, quirk A7); per-epoch records go to JSONL.
"""
from __future__ import annotations

import argparse
import math
import sys
import time
from pathlib import Path

import numpy as np
import torch

from .. import ckpt
from ..engine import build_trainer
from ..engine.base import TrainerConfig
from ..engine.data import contiguous_schedule, make_dataset
from ..utils.metrics import MetricsLog, log
from ..utils.progress import format_time
from .client import pick_device


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description="fedmi standalone trainer (one GPU)")
    ap.add_argument("--lr", type=float, default=0.1, help="learning rate")
    ap.add_argument("-r", "--resume", action="store_true", help="resume from checkpoint/<address>.pth")
    ap.add_argument("-a", "--address", default="temp", help="checkpoint name (reference: listen address)")
    ap.add_argument("-c", "--compressFlag", help="accepted for argv compatibility; unused standalone")
    ap.add_argument("--model", default="lenet")
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--cosine", action="store_true", help="step CosineAnnealingLR(T_max) every epoch")
    ap.add_argument("--t-max", type=int, default=200)
    ap.add_argument("--no-shuffle", action="store_true")
    ap.add_argument("--device", default="auto")
    ap.add_argument("--data", default="synthetic-cifar10")
    ap.add_argument("--n-train", type=int, default=None)
    ap.add_argument("--n-test", type=int, default=None)
    ap.add_argument("--batch-size", type=int, default=128)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--root", default=".")
    ap.add_argument("--metrics", default=None)
    return ap


def cosine_lr(base: float, epoch: int, t_max: int) -> float:
    """torch CosineAnnealingLR closed form (eta_min = 0)."""
    return 0.5 * base * (1.0 + math.cos(math.pi * epoch / t_max))


def main(argv=None) -> int:
    a = build_parser().parse_args(argv)
    dev = pick_device(a.device)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    data = make_dataset(a.data, device=dev, n_train=a.n_train, n_test=a.n_test, seed=a.seed)
    path = ckpt.client_ckpt_path(a.root, a.address)
    start_epoch, best_acc, init = 0, 0.0, None
    if a.resume:
        if not path.exists():
            raise SystemExit(f"--resume: no checkpoint at {path}")
        c = ckpt.load(path)
        init, best_acc, start_epoch = c["net"], float(c.get("acc", 0.0)), int(c.get("epoch", 0)) + 1
        log("train", f"Resuming from {path} (epoch {start_epoch - 1}, acc {best_acc:.2f})")
    trainer = build_trainer(a.model, data, dev, TrainerConfig(lr=a.lr, batch_size=a.batch_size, seed=a.seed),
                            init_state=init)
    full = data.train
    rng = np.random.default_rng(a.seed)
    metrics = MetricsLog(a.metrics)
    for epoch in range(start_epoch, start_epoch + a.epochs):
        if a.cosine:
            trainer.set_lr(cosine_lr(a.lr, epoch, a.t_max))
        if not a.no_shuffle:   # shuffled loader (src/main.py:51): permute the device-resident set
            trainer.set_train_data(full.subset(rng.permutation(len(full))))
        trainer.set_schedule(*contiguous_schedule(len(trainer.train_set), a.batch_size))
        t0 = time.perf_counter()
        trainer.train_epoch()
        trainer.evaluate()
        tr, te = trainer.train_stats(), trainer.eval_stats()
        dt = time.perf_counter() - t0
        log("train", f"Epoch {epoch}: train loss {tr.loss:.3f} acc {tr.acc:.2f}% | test loss {te.loss:.3f} "
                     f"acc {te.acc:.2f}% ({te.correct}/{te.count}) | {format_time(dt)}")
        metrics.write(epoch=epoch, lr=trainer.cfg.lr, epoch_s=dt, **tr.as_dict("train"), **te.as_dict("test"))
        if te.acc > best_acc:   # src/main.py:215-227
            log("train", "Saving..")
            Path(path).parent.mkdir(parents=True, exist_ok=True)
            ckpt.save(path, ckpt.make_checkpoint(trainer.state_dict(), acc=te.acc, epoch=epoch))
            best_acc = te.acc
    return 0


if __name__ == "__main__":
    sys.exit(main())
