#!/usr/bin/env python
"""Plain PyTorch fp32 training of a zoo model on the bench's synthetic data (no fedmi kernels):
the numerics reference for "does this model train at the reference's recipe on this data".

    python tools/diag_fp32_reference.py <model> [epochs] [lr]

Same recipe as the reference (src/main.py:99-100: SGD lr 0.1, momentum 0.9, wd 5e-4, batch 128,
RandomCrop+HFlip+Normalize); prints the running train loss every 50 steps and the test accuracy
per epoch, and whether the loss went non-finite.
"""
import math
import sys
import time
from pathlib import Path

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

from fedmi.engine.data import augment_normalize, make_dataset  # noqa: E402
from fedmi.models import build_model  # noqa: E402


def main():
    name = sys.argv[1]
    epochs = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    lr = float(sys.argv[3]) if len(sys.argv) > 3 else 0.1
    dev = torch.device("cuda", 0)
    ds = make_dataset("synthetic-cifar10", device=dev, n_train=50000, n_test=10000, seed=0)
    torch.manual_seed(17)
    m = build_model(name).to(dev)
    opt = torch.optim.SGD(m.parameters(), lr=lr, momentum=0.9, weight_decay=5e-4)
    n = len(ds.train.y)
    for ep in range(epochs):
        m.train()
        t0, run, k, bad = time.perf_counter(), 0.0, 0, None
        for i, s in enumerate(range(0, n, 128)):
            idx = np.arange(s, min(n, s + 128))
            x = augment_normalize(ds.train.x[s:s + len(idx)], idx, 17, ep)
            loss = F.cross_entropy(m(x), ds.train.y[s:s + len(idx)].long())
            opt.zero_grad()
            loss.backward()
            opt.step()
            v = loss.item()
            if not math.isfinite(v) and bad is None:
                bad = i
            run += v
            k += 1
            if (i + 1) % 50 == 0:
                print(f"[{name}] epoch {ep} step {i + 1}: loss {run / k:.4f}", flush=True)
                run, k = 0.0, 0
        m.eval()
        correct = 0
        with torch.no_grad():
            for s in range(0, len(ds.test.y), 500):
                x = augment_normalize(ds.test.x[s:s + 500], None, 0, 0)
                correct += int((m(x).argmax(1) == ds.test.y[s:s + 500].long()).sum())
        print(f"[{name}] epoch {ep}: test acc {100.0 * correct / len(ds.test.y):.2f} %, first non-finite step "
              f"{bad}, {time.perf_counter() - t0:.1f} s", flush=True)


if __name__ == "__main__":
    main()
