"""Per-phase cycle breakdown of the fused LeNet step (diagnostic stamps build).

Run with FEDMI_NATIVE_VARIANT=stamps (the -DFEDMI_STAMPS extension).  Executes a
few warm-up steps, then one eager step of 128 samples, and prints, per kernel,
the median (and max) cycles each workgroup spent in every phase, plus the
spread of workgroup start times.
"""
import os
import sys
from pathlib import Path

os.environ.setdefault("FEDMI_NATIVE_VARIANT", "stamps")
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from fedmi import native  # noqa: E402
from fedmi.engine.base import TrainerConfig  # noqa: E402
from fedmi.engine.data import make_dataset  # noqa: E402
from fedmi.engine.lenet_native import LeNetNativeTrainer  # noqa: E402


def main():
    nat = native.require()
    assert nat.stamps_enabled(), "not the stamps build"
    dev = torch.device("cuda", 0)
    ds = make_dataset("synthetic-cifar10", device=dev, n_train=4096, n_test=1024)
    tr = LeNetNativeTrainer(ds, dev, TrainerConfig(seed=1))
    nat.set_ks1_diag(int(os.environ.get("FEDMI_KS1_DIAG", "0")))   # staging probes (sample path)
    for i in range(8):
        tr.train_step(128 * i, 128)
    torch.cuda.synchronize()
    nat.read_stamps(True)
    tr.train_step(0, 128)
    torch.cuda.synchronize()
    st = np.frombuffer(nat.read_stamps(True), dtype=np.uint64).reshape(nat.STAMP_SHAPE).astype(np.int64)
    if True:   # KS1 + KS2 (the only training path)
        # KS1: forward slots 0..6 under kernel 0, its backward slots 2..5 under kernel 2; KS2 under kernel 3
        ks1 = np.concatenate([st[0, :128, :7], st[2, :128, 2:6]], axis=1)
        phases = ["stage+aug", "conv1", "pool1", "conv2", "pool2+zero+shift", "fc fwd+bwd", "dY2 scatter",
                  "c2 wgrad+dgrad", "c1 wgrad", "slab store"]
        a = ks1[ks1[:, 0] > 0]
        d = np.diff(a, axis=1)
        tot = a[:, -1] - a[:, 0]
        print(f"sample    wgs={len(a):4d} total med {np.median(tot):8.0f} max {tot.max():8.0f} cyc")
        for j, ph in enumerate(phases):
            print(f"    {ph:16s} med {np.median(d[:, j]):8.0f}  max {d[:, j].max():8.0f}")
        f = st[1, :128]
        f = f[(f[:, 0] > 0)]
        k0 = st[0, :128]
        k0 = k0[k0[:, 0] > 0]
        if len(f) and len(k0):
            print(f"    stage loads landed med {np.median(k0[:len(f), 0] * 0 + f[:, 7] - k0[:len(f), 0]):8.0f}")
            fcn = ["fc1+h1T", "fc2", "fc3|shift build", "CE", "dH2", "dH1"]
            prev = k0[:len(f), 5]
            for j, nm in enumerate(fcn):
                print(f"    fc.{nm:14s} med {np.median(f[:, j] - prev):8.0f}")
                prev = f[:, j]
            print(f"    fc.dX          med {np.median(k0[:len(f), 6] - prev):8.0f}")
        b2 = st[2, :128]
        b2 = b2[b2[:, 2] > 0]
        if len(b2) and (b2[:, 6] > 0).all():
            print(f"    bwd: dY2 scatter->dgrad MFMAs done (wave 0) med {np.median(b2[:, 6] - b2[:, 2]):8.0f}  "
                  f"pool1 bwd scatter med {np.median(b2[:, 7] - b2[:, 6]):8.0f}  -> barrier med {np.median(b2[:, 3] - b2[:, 7]):8.0f}")
        names = {3: ("sgd2", ["all"])}
        nwg = {3: 249}
        # KS2 by role (lenet_sgd2 block ranges): conv slab combine, fc1 / fc2 / fc3 weight tiles, biases + loss
        k2 = st[3, :249, :2]
        dur = k2[:, 1] - k2[:, 0]
        t0 = k2[k2[:, 0] > 0, 0].min()
        for role, lo, hi in (("conv slab", 0, 180), ("fc1 tiles", 180, 230), ("fc2 tiles", 230, 242),
                             ("fc3 tiles", 242, 244), ("bias+loss", 244, 249)):
            d = dur[lo:hi]
            end = k2[lo:hi, 1] - t0
            print(f"    sgd2 {role:10s} med {np.median(d):8.0f}  max {d.max():8.0f}  last end {end.max():8.0f}")
        f1 = st[3, 180:230, :4]
        f1 = f1[f1[:, 2] > 0]
        if len(f1):
            print(f"    sgd2 fc1 split: start->operands+MFMA med {np.median(f1[:, 2] - f1[:, 0]):8.0f}  "
                  f"SGD stores issued med {np.median(f1[:, 3] - f1[:, 2]):8.0f}  -> end med {np.median(f1[:, 1] - f1[:, 3]):8.0f}")
    for k, (name, phases) in names.items():
        a = st[k, :nwg[k], :len(phases) + 1]
        a = a[a[:, 0] > 0]
        d = np.diff(a, axis=1)
        tot = a[:, -1] - a[:, 0]
        starts = a[:, 0] - a[:, 0].min()
        print(f"{name:9s} wgs={len(a):4d} total med {np.median(tot):8.0f} max {tot.max():8.0f} cyc | "
              f"start spread {starts.max():7d} cyc")
        for j, ph in enumerate(phases):
            print(f"    {ph:16s} med {np.median(d[:, j]):8.0f}  max {d[:, j].max():8.0f}")


if __name__ == "__main__":
    main()
