#!/usr/bin/env python
"""Per-parameter gradient parity of the native CNN engine: native vs native (determinism), native vs
its PyTorch-twin emulation (tests/emulate.py, same schedule and bf16 buffers), native vs fp32 PyTorch.
Prints, per model, min / median cosine and the tensors under 0.99.

  python tools/diag_engine_parity.py ResNet18 MobileNet [--warm K]   (--warm: K SGD steps first)
"""
import argparse
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from fedmi.engine.base import TrainerConfig  # noqa: E402
from fedmi.engine.data import augment_normalize, contiguous_schedule, make_dataset  # noqa: E402
from fedmi.models import build_model  # noqa: E402


def cos(a, b):
    return float(F.cosine_similarity(a.flatten().double(), b.flatten().double(), dim=0))


def grads(name, data, dev, init, emulate=False, nb=64):
    from fedmi.engine.cnn_native import CNNNativeTrainer

    cfg = TrainerConfig(batch_size=nb, augment=False, use_graph=False)
    if emulate:
        from emulate import emulated
        with emulated():
            tr = CNNNativeTrainer(name, data, dev, cfg, init_state=init)
            tr.grads_for_batch(0, nb)
            tr.grads_for_batch(0, nb)
    else:
        tr = CNNNativeTrainer(name, data, dev, cfg, init_state=init)
        tr.grads_for_batch(0, nb)
        tr.grads_for_batch(0, nb)
    torch.cuda.synchronize()
    return {k: p.grad.detach().clone() for k, p in tr.model.named_parameters()}


def torch_grads(name, data, dev, init, nb=64):
    ref = build_model(name).to(dev)
    ref.load_state_dict(init)
    ref.train()
    x = augment_normalize(data.train.x[:nb], None, 0, 0)
    with torch.no_grad():
        ref(x)
    F.cross_entropy(ref(x), data.train.y[:nb].long()).backward()
    return {k: p.grad.detach().clone() for k, p in ref.named_parameters()}


def summary(tag, a, b):
    cs = {k: cos(a[k], b[k]) for k in a}
    low = sorted((v, k) for k, v in cs.items() if v < 0.99)
    print(f"  {tag}: min {min(cs.values()):.4f} median {statistics.median(cs.values()):.4f} "
          f"<0.99: {len(low)}/{len(cs)} {[(k, round(v, 3)) for v, k in low[:6]]}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("models", nargs="*", default=["ResNet18", "MobileNet", "MobileNetV2"])
    ap.add_argument("--warm", type=int, default=0, help="native SGD steps before the comparison")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    data = make_dataset("synthetic-cifar10", device=dev, n_train=2560, n_test=64, seed=0)
    for name in a.models:
        init = build_model(name).state_dict()
        if a.warm:
            from fedmi.engine.cnn_native import CNNNativeTrainer
            tr = CNNNativeTrainer(name, data, dev, TrainerConfig(batch_size=128, lr=0.02), init_state=init)
            tr.set_schedule(*contiguous_schedule(128 * a.warm, 128))
            tr.train_epoch()
            init = {k: v.detach().cpu().clone() for k, v in tr.state_dict().items()}
        print(f"{name} (warm {a.warm} steps)", flush=True)
        g1 = grads(name, data, dev, init)
        g2 = grads(name, data, dev, init)
        same = sum(torch.equal(g1[k], g2[k]) for k in g1)
        print(f"  native vs native: {same}/{len(g1)} tensors bit-identical", flush=True)
        summary("native vs emulated", g1, grads(name, data, dev, init, emulate=True))
        summary("native vs fp32 torch", g1, torch_grads(name, data, dev, init))


if __name__ == "__main__":
    main()
