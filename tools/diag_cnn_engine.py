"""Unit-by-unit comparison of the native CNN engine with the PyTorch fp32 model:
conv output z (forward) and dL/dz (backward) for every conv of the network.

    python tools/diag_cnn_engine.py MobileNet [nb]
"""
from __future__ import annotations

import sys
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from fedmi.engine.base import TrainerConfig  # noqa: E402
from fedmi.engine.cnn_native import CNNNativeTrainer  # noqa: E402
from fedmi.engine.data import augment_normalize, make_dataset  # noqa: E402
from fedmi.models import build_model  # noqa: E402


def cos(a, b):
    return float(F.cosine_similarity(a.flatten().double(), b.flatten().double(), dim=0))


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "MobileNet"
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    dev = torch.device("cuda", 0)
    data = make_dataset("synthetic-cifar10", device=dev, n_train=64, n_test=64, seed=0)
    tr = CNNNativeTrainer(name, data, dev, TrainerConfig(batch_size=nb, augment=False, use_graph=False))
    init = {k: v.detach().clone() for k, v in tr.state_dict().items()}
    tr.grads_for_batch(0, nb)
    torch.cuda.synchronize()
    ref = build_model(name).to(dev)
    ref.load_state_dict(init)
    ref.train()
    zs, gz = {}, {}
    names = {m: n for n, m in ref.named_modules()}

    def fhook(mod, inp, out):
        n = names[mod]
        zs[n] = out
        out.register_hook(lambda g, n=n: gz.__setitem__(n, g))

    for m in ref.modules():
        if isinstance(m, torch.nn.Conv2d):
            m.register_forward_hook(fhook)
    x = augment_normalize(data.train.x[:nb], None, 0, 0)
    loss = F.cross_entropy(ref(x), data.train.y[:nb].long())
    loss.backward()
    conv_name = {id(m): n for n, m in tr.model.named_modules()}
    print(f"{'conv':36s} {'fwd cos':>9s} {'bwd cos':>9s} {'bwd norm':>9s}")
    for u in tr.units:
        n = conv_name[id(u.conv)]
        z = u.view(u.z, nb).float().permute(0, 3, 1, 2)
        dz = u.view(u.dz, nb).float().permute(0, 3, 1, 2)
        r, g = zs[n].detach(), gz[n]
        print(f"{n:36s} {cos(z, r):9.5f} {cos(dz, g):9.5f} {float(dz.norm() / g.norm()):9.4f}")


if __name__ == "__main__":
    main()
