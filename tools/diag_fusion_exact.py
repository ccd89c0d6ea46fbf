"""Fused vs unfused native-mode training step of one zoo model (the setup of
tests/test_native_mode_gpu.py::test_bn_relu_fusion_is_exact): prints every parameter whose weights differ
after the step, with its max |diff|, in state-dict order.
  python tools/diag_fusion_exact.py [model]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from fedmi.engine import build_trainer  # noqa: E402
from fedmi.engine.base import TrainerConfig  # noqa: E402
from fedmi.engine.data import make_dataset  # noqa: E402
from fedmi.models import build_model  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "densenet_cifar"
dev = torch.device("cuda:0")
data = make_dataset("synthetic-cifar10", device=dev, n_train=128, n_test=64, seed=0)
cfg = TrainerConfig(batch_size=64, lr=0.02, seed=7, augment=False, use_graph=False)
init = build_model(name).state_dict()
res = {}
for fuse in (False, True):
    tr = build_trainer(name, data, dev, cfg, init_state=init)
    tr.use_graph = False
    tr.mode.fuse = fuse
    tr.set_schedule([0], [64])          # one step: the first diverging gradient shows directly
    tr.train_epoch()
    torch.cuda.synchronize()
    res[fuse] = {k: v.detach().float().clone() for k, v in tr.state_dict().items()}
n = 0
for k, a in res[False].items():
    b = res[True][k]
    if not torch.equal(a, b):
        d = (a - b).abs()
        print(f"DIFF {k} {tuple(a.shape)} max {d.max().item():.3e} count {(d > 0).sum().item()}")
        n += 1
print(f"{name}: {n} of {len(res[False])} entries differ")
