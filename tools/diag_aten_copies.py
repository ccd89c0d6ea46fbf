"""Find where a native-mode step still launches an ATen kernel: profile one eager step with Python
stacks and print every ATen op that owns a GPU kernel, with its shapes and the innermost frames.

    python tools/diag_aten_copies.py RegNetX_200MF
"""
import sys

import torch
from torch.profiler import ProfilerActivity, profile

from fedmi.engine import build_trainer
from fedmi.engine.base import TrainerConfig
from fedmi.engine.data import make_dataset


def main(name: str) -> None:
    dev = torch.device("cuda:0")
    data = make_dataset("synthetic-cifar10", device=dev, n_train=256, n_test=64, seed=0)
    tr = build_trainer(name, data, dev, TrainerConfig(batch_size=128, seed=1, augment=False))
    tr.use_graph = False
    x, y = tr._batch(0, 128)
    tr.model.train()
    tr._step_body(x, y)
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True,
                 record_shapes=True) as prof:
        tr._step_body(x, y)
        torch.cuda.synchronize()
    seen = set()
    for e in prof.events():
        if e.device_type != torch.autograd.DeviceType.CPU or not e.name.startswith("aten::"):
            continue
        kern = [k.name for k in e.kernels if "at::native" in k.name]
        if not kern:
            continue
        stack = tuple(s for s in (e.stack or []) if "fedmi" in s or "models" in s)[:6]
        key = (e.name, str(e.input_shapes), stack)
        if key in seen:
            continue
        seen.add(key)
        print(e.name, e.input_shapes, kern[0][:80])
        for s in stack:
            print("    ", s)
    print("fallbacks:", dict(tr.mode.fallbacks))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "RegNetX_200MF")
