"""Run K graph-replayed training steps of one zoo model on the native aten backend (for rocprofv3).

    rocprofv3 --kernel-trace --stats -d gpurun_out/p -- python tools/prof_native_mode.py RegNetY_400MF 10
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402

from fedmi.engine.base import TrainerConfig  # noqa: E402
from fedmi.engine.data import make_dataset  # noqa: E402
from fedmi.engine.torch_engine import TorchTrainer  # noqa: E402

name = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
dev = torch.device("cuda", 0)
data = make_dataset("synthetic-cifar10", device=dev, n_train=128 * 4, n_test=128, seed=0)
tr = TorchTrainer(name, data, dev, TrainerConfig(seed=1, augment=False), hybrid=True)
tr.mode.diag = True
tr.model.train()
for i in range(steps):
    tr.train_step(128 * (i % 4), 128)
torch.cuda.synchronize()
print(name, "fallbacks", dict(tr.mode.fallbacks), "fused", dict(tr.mode.fused), flush=True)
for k, v in tr.mode.scalar_ew.most_common(12):
    print("scalar ew", v, k, flush=True)
for k, v in tr.mode.ew_ops.most_common(24):
    print("ew op", v, k, flush=True)
