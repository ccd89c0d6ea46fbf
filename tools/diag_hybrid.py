"""Hybrid engine eager vs graph: losses, eval accuracy and BN running-stat norms per mode.
python tools/diag_hybrid.py SimpleDLA"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402

from fedmi.engine.base import TrainerConfig  # noqa: E402
from fedmi.engine.data import contiguous_schedule, make_dataset  # noqa: E402
from fedmi.engine.torch_engine import TorchTrainer  # noqa: E402
from fedmi.models import build_model  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "SimpleDLA"
dev = torch.device("cuda", 0)
data = make_dataset("synthetic-cifar10-easy", device=dev, n_train=1280, n_test=500, seed=0)
init = build_model(name).state_dict()
for mode in ("fp32", "hyb-eager", "hyb-graph"):
    tr = TorchTrainer(name, data, dev, TrainerConfig(batch_size=128, lr=0.02, seed=7, use_graph=mode == "hyb-graph"),
                      init_state=init, hybrid=mode != "fp32")
    tr.set_schedule(*contiguous_schedule(len(data.train), 128))
    losses = []
    for _ in range(3):
        tr.train_epoch()
        losses.append(round(tr.train_stats().loss, 4))
    tr.evaluate()
    sd = tr.state_dict()
    rm = sum(float(v.float().norm()) for k, v in sd.items() if k.endswith("running_mean"))
    rv = sum(float(v.float().norm()) for k, v in sd.items() if k.endswith("running_var"))
    nbt = [int(v) for k, v in sd.items() if k.endswith("num_batches_tracked")][:3]
    tr.model.train()
    with torch.no_grad():
        x, y = tr._batch(0, 128)
        acc_train_mode = float((tr._run(x).argmax(1) == y).float().mean())
    print(mode, "losses", losses, "eval", tr.eval_stats().acc, "rm", round(rm, 3), "rv", round(rv, 3), "nbt", nbt,
          "train-mode-acc(batch0)", acc_train_mode, flush=True)
