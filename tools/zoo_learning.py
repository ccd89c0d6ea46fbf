"""Learning curves of the zoo families on the native aten backend vs the PyTorch fp32 engine.

    python tools/zoo_learning.py [model ...] [--seeds 0 1 2] [--lr 0.02] [--epochs 4]
      -> one JSON line per (model, seed, engine): per-epoch train loss / acc and the final test
         accuracy, synthetic-cifar10-easy (class-structured), both engines from the same init.
"""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402

from fedmi.engine import build_trainer  # noqa: E402
from fedmi.engine.base import TrainerConfig  # noqa: E402
from fedmi.engine.data import contiguous_schedule, make_dataset  # noqa: E402
from fedmi.engine.torch_engine import TorchTrainer  # noqa: E402
from fedmi.models import build_model  # noqa: E402

import argparse  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("models", nargs="*", default=["ResNeXt29_2x64d", "ResNeXt29_32x4d", "DPN26", "densenet_cifar",
                                              "SENet18", "EfficientNetB0", "RegNetX_200MF", "RegNetY_400MF",
                                              "ShuffleNetG2", "ShuffleNetV2", "PNASNetA", "DLA", "SimpleDLA"])
ap.add_argument("--seeds", type=int, nargs="*", default=[0], help="model-init / trainer seeds (one run each)")
ap.add_argument("--epochs", type=int, default=4)
ap.add_argument("--lr", type=float, default=0.02)
args = ap.parse_args()
dev = torch.device("cuda", 0)
data = make_dataset("synthetic-cifar10-easy", device=dev, n_train=2560, n_test=1000, seed=0)
for name in args.models:
    for seed in args.seeds:
        cfg = TrainerConfig(batch_size=128, lr=args.lr, seed=7 + seed)
        torch.manual_seed(seed)
        init = build_model(name).state_dict()
        for kind in ("native", "fp32"):
            tr = (build_trainer(name, data, dev, cfg, init_state=init) if kind == "native"
                  else TorchTrainer(name, data, dev, cfg, init_state=init))
            tr.set_schedule(*contiguous_schedule(len(data.train), 128))
            t0 = time.perf_counter()
            curve = []
            for _ in range(args.epochs):
                tr.train_epoch()
                st = tr.train_stats()
                curve.append([round(st.loss, 4), round(st.acc, 2)])
            tr.evaluate()
            ev = tr.eval_stats()
            torch.cuda.synchronize()
            print(json.dumps({"model": name, "engine": kind, "seed": seed, "lr": args.lr, "epochs": curve,
                              "test_acc": round(ev.acc, 2), "test_loss": round(ev.loss, 4),
                              "wall_s": round(time.perf_counter() - t0, 2),
                              "fallbacks": (dict(tr.mode.fallbacks) if getattr(tr, "mode", None) is not None
                                            else None)}), flush=True)
            del tr
            torch.cuda.empty_cache()
