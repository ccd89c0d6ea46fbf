"""Per-step time of the generic engine on zoo models without a whole-network native engine:
PyTorch fp32 (MIOpen / rocBLAS / ATen), PyTorch autocast-bf16 (the same-precision vendor baseline:
MIOpen / hipBLASLt bf16 kernels, mode ``torch-bf16``) vs the native aten backend (fedmi.ops.native_mode:
every op on fedmi's HIP kernels), eager and HIP-graph replayed.

    python tools/bench_hybrid.py [model ...]      -> one JSON line per (model, mode)
"""
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402

from fedmi.engine.base import TrainerConfig  # noqa: E402
from fedmi.engine.data import make_dataset  # noqa: E402
from fedmi.engine.torch_engine import TorchTrainer  # noqa: E402
from fedmi.models import build_model  # noqa: E402

MODELS = sys.argv[1:] or ["DenseNet121", "SENet18", "SimpleDLA", "DPN26", "RegNetX_200MF", "ResNeXt29_2x64d",
                          "EfficientNetB0", "ShuffleNetV2"]
dev = torch.device("cuda", 0)
data = make_dataset("synthetic-cifar10", device=dev, n_train=128 * 12, n_test=1000, seed=0)
for name in MODELS:
    init = build_model(name).state_dict()
    modes = ("fp32", "torch-bf16", "native-eager", "native-graph-nofuse", "native-graph")
    if os.environ.get("BENCH_MODES"):
        modes = tuple(os.environ["BENCH_MODES"].split(","))
    for mode in modes:
        tr = TorchTrainer(name, data, dev, TrainerConfig(seed=1), init_state=init, hybrid=mode.startswith("native"))
        tr.use_graph = "graph" in mode
        if mode == "torch-bf16":
            def run(x, m=tr.model):
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    return m(x).float()
            tr._run = run
        if tr.mode is not None:
            tr.mode.fuse = not mode.endswith("nofuse")     # BN -> ReLU / ReLU-bwd -> BN-bwd fusion
        tr.model.train()
        for i in range(3):
            tr.train_step(128 * i, 128)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 9
        for i in range(n):
            tr.train_step(128 * (3 + i), 128)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / n * 1e3
        tr.evaluate()
        print(json.dumps({"model": name, "mode": mode, "ms_per_step": round(ms, 3),
                          "fallbacks": dict(tr.mode.fallbacks) if tr.mode is not None else None,
                          "eval_acc": round(tr.eval_stats().acc, 2)}), flush=True)
        del tr
        torch.cuda.empty_cache()
