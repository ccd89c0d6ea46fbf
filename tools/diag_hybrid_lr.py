"""Hybrid engine stability at the reference lr (0.1): per-epoch-chunk loss for fp32 / hybrid eager /
hybrid graph on the bench's synthetic data.  python tools/diag_hybrid_lr.py SENet18 [n_train]"""
import math
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402

from fedmi.engine.base import TrainerConfig  # noqa: E402
from fedmi.engine.data import make_dataset  # noqa: E402
from fedmi.engine.torch_engine import TorchTrainer  # noqa: E402
from fedmi.models import build_model  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "SENet18"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 128 * 60
dev = torch.device("cuda", 0)
data = make_dataset("synthetic-cifar10", device=dev, n_train=n, n_test=500, seed=0)
init = build_model(name).state_dict()
MODES = sys.argv[3].split(",") if len(sys.argv) > 3 else ["fp32", "hyb-eager", "hyb-graph"]
for mode in MODES:
    # *-nchw: NCHW input; hyb-graph-nomiopen: MIOpen off (PyTorch's own BN / conv kernels) ; bf16-graph: native convs removed
    torch.backends.cudnn.enabled = mode != "hyb-graph-nomiopen"
    tr = TorchTrainer(name, data, dev, TrainerConfig(lr=0.02 if mode.endswith("lr02") else 0.1, seed=1,
                                                     use_graph="graph" in mode),
                      init_state=init, hybrid=not mode.startswith("fp32"))
    tr.use_graph = "graph" in mode
    if "meanpool" in mode:                    # SE global pool as an fp32 mean instead of adaptive_avg_pool2d
        import torch.nn.functional as F
        from fedmi.models.zoo import residual as _res

        class _F:
            def __getattr__(self, k):
                return getattr(F, k)

            @staticmethod
            def adaptive_avg_pool2d(x, out):
                return x.float().mean((2, 3), keepdim=True).to(x.dtype)
        _res.F = _F()
    torch.backends.cuda.preferred_blas_library("cublas" if "rocblas" in mode else "default")
    if "fp32linear" in mode:                  # classifier GEMMs outside autocast
        import types
        from torch import nn

        def _lin(self, x):
            with torch.autocast("cuda", enabled=False):
                return nn.functional.linear(x.float(), self.weight, self.bias)
        for m in tr.model.modules():
            if isinstance(m, nn.Linear):
                m.forward = types.MethodType(_lin, m)
    if "nchw" in mode:                       # keep the network input NCHW (no channels-last propagation)
        tr._layout = lambda x: x
    if mode == "bf16-graph":
        for m in tr.model.modules():
            m.__dict__.pop("forward", None)
    tr.model.train()
    out = []
    steps = n // 128
    for j in range(2 * steps):
        i = j % steps
        loss = tr.train_step(128 * i, 128)
        if "sync" in mode:                    # host waits for every replay (no launch run-ahead)
            torch.cuda.synchronize()
        if j % 30 == 29:
            v = float(loss.detach())
            out.append(round(v, 3))
            if not math.isfinite(v):
                break
    bad = [k for k, v in tr.state_dict().items() if v.is_floating_point() and not torch.isfinite(v).all()]
    print(mode, out, "nonfinite:", bad[:5], flush=True)
