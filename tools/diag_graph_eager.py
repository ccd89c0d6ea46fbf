"""Native-mode trainer: eager vs eager (run-to-run) vs graph-replayed, per-tensor max |diff| after K steps."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402

from fedmi.engine import build_trainer  # noqa: E402
from fedmi.engine.base import TrainerConfig  # noqa: E402
from fedmi.engine.data import contiguous_schedule, make_dataset  # noqa: E402
from fedmi.models import build_model  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "SimpleDLA"
dev = torch.device("cuda", 0)
data = make_dataset("synthetic-cifar10", device=dev, n_train=640, n_test=64, seed=0)
cfg = TrainerConfig(batch_size=128, lr=0.02, seed=7, augment=False)
init = build_model(name).state_dict()
runs = {}
for tag, graph in (("eager1", False), ("eager2", False), ("graph", True)):
    tr = build_trainer(name, data, dev, cfg, init_state=init)
    tr.use_graph = graph
    tr.set_schedule(*contiguous_schedule(640, 128))
    for _ in range(2):
        tr.train_epoch()
    runs[tag] = ({k: v.detach().float().clone() for k, v in tr.model.state_dict().items()}, tr.train_stats().loss)
ref = runs["eager1"][0]
for tag in ("eager2", "graph"):
    sd, loss = runs[tag]
    worst = sorted(((float((sd[k] - ref[k]).abs().max()), k, float(ref[k].abs().max())) for k in ref), reverse=True)[:5]
    print(tag, "loss", loss, "vs", runs["eager1"][1])
    for d, k, m in worst:
        print(f"   {k}: max|diff| {d:.4g} (max|ref| {m:.4g})")
