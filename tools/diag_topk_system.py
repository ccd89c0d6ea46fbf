"""Diagnose the -c Y system-test failure: the top-k compressor on real LeNet deltas in one process, with
guard tensors around idx / val and a check of the trainer's stats words after every step."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from fedmi.engine import build_trainer  # noqa: E402
from fedmi.engine.base import TrainerConfig  # noqa: E402
from fedmi.engine.data import make_dataset, strided_schedule  # noqa: E402
from fedmi.parallel.compress import TopKCompressor  # noqa: E402

dev = torch.device("cuda", 0)
data = make_dataset("synthetic-cifar10", device=dev, n_train=2560, n_test=1000, seed=0)
tr = build_trainer("lenet", data, dev, TrainerConfig(seed=1))
tr.set_schedule(*strided_schedule(2560, 128, 0, 2))
comp = TopKCompressor(tr, 0.01)
# idx / val inside larger buffers: entries past k must stay untouched
big_idx = torch.full((comp.k + 256,), -7, dtype=torch.int32, device=dev)
big_val = torch.full((comp.k + 256,), -7.0, device=dev)
comp.idx, comp.val = big_idx[:comp.k], big_val[:comp.k]
guard = torch.full((4096,), 7, dtype=torch.int32, device=dev)
for rnd in range(4):
    tr.train_epoch()
    raw = tr.stats.cpu().tolist()
    print("round", rnd, "stats after train", raw, flush=True)
    comp.compress(tr.float_state())
    torch.cuda.synchronize()
    idx = comp.idx.cpu()
    ok = bool((idx >= 0).all() and (idx < comp.n).all()) and len(set(idx.tolist())) == comp.k
    tail_ok = bool((big_idx[comp.k:] == -7).all() and (big_val[comp.k:] == -7.0).all())
    flag = int(comp.state[8212:8216].view(torch.int32).item())
    print("  payload tail untouched", tail_ok, "overflow flag", flag, flush=True)
    print("  topk idx ok", ok, "min", int(idx.min()), "max", int(idx.max()), "unique", len(set(idx.tolist())),
          "k", comp.k, "guard intact", bool((guard == 7).all()), flush=True)
    tr.evaluate()
    ev = tr.eval_stats()
    raw = tr.stats.cpu().tolist()
    print("  stats after eval", raw, "eval", ev, flush=True)
    try:
        print("  train stats", tr.train_stats(), flush=True)
    except Exception as e:
        print("  train_stats raised:", e, flush=True)
