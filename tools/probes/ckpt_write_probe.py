"""Probe: wall time of ONE per-round checkpoint write of the LeNet state (the native writer: pinned snapshot,
pickle/zip template, CRC, tmp + rename per target), device idle -- the tail bench.py's timed region pays once
after the last round.  Targets: bench.py's pair (Primary/optimizedModel.pth + the client checkpoint) in a
mkdtemp directory (bench.py's default) and in the working directory; independent files vs hard links.

    python tools/probes/ckpt_write_probe.py
"""
import json
import sys
import tempfile
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

import torch  # noqa: E402

from fedmi.ckpt import RoundCheckpointWriter  # noqa: E402
from fedmi.engine import build_trainer  # noqa: E402
from fedmi.engine.base import TrainerConfig  # noqa: E402
from fedmi.engine.data import make_dataset  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    data = make_dataset("synthetic-cifar10", device=dev, n_train=256, n_test=128, seed=0)
    tr = build_trainer("lenet", data, dev, TrainerConfig(seed=1))
    sd = tr.state_dict()
    roots = {"mkdtemp": Path(tempfile.mkdtemp(prefix="fedmi_probe_")),
             "cwd": Path(tempfile.mkdtemp(prefix="fedmi_probe_", dir=str(Path.cwd())))}
    for where, root in roots.items():
        (root / "Primary").mkdir(exist_ok=True)
        (root / "checkpoint").mkdir(exist_ok=True)
        paths = [root / "Primary" / "optimizedModel.pth", root / "checkpoint" / "client0.pth"]
        for link in (False, True):
            w = RoundCheckpointWriter(slots=4, link=link)
            ts = []
            for r in range(30):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                w.submit(paths, sd, acc=1, epoch=r)
                w.flush()
                ts.append((time.perf_counter() - t0) * 1e3)
            ts = sorted(ts[5:])
            print(json.dumps({"dir": where, "link": link, "backend": w.backend, "median_ms": round(ts[len(ts) // 2], 3),
                              "min_ms": round(ts[0], 3), "max_ms": round(ts[-1], 3),
                              "bytes": paths[0].stat().st_size}), flush=True)


if __name__ == "__main__":
    main()
