#!/usr/bin/env python
"""Where the per-round checkpoint time goes on this host: the native writer's sustained rate (submit as
fast as it accepts) with 1 and 2 target files, in $TMPDIR and /dev/shm, plus the raw cost of one
250 KB tmp-write + rename and of the event-synchronised D2H snapshot.  One JSON line per case."""
from __future__ import annotations

import json
import os
import sys
import tempfile
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tools.bench_ckpt_writer import lenet_state  # noqa: E402


def main() -> int:
    from fedmi.ckpt import RoundCheckpointWriter

    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    flat, sd = lenet_state(dev)
    for base in (tempfile.gettempdir(), "/dev/shm"):
        root = Path(tempfile.mkdtemp(prefix="ckio_", dir=base))
        paths = [root / "Primary" / "optimizedModel.pth", root / "checkpoint" / "client0.pth"]
        for p in paths:
            p.parent.mkdir(parents=True, exist_ok=True)
        for npaths in (1, 2):
            w = RoundCheckpointWriter()
            w.submit(paths[:npaths], sd, acc=1, epoch=0)
            w.flush()
            n = 300
            t = time.perf_counter()
            for r in range(n):
                w.submit(paths[:npaths], sd, acc=1, epoch=r + 1)
            w.flush()
            ms = (time.perf_counter() - t) / n * 1e3
            w.close()
            print(json.dumps({"case": "native_writer_max_rate", "dir": base, "paths": npaths,
                              "ms_per_round": round(ms, 4)}), flush=True)
        b = os.urandom(248024)
        t = time.perf_counter()
        for i in range(300):
            tmp = root / "raw.tmp"
            with open(tmp, "wb") as f:
                f.write(b)
            os.replace(tmp, root / "raw")
        print(json.dumps({"case": "python_write_rename_250KB", "dir": base,
                          "ms": round((time.perf_counter() - t) / 300 * 1e3, 4)}), flush=True)
    if dev.type == "cuda":
        pin = torch.empty(flat.numel(), dtype=torch.float32, pin_memory=True)
        ev = torch.cuda.Event()
        t = time.perf_counter()
        for _ in range(300):
            pin.copy_(flat, non_blocking=True)
            ev.record()
            ev.synchronize()
        print(json.dumps({"case": "d2h_248KB_event_sync", "ms": round((time.perf_counter() - t) / 300 * 1e3, 4)}),
              flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
