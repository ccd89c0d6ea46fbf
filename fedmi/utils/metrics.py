"""Structured per-round metrics (JSONL) and timestamped console logging.

The reference prints unstructured lines and progress bars only
(src/main.py:124-125,158-159; src/server.py:121,130,148) and under-reports the
train loss by ~world x (loss summed over owned batches but divided by ALL batch
indices, src/main.py:158-159, quirk A10).  fedmi reports per-round means over
the samples actually trained, plus timings, as one JSON object per line.
"""
from __future__ import annotations

import json
import sys
import threading
import time
from collections import deque
from pathlib import Path
from typing import Optional


class MetricsLog:
    """JSONL sink.  ``records`` keeps only the newest ``keep`` records in memory (a
    coordinator may run for millions of rounds); the file has all of them."""

    def __init__(self, path: Optional[str | Path] = None, echo: bool = False, keep: int = 1024):
        self.path = Path(path) if path else None
        self.echo = echo
        self._lock = threading.Lock()
        self.records: deque = deque(maxlen=keep)
        self.count = 0
        self._f = None
        if self.path:
            self.path.parent.mkdir(parents=True, exist_ok=True)
            self._f = open(self.path, "a", buffering=1)      # line-buffered: readable while running

    def write(self, **rec) -> dict:
        rec.setdefault("ts", time.time())
        line = json.dumps(rec, default=float)
        with self._lock:
            self.records.append(rec)
            self.count += 1
            if self._f is not None:
                self._f.write(line + "\n")
            if self.echo:
                print(line, flush=True)
        return rec

    def close(self) -> None:
        with self._lock:
            if self._f is not None:
                self._f.close()
                self._f = None


def log(role: str, msg: str, stream=None) -> None:
    t = time.strftime("%H:%M:%S") + f".{int(time.time() * 1000) % 1000:03d}"
    print(f"[{t}] [{role}] {msg}", file=stream or sys.stdout, flush=True)


class Timer:
    def __init__(self):
        self.t0 = time.perf_counter()

    def ms(self) -> float:
        return (time.perf_counter() - self.t0) * 1e3
