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
    coordinator may run for millions of rounds); the file has all of them.

    ``background=True`` (the client agents): ``write`` only queues the record; a writer thread
    serialises and appends it, so a leased round's bookkeeping stays off the round loop (the thread
    mostly runs while the caller waits on the GPU).  ``flush`` / ``close`` drain the queue."""

    def __init__(self, path: Optional[str | Path] = None, echo: bool = False, keep: int = 1024,
                 background: bool = False):
        self.path = Path(path) if path else None
        self.echo = echo
        self._lock = threading.Lock()
        self.records: deque = deque(maxlen=keep)
        self.count = 0
        self._f = None
        if self.path:
            self.path.parent.mkdir(parents=True, exist_ok=True)
            self._f = open(self.path, "a", buffering=1)      # line-buffered: readable while running
        self._q: Optional[deque] = None
        if background and (self._f is not None or echo):
            self._q = deque()
            self._cv = threading.Condition()
            self._pending = 0
            self._stop = False
            self._thr = threading.Thread(target=self._drain, name="metrics-writer", daemon=True)
            self._thr.start()

    def write(self, **rec) -> dict:
        rec.setdefault("ts", time.time())
        if self._q is not None:
            with self._lock:
                self.records.append(rec)
                self.count += 1
            with self._cv:
                self._q.append(rec)
                self._pending += 1
                self._cv.notify()
            return rec
        line = json.dumps(rec, default=float)
        with self._lock:
            self.records.append(rec)
            self.count += 1
            self._emit(line)
        return rec

    def _emit(self, line: str) -> None:
        if self._f is not None:
            self._f.write(line + "\n")
        if self.echo:
            print(line, flush=True)

    def _drain(self) -> None:
        while True:
            with self._cv:
                while not self._q and not self._stop:
                    self._cv.wait()
                if not self._q and self._stop:
                    return
                batch = list(self._q)
                self._q.clear()
            lines = []
            for r in batch:
                try:
                    lines.append(json.dumps(r, default=float))
                except (TypeError, ValueError) as e:   # never let one bad record stop the writer
                    lines.append(json.dumps({"event": "metrics_error", "error": str(e)[:200], "ts": r.get("ts")}))
            with self._lock:
                for line in lines:
                    self._emit(line)
            with self._cv:
                self._pending -= len(batch)
                self._cv.notify_all()

    def flush(self, timeout: float = 10.0) -> None:
        """Wait until every queued record is written (background mode; a no-op otherwise)."""
        if self._q is None:
            return
        with self._cv:
            self._cv.wait_for(lambda: self._pending == 0, timeout=timeout)

    def close(self) -> None:
        if self._q is not None:
            self.flush()
            with self._cv:
                self._stop = True
                self._cv.notify_all()
            self._thr.join(timeout=10.0)
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
