"""Checkpoint format, directory layout and an asynchronous writer.

Format (byte-compatible with the reference): ``torch.save({'net': state_dict,
'acc': number, 'epoch': int})`` with un-prefixed keys and CPU fp32 tensors
(src/main.py:160-165, src/server.py:174-179).  fedmi stores the real round in
``epoch`` so a promoted backup or restarted coordinator resumes instead of
restarting at round 0 (reference quirk A8, src/server.py:64 TODO).

Layout (relative to the process CWD or an explicit root):
  coordinator:  Primary/ | Backup/  ->  test_<rank>.pth, optimizedModel.pth
  client:       checkpoint/<address>.pth
"""
from __future__ import annotations

import base64
import io
import os
import queue
import threading
from collections import OrderedDict
from pathlib import Path
from typing import Dict, Optional

import torch

OPTIMIZED_MODEL = "optimizedModel.pth"


def mount_dir(root: Path | str, primary: bool) -> Path:
    d = Path(root) / ("Primary" if primary else "Backup")
    d.mkdir(parents=True, exist_ok=True)
    return d


def client_ckpt_path(root: Path | str, address: str) -> Path:
    d = Path(root) / "checkpoint"
    d.mkdir(parents=True, exist_ok=True)          # reference crashes if missing (quirk A13)
    return d / f"{address}.pth"


def make_checkpoint(state_dict, acc=1, epoch: int = 0) -> dict:
    net = OrderedDict()
    for k, v in state_dict.items():
        k = k[7:] if k.startswith("module.") else k   # never DataParallel-prefixed (quirk A1)
        net[k] = v.detach().to("cpu", copy=True).contiguous()
    return {"net": net, "acc": acc, "epoch": int(epoch)}


def to_bytes(ckpt: dict) -> bytes:
    buf = io.BytesIO()
    torch.save(ckpt, buf)
    return buf.getvalue()


def from_bytes(data: bytes) -> dict:
    # weights_only: never execute anything from a checkpoint received over the wire
    return torch.load(io.BytesIO(data), map_location="cpu", weights_only=True)


def to_b64(data: bytes) -> str:
    return base64.b64encode(data).decode("ascii")


def from_b64(text) -> bytes:
    return base64.b64decode(text)


def atomic_write(path: Path | str, data: bytes) -> None:
    path = Path(path)
    path.parent.mkdir(parents=True, exist_ok=True)
    tmp = path.with_name(path.name + f".tmp{os.getpid()}.{threading.get_ident()}")
    with open(tmp, "wb") as f:
        f.write(data)
    os.replace(tmp, path)


def save(path: Path | str, ckpt: dict) -> None:
    atomic_write(path, to_bytes(ckpt))


def load(path: Path | str) -> dict:
    with open(path, "rb") as f:
        return from_bytes(f.read())


def read_epoch(path: Path | str) -> Optional[int]:
    try:
        return int(load(path).get("epoch", 0))
    except (FileNotFoundError, RuntimeError, EOFError, ValueError):
        return None


class AsyncCheckpointWriter:
    """Serialise + write checkpoints off the critical path.

    ``submit`` snapshots the device tensors into pinned host memory with a
    non-blocking copy on the current stream and records an event; the writer
    thread waits for that event, then ``torch.save``s atomically.  The GPU
    stream never blocks on file I/O.  Pinned snapshot buffers are pooled per
    (storage span, dtype) and recycled once the writer has serialised them, so a
    per-round checkpoint allocates no pinned memory in steady state.
    """

    def __init__(self, max_pending: int = 4):
        self._q: "queue.Queue" = queue.Queue(maxsize=max_pending)
        self._err: Optional[BaseException] = None
        self._pool: Dict[tuple, list] = {}
        self._pin_lock = threading.Lock()
        self._t = threading.Thread(target=self._run, name="fedmi-ckpt-writer", daemon=True)
        self._t.start()
        self.written = 0
        self.pinned_allocs = 0

    def _pinned(self, key: tuple, n: int, dtype) -> torch.Tensor:
        with self._pin_lock:
            free = self._pool.get(key)
            if free:
                return free.pop()
        self.pinned_allocs += 1
        return torch.empty(n, dtype=dtype, pin_memory=True)

    def _recycle(self, bufs) -> None:
        with self._pin_lock:
            for key, b in bufs:
                self._pool.setdefault(key, []).append(b)

    def _snapshot(self, state_dict):
        """Device->pinned-host copy of a state dict: ONE copy per device storage.

        State dicts of the fedmi engines are views into one flat fp32 buffer;
        copying the covered span once replaces a copy (+ pinned alloc) per
        tensor.  The writer thread later clones every view into its own storage
        so the file layout is the reference's (one storage per tensor)."""
        out = OrderedDict()
        ev = None
        pooled = []
        groups: Dict[tuple, list] = {}
        for k, v in state_dict.items():
            v = v.detach()
            if v.is_cuda and v.is_contiguous():
                key = (v.untyped_storage().data_ptr(), v.dtype, v.device)
                groups.setdefault(key, []).append((k, v))
                out[k] = None
            elif v.is_cuda:
                host = torch.empty(v.shape, dtype=v.dtype, pin_memory=True)
                host.copy_(v, non_blocking=True)
                out[k] = host
            else:
                out[k] = v.clone()
        for (ptr, dt, dev), items in groups.items():
            lo = min(v.storage_offset() for _, v in items)
            hi = max(v.storage_offset() + v.numel() for _, v in items)
            base = torch.empty(0, dtype=dt, device=dev).set_(items[0][1].untyped_storage())
            pkey = (ptr, lo, hi, dt)
            host = self._pinned(pkey, hi - lo, dt)
            host.copy_(base[lo:hi], non_blocking=True)
            pooled.append((pkey, host))
            for k, v in items:
                o = v.storage_offset() - lo
                out[k] = host[o:o + v.numel()].view(v.shape)
        if any(v.is_cuda for v in state_dict.values()):
            ev = torch.cuda.Event()
            ev.record()
        return out, ev, pooled

    def submit(self, path, state_dict, acc=1, epoch: int = 0, on_done=None) -> None:
        """Queue ``{'net','acc','epoch'}`` for ``path`` (a path, a list of paths sharing one snapshot,
        or None: serialise only and hand the bytes to ``on_done(None, data)``)."""
        if self._err:
            raise RuntimeError("checkpoint writer failed") from self._err
        snap, ev, pooled = self._snapshot(state_dict)
        paths = [] if path is None else [Path(p) for p in path] if isinstance(path, (list, tuple)) else [Path(path)]
        self._q.put(("ckpt", paths, snap, ev, acc, epoch, on_done, pooled))

    def submit_bytes(self, path, data: bytes) -> None:
        """Queue an already-serialised checkpoint (e.g. a received model) for an atomic write."""
        if self._err:
            raise RuntimeError("checkpoint writer failed") from self._err
        self._q.put(("bytes", [Path(path)], data, None, None, None, None, []))

    def _run(self):
        while True:
            item = self._q.get()
            if item is None:
                self._q.task_done()
                return
            kind, paths, snap, ev, acc, epoch, on_done, pooled = item
            try:
                if kind == "bytes":
                    for path in paths:
                        atomic_write(path, snap)
                        self.written += 1
                    continue
                if ev is not None:
                    ev.synchronize()
                # one storage per tensor, like a plain module.state_dict()
                net = OrderedDict((k, v.clone() if v.untyped_storage().nbytes() != v.nbytes else v)
                                  for k, v in snap.items())
                data = to_bytes({"net": net, "acc": acc, "epoch": int(epoch)})
                self._recycle(pooled)
                for path in paths:
                    atomic_write(path, data)
                    self.written += 1
                if on_done is not None:
                    on_done(paths[0] if paths else None, data)
            except BaseException as e:  # pragma: no cover
                self._err = e
            finally:
                self._q.task_done()

    def flush(self) -> None:
        self._q.join()
        if self._err:
            raise RuntimeError("checkpoint writer failed") from self._err

    def close(self) -> None:
        self.flush()
        self._q.put(None)
        self._t.join(timeout=10)
