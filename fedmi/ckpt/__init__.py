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
import collections
import io
import os
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


def state_digest(net) -> str:
    """Hash of the bytes of every floating-point entry of a state dict (key order): an exact identity
    check that two processes hold the same model, independent of reduction order or thread count."""
    import hashlib

    h = hashlib.blake2b(digest_size=16)
    for k, v in net.items():
        if v.is_floating_point():
            h.update(k.encode())
            h.update(v.detach().to("cpu").contiguous().view(-1).view(torch.uint8).numpy().tobytes())
    return h.hexdigest()


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

    Coalescing (default): a checkpoint submitted for the same file(s) as one that
    is still queued (not yet picked up by the writer) REPLACES it -- the file holds
    the newest model either way (the reference overwrites ``checkpoint/<addr>.pth``
    and ``optimizedModel.pth`` every round, src/main.py:160-165,
    src/server.py:174-179), so a writer slower than the round cadence drops
    superseded intermediate rounds instead of back-pressuring the round loop
    (``submit`` never blocks on a full queue of same-path checkpoints).  ``flush``
    still guarantees that the newest submission is on disk.  ``coalesce=False``
    writes every submission in order (bounded queue, ``submit`` blocks when full).
    """

    def __init__(self, max_pending: int = 4, coalesce: bool = True):
        self._pending: "collections.deque" = collections.deque()
        self._cv = threading.Condition()
        self._busy = False
        self._closing = False
        self._max = max(1, int(max_pending))
        self._coalesce = coalesce
        self._err: Optional[BaseException] = None
        self._pool: Dict[tuple, list] = {}
        self._pin_lock = threading.Lock()
        self._t = threading.Thread(target=self._run, name="fedmi-ckpt-writer", daemon=True)
        self._t.start()
        self.written = 0          # files written
        self.submitted = 0        # submit()/submit_bytes() calls
        self.coalesced = 0        # queued checkpoints superseded before being written
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

    def _enqueue(self, item) -> None:
        kind, paths = item[0], item[1]
        key = (kind, tuple(str(p) for p in paths))
        stale = None
        with self._cv:
            if self._err:
                raise RuntimeError("checkpoint writer failed") from self._err
            self.submitted += 1
            if self._coalesce and paths and item[6] is None:
                for i, old in enumerate(self._pending):
                    if old[6] is None and (old[0], tuple(str(p) for p in old[1])) == key:
                        stale = old
                        self._pending[i] = item        # keep its place in the FIFO
                        self.coalesced += 1
                        break
            if stale is None:
                while len(self._pending) >= self._max and not self._err:
                    self._cv.wait()
                self._pending.append(item)
            self._cv.notify_all()
        if stale is not None:
            # its device->host copy precedes any later reuse of the buffers on the same stream
            self._recycle(stale[7])

    def submit(self, path, state_dict, acc=1, epoch: int = 0, on_done=None) -> None:
        """Queue ``{'net','acc','epoch'}`` for ``path`` (a path, a list of paths sharing one snapshot,
        or None: serialise only and hand the bytes to ``on_done(None, data)``).  Submissions with an
        ``on_done`` callback are never coalesced away."""
        if self._err:
            raise RuntimeError("checkpoint writer failed") from self._err
        snap, ev, pooled = self._snapshot(state_dict)
        paths = [] if path is None else [Path(p) for p in path] if isinstance(path, (list, tuple)) else [Path(path)]
        self._enqueue(("ckpt", paths, snap, ev, acc, epoch, on_done, pooled))

    def submit_bytes(self, path, data: bytes) -> None:
        """Queue an already-serialised checkpoint (e.g. a received model) for an atomic write."""
        self._enqueue(("bytes", [Path(path)], data, None, None, None, None, []))

    def _run(self):
        while True:
            with self._cv:
                while not self._pending and not self._closing:
                    self._cv.wait()
                if not self._pending:
                    return
                item = self._pending.popleft()
                self._busy = True
                self._cv.notify_all()
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
                with self._cv:
                    self._busy = False
                    self._cv.notify_all()

    def flush(self) -> None:
        with self._cv:
            while (self._pending or self._busy) and not self._err:
                self._cv.wait()
        if self._err:
            raise RuntimeError("checkpoint writer failed") from self._err

    def close(self) -> None:
        self.flush()
        with self._cv:
            self._closing = True
            self._cv.notify_all()
        self._t.join(timeout=10)


# --------------------------------------------------------------------------------------------
# Native per-round writer (csrc/runtime/ckpt_writer.cpp): no Python on the write path.

_EPOCH_SENTINEL = 0x5EED1234


def _zip_layout(blob: bytes):
    """(name -> (data_off, size, [crc field offsets])) for a stored (uncompressed) zip archive."""
    import struct
    import zipfile

    zf = zipfile.ZipFile(io.BytesIO(blob))
    eocd = blob.rfind(b"PK\x05\x06")
    if eocd < 0:
        raise ValueError("no end-of-central-directory record")
    n_ent, = struct.unpack_from("<H", blob, eocd + 10)
    cd_off, = struct.unpack_from("<I", blob, eocd + 16)
    if cd_off == 0xFFFFFFFF or n_ent == 0xFFFF:
        raise ValueError("zip64 archive: not supported by the native writer")
    cd_crc = {}
    o = cd_off
    for _ in range(n_ent):
        if struct.unpack_from("<I", blob, o)[0] != 0x02014B50:
            raise ValueError("bad central directory entry")
        fnl, exl, cml = struct.unpack_from("<HHH", blob, o + 28)
        cd_crc[blob[o + 46:o + 46 + fnl].decode("utf-8")] = o + 16
        o += 46 + fnl + exl + cml
    out = {}
    for info in zf.infolist():
        if info.compress_type != zipfile.ZIP_STORED or info.file_size != info.compress_size:
            raise ValueError(f"record {info.filename} is compressed")
        h = info.header_offset
        flag, = struct.unpack_from("<H", blob, h + 6)
        fnl, exl = struct.unpack_from("<HH", blob, h + 26)
        data = h + 30 + fnl + exl
        crcs = [cd_crc[info.filename]]
        if flag & 0x8:            # data descriptor after the data (optionally signed)
            end = data + info.file_size
            crcs.append(end + 4 if struct.unpack_from("<I", blob, end)[0] == 0x08074B50 else end)
        else:
            crcs.append(h + 14)
        out[info.filename] = (data, info.file_size, crcs)
    return out


class NativeCheckpointWriter:
    """One model's per-round checkpoint to a fixed set of files, written by a C++ thread.

    Built from the live state dict: a torch.save template (sentinel epoch) is made
    once and parsed into record offsets; every later ``submit`` is one async
    device->pinned copy per source storage + an event, and the C++ writer patches
    storages, epoch and CRC-32s into the template -- the same bytes torch.save
    writes.  Every submission is written in order; ``slots`` snapshot buffers
    bound how far the host may run ahead (``submit`` waits for a free one), or,
    with ``coalesce``, a submission that finds every slot taken supersedes the
    newest queued one.  Raises ``ValueError`` for state dicts it cannot map
    (mixed devices, non-contiguous tensors); :class:`RoundCheckpointWriter` then
    uses Python."""

    def __init__(self, paths, state_dict, acc=1, slots: int = 4, coalesce: bool = False, link: bool = False):
        from .. import native

        nat = native.require()
        items = [(k[7:] if k.startswith("module.") else k, v.detach()) for k, v in state_dict.items()]
        devs = {v.device.type for _, v in items}
        if len(devs) != 1 or not all(v.is_contiguous() for _, v in items):
            raise ValueError("native checkpoint writer needs contiguous tensors on one device type")
        self.device = devs.pop() == "cuda"
        self.acc = acc
        self.signature = self._signature(state_dict)
        # source storages -> snapshot segments (64-B aligned)
        spans: Dict[int, tuple] = {}
        for _, v in items:
            key = v.untyped_storage().data_ptr()
            a = v.storage_offset() * v.element_size()
            b = a + v.numel() * v.element_size()
            lo, hi = spans.get(key, (a, b))
            spans[key] = (min(lo, a), max(hi, b))
        segs, seg_of, snap = [], {}, 0
        for key, (lo, hi) in spans.items():
            seg_of[key] = (lo, snap)
            segs.append((key + lo, hi - lo, snap))
            snap += (hi - lo + 63) // 64 * 64
        # template: distinct byte patterns per tensor, so the storage-record mapping is checked
        g = torch.Generator().manual_seed(1234)
        net = OrderedDict()
        for i, (k, v) in enumerate(items):
            t = torch.empty(v.shape, dtype=v.dtype)
            if t.numel():
                t.view(-1).view(torch.uint8).copy_(torch.randint(0, 256, (v.numel() * v.element_size(),),
                                                                 generator=g, dtype=torch.uint8))
            net[k] = t
        blob = to_bytes({"net": net, "acc": acc, "epoch": _EPOCH_SENTINEL})
        lay = _zip_layout(blob)
        pkl = [n for n in lay if n.endswith("/data.pkl")]
        if len(pkl) != 1:
            raise ValueError("template has no data.pkl")
        p_off, p_len, p_crc = lay[pkl[0]]
        sent = b"J" + _EPOCH_SENTINEL.to_bytes(4, "little")
        at = blob.find(sent, p_off, p_off + p_len)
        if at < 0 or blob.find(sent, at + 1, p_off + p_len) >= 0:
            raise ValueError("epoch sentinel not found exactly once in data.pkl")
        recs = [(p_off, p_len, -1, p_crc)]
        prefix = pkl[0][: -len("data.pkl")]
        for i, (k, v) in enumerate(items):
            name = f"{prefix}data/{i}"
            if name not in lay:
                raise ValueError(f"storage record {name} missing")
            d_off, d_len, d_crc = lay[name]
            nb = v.numel() * v.element_size()
            ref = net[k].reshape(-1).view(torch.uint8).numpy().tobytes() if nb else b""
            if d_len != nb or blob[d_off:d_off + d_len] != ref:
                raise ValueError(f"storage record {name} does not hold tensor {k}")
            lo, s_off = seg_of[v.untyped_storage().data_ptr()]
            recs.append((d_off, d_len, s_off + v.storage_offset() * v.element_size() - lo, d_crc))
        self.paths = [str(Path(p)) for p in paths]
        for p in self.paths:
            Path(p).parent.mkdir(parents=True, exist_ok=True)
        self.w = nat.CkptWriter(blob, segs, recs, at + 1, self.paths, self.device, int(slots), bool(coalesce),
                                bool(link))
        self._stream = native.stream_handle if self.device else None

    @staticmethod
    def _signature(state_dict):
        return tuple((k, v.data_ptr(), tuple(v.shape), v.dtype, v.device) for k, v in state_dict.items())

    def matches(self, state_dict, acc) -> bool:
        return acc == self.acc and self._signature(state_dict) == self.signature

    def submit(self, epoch: int) -> None:
        if not -(1 << 31) <= int(epoch) < (1 << 31):
            raise ValueError("epoch must fit in int32")
        self.w.submit(self._stream() if self.device else 0, int(epoch))

    def flush(self) -> None:
        self.w.flush()

    @property
    def written(self) -> int:
        return int(self.w.written)

    @property
    def coalesced(self) -> int:
        return int(self.w.coalesced)


class RoundCheckpointWriter:
    """Per-round checkpoints (same files every round): the native writer where the state dict
    maps onto it, else :class:`AsyncCheckpointWriter`.  Every round is written unless
    ``coalesce`` (then a host that outruns the writer by ``slots`` rounds supersedes queued
    rounds instead of waiting).  Every target is an independent file unless ``link`` (opt-in, only
    for target sets in directories fedmi owns alone): then the native writer writes the bytes once
    and hard-links the other targets -- a peer that rewrites one of them in place (the reference's
    torch.save) would then change the others too.  FEDMI_NATIVE_CKPT=0 forces the Python writer."""

    def __init__(self, slots: int = 4, coalesce: bool = False, link: bool = False):
        self.slots, self.coalesce, self.link = slots, coalesce, link
        self._native: Dict[tuple, NativeCheckpointWriter] = {}
        self._py: Optional[AsyncCheckpointWriter] = None
        self.backend = None
        self._retired = [0, 0]          # (written, coalesced) of writers already torn down

    def _retire(self, w: "NativeCheckpointWriter") -> None:
        w.flush()
        self._retired[0] += w.written
        self._retired[1] += w.coalesced

    def _python(self) -> AsyncCheckpointWriter:
        if self._py is None:
            self._py = AsyncCheckpointWriter(max_pending=self.slots, coalesce=self.coalesce)
        return self._py

    def submit(self, path, state_dict, acc=1, epoch: int = 0) -> None:
        paths = tuple(str(p) for p in (path if isinstance(path, (list, tuple)) else [path]))
        if os.environ.get("FEDMI_NATIVE_CKPT", "1") != "0":
            w = self._native.get(paths)
            if w is not None and not w.matches(state_dict, acc):
                self._retire(self._native.pop(paths))
                w = None
            if w is None:
                try:
                    w = NativeCheckpointWriter(paths, state_dict, acc, self.slots, self.coalesce, self.link)
                    self._native[paths] = w
                except (ValueError, RuntimeError):
                    w = None
            if w is not None:
                # another writer covering one of these files must land first, or its older round could
                # overwrite this one (the writers run independently)
                for k, o in self._native.items():
                    if k != paths and set(k) & set(paths):
                        o.flush()
                self.backend = "native"
                w.submit(epoch)
                return
        self.backend = "python"
        self._python().submit(list(paths), state_dict, acc=acc, epoch=epoch)

    def flush(self) -> None:
        for w in self._native.values():
            w.flush()
        if self._py is not None:
            self._py.flush()

    def close(self) -> None:
        self.flush()
        for k in list(self._native):
            self._retire(self._native.pop(k))
        if self._py is not None:
            self._py.close()

    @property
    def written(self) -> int:
        return (self._retired[0] + sum(w.written for w in self._native.values())
                + (self._py.written if self._py else 0))

    @property
    def coalesced(self) -> int:
        return (self._retired[1] + sum(w.coalesced for w in self._native.values())
                + (self._py.coalesced if self._py else 0))
