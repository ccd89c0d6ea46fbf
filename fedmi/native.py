"""Loader for the in-tree native extension ``fedmi/_fedmi_native*.so``.

On a GPU the HIP path is mandatory: :func:`require` raises if the extension is
missing or fails to load, so a GPU run never silently falls back to PyTorch.
On CPU-only hosts (unit tests of the control plane) the native module is
optional and :func:`available` reports whether it could be imported.
"""
from __future__ import annotations

import importlib
import os
import threading

import torch

_lock = threading.Lock()
_mod = None
_err: Exception | None = None


def _load():
    global _mod, _err
    with _lock:
        if _mod is not None or _err is not None:
            return
        variant = os.environ.get("FEDMI_NATIVE_VARIANT", "")
        name = "fedmi._fedmi_native" + (f"_{variant}" if variant else "")
        try:
            mod = importlib.import_module(name)
            from .ops.conv import STAT_REP

            if getattr(mod, "STAT_REP", STAT_REP) != STAT_REP:
                raise ImportError(f"{name}: STAT_REP {mod.STAT_REP} != fedmi.ops.conv.STAT_REP {STAT_REP}")
            _mod = mod
        except Exception as e:  # pragma: no cover - depends on build state
            _err = e


def available() -> bool:
    _load()
    return _mod is not None


def require():
    """Return the native module or raise loudly (never fall back on a GPU)."""
    _load()
    if _mod is None:
        raise RuntimeError(
            "fedmi native extension is not built or failed to load "
            f"({_err!r}); run `python -m fedmi._build` (hipcc, gfx950)")
    return _mod


def stream_handle(device: torch.device | None = None) -> int:
    """Raw hipStream_t of torch's current stream (launches stay stream-ordered)."""
    return int(torch.cuda.current_stream(device).cuda_stream)


def stream_handle_of(stream: "torch.cuda.Stream") -> int:
    """Raw hipStream_t of a given torch stream."""
    return int(stream.cuda_stream)


def on_gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


def force_torch_path() -> bool:
    """Debug switch (FEDMI_TORCH_PATH=1): run the pure-PyTorch reference engine on GPU."""
    return os.environ.get("FEDMI_TORCH_PATH", "0") == "1"
