"""roctx ranges around the federated round's phases.

``with phase("local-train"):`` pushes a roctx range (``torch.cuda.nvtx`` is
roctx on ROCm builds), so ``rocprofv3 --marker-trace`` shows the round split
into local-train / allreduce / eval / checkpoint / rpc next to the kernels.
Ranges are on by default when a GPU is present; ``FEDMI_ROCTX=0`` disables
them, ``FEDMI_ROCTX=1`` forces them on.  A range costs ~1 µs of host time.
"""
from __future__ import annotations

import contextlib
import os

import torch

_enabled = None


def enabled() -> bool:
    global _enabled
    if _enabled is None:
        flag = os.environ.get("FEDMI_ROCTX")
        if flag is not None:
            _enabled = flag == "1"
        else:
            _enabled = torch.cuda.is_available()
    return _enabled


@contextlib.contextmanager
def phase(name: str):
    if not enabled():
        yield
        return
    torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        torch.cuda.nvtx.range_pop()


def mark(name: str) -> None:
    if enabled():
        torch.cuda.nvtx.mark(name)
