"""Flat-buffer kernels (csrc/kernels/flat_ops.hip): multi-tensor SGD over one
fp32 parameter buffer, weighted FedAvg reduce of K buffers, in-place scale.

These replace the reference's per-tensor optimizer ops (src/main.py:147-151)
and its CPU Python FedAvg loop (src/server.py:155-179).
"""
from __future__ import annotations

from typing import Sequence

import torch

from .. import native


def sgd_(p: torch.Tensor, g: torch.Tensor, mom: torch.Tensor, lr: float, momentum: float = 0.9,
         weight_decay: float = 5e-4, dampening: float = 0.0, nesterov: bool = False, first: bool = False) -> None:
    """torch.optim.SGD step on flat fp32 buffers (``first``: momentum buffer initialised to d)."""
    for t in (p, g, mom):
        if t.dtype != torch.float32 or not t.is_contiguous() or t.numel() != p.numel():
            raise ValueError("sgd_: flat contiguous fp32 buffers of equal size required")
    native.require().sgd_flat(native.stream_handle(p.device), p.data_ptr(), g.data_ptr(), mom.data_ptr(), p.numel(),
                              lr, momentum, weight_decay, dampening, nesterov, first)


def fedavg_reduce(inputs: Sequence[torch.Tensor], weights: Sequence[float], out: torch.Tensor) -> torch.Tensor:
    """out = sum_k weights[k] * inputs[k] (one launch, <= fedavg_max_inputs() inputs)."""
    nat = native.require()
    if len(inputs) != len(weights) or not 1 <= len(inputs) <= nat.fedavg_max_inputs():
        raise ValueError("fedavg_reduce: bad input count")
    for t in inputs:
        if t.numel() != out.numel() or t.dtype != torch.float32:
            raise ValueError("fedavg_reduce: size/dtype mismatch")
    nat.fedavg_reduce(native.stream_handle(out.device), [t.data_ptr() for t in inputs], [float(w) for w in weights],
                      out.data_ptr(), out.numel())
    return out


def scale_(x: torch.Tensor, alpha: float) -> torch.Tensor:
    native.require().scale(native.stream_handle(x.device), x.data_ptr(), x.numel(), float(alpha))
    return x
