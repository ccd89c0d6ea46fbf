"""Local-trainer interface shared by the fused-HIP LeNet engine and the generic
PyTorch engine.

A *local trainer* is the on-device replacement for the reference's import-time
singleton ``main.py`` (src/main.py:20-242): it owns the model state, the
optimizer state (momentum persists across rounds, src/main.py:99-100,134), the
client's data and its shard schedule, and exposes one local epoch
(``train(epoch, rank, world)``, src/main.py:128-165) and one evaluation pass
(``test(epoch, count)``, src/main.py:167-191).
"""
from __future__ import annotations

import abc
from collections import OrderedDict
from dataclasses import dataclass
from typing import List

import torch


@dataclass
class EpochStats:
    loss_sum: float = 0.0
    correct: int = 0
    count: int = 0

    @property
    def loss(self) -> float:
        return self.loss_sum / max(1, self.count)

    @property
    def acc(self) -> float:
        return 100.0 * self.correct / max(1, self.count)

    def as_dict(self, prefix: str) -> dict:
        return {f"{prefix}_loss": self.loss, f"{prefix}_acc": self.acc, f"{prefix}_samples": self.count}


@dataclass
class TrainerConfig:
    lr: float = 0.1                # src/main.py:21
    momentum: float = 0.9          # src/main.py:99
    weight_decay: float = 5e-4     # src/main.py:100
    batch_size: int = 128          # src/main.py:51,140
    eval_batch_size: int = 1000
    seed: int = 0
    augment: bool = True
    use_graph: bool = True


class LocalTrainer(abc.ABC):
    """Device-resident local training engine of one federated client."""

    model_name: str = ""
    round_idx: int = 0                     # local epochs completed (augmentation RNG key)

    # --- state -----------------------------------------------------------------
    @abc.abstractmethod
    def state_dict(self) -> "OrderedDict[str, torch.Tensor]":
        """Reference-compatible state dict (un-prefixed keys, device tensors, views)."""

    @abc.abstractmethod
    def load_state_dict(self, sd) -> None:
        ...

    @abc.abstractmethod
    def float_state(self) -> torch.Tensor:
        """One flat fp32 tensor holding every averaged floating entry (params + float buffers)."""

    def int_state(self) -> List[torch.Tensor]:
        """Integer buffers (BN num_batches_tracked) averaged with truncation like the reference."""
        return []

    def after_aggregate(self) -> None:
        """Called after float_state() was overwritten (FedAvg / load)."""

    # --- data --------------------------------------------------------------------
    @abc.abstractmethod
    def set_schedule(self, starts: List[int], sizes: List[int]) -> None:
        ...

    # --- compute -----------------------------------------------------------------
    @abc.abstractmethod
    def train_epoch(self) -> None:
        """Enqueue one local epoch over the schedule (asynchronous on GPU)."""

    @abc.abstractmethod
    def train_stats(self) -> EpochStats:
        ...

    @abc.abstractmethod
    def evaluate(self) -> None:
        """Enqueue evaluation over the client's test set."""

    @abc.abstractmethod
    def eval_stats(self) -> EpochStats:
        ...

    def set_test_data(self, data) -> None:
        """Replace the evaluation set (e.g. this client's slice of a data-parallel eval)."""
        es = self.eval_stream()
        if es is not None:
            es.synchronize()                   # an overlapped eval may still read the old set
        t = data.to(self.device)
        if self.device.type == "cuda" and t.y.dtype != torch.int32:
            t.y = t.y.to(torch.int32)          # native engines read int32 labels
        self.test_set = t

    def eval_stats_raw(self) -> torch.Tensor:
        """Device-resident eval accumulator of the last :meth:`evaluate` (engine-specific layout);
        :meth:`decode_stats` turns a host copy of it into :class:`EpochStats`.  Valid on
        :meth:`eval_stream` (device consumers order themselves after it)."""
        raise NotImplementedError

    def eval_stream(self):
        """The stream :meth:`evaluate` runs on when it overlaps later work (None: the current stream)."""
        return None

    def decode_stats(self, raw: torch.Tensor) -> EpochStats:
        raise NotImplementedError

    @property
    @abc.abstractmethod
    def device(self) -> torch.device:
        ...

    def set_lr(self, lr: float) -> None:
        raise NotImplementedError

    def synchronize(self) -> None:
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)


def ordered_views(flat: torch.Tensor, spec) -> "OrderedDict[str, torch.Tensor]":
    out = OrderedDict()
    off = 0
    for name, shape in spec:
        n = 1
        for s in shape:
            n *= s
        out[name] = flat[off:off + n].view(shape)
        off += n
    return out
