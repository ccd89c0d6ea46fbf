"""LeNet local trainer on the fused HIP kernels + native hipGraph executor.

Device memory is allocated through PyTorch (caching allocator) and handed to
``_fedmi_native.LeNetEngine`` as raw pointers.  Per round the host issues:
one graph launch (the whole local epoch: 2 kernels x #owned batches -- KS1
``lenet_sample_step`` and KS2 ``lenet_sgd2``, csrc/kernels/lenet_kernels.hip), the
FedAvg all-reduce on :meth:`float_state`, one pack launch, and three eval
launches — no per-step host synchronisation (the reference syncs twice per
step via ``.item()``, src/main.py:153-156).
"""
from __future__ import annotations

from collections import OrderedDict
from typing import List, Optional

import dataclasses

import torch

from .. import native
from ..models.small import LeNet
from .base import EpochStats, LocalTrainer, TrainerConfig, ordered_views
from .data import FedDataset, ImageSet

LENET_SPEC = [
    ("conv1.weight", (6, 3, 5, 5)), ("conv1.bias", (6,)),
    ("conv2.weight", (16, 6, 5, 5)), ("conv2.bias", (16,)),
    ("fc1.weight", (120, 400)), ("fc1.bias", (120,)),
    ("fc2.weight", (84, 120)), ("fc2.bias", (84,)),
    ("fc3.weight", (10, 84)), ("fc3.bias", (10,)),
]


def _ptr(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else int(t.data_ptr())


class LeNetNativeTrainer(LocalTrainer):
    model_name = "lenet"

    def __init__(self, data: FedDataset, device: torch.device, cfg: TrainerConfig = TrainerConfig(),
                 init_state=None):
        if device.type != "cuda":
            raise ValueError("LeNetNativeTrainer runs on a GPU (use TorchTrainer on CPU)")
        if tuple(data.train.x.shape[1:]) != (3, 32, 32):
            raise ValueError("LeNet native engine expects 3x32x32 uint8 images")
        nat = native.require()
        self._nat = nat
        self.L = L = nat.lenet_layout()
        self.cfg = dataclasses.replace(cfg)   # private copy: set_lr mutates it
        self._device = device
        self.round_idx = 0
        with torch.cuda.device(device):
            self.train_set = data.train.to(device)
            self.test_set = data.test.to(device)
            if self.train_set.y.dtype != torch.int32:
                self.train_set.y = self.train_set.y.to(torch.int32)
            if self.test_set.y.dtype != torch.int32:
                self.test_set.y = self.test_set.y.to(torch.int32)
            z = lambda *s, dt=torch.float32: torch.zeros(*s, dtype=dt, device=device)  # noqa: E731
            B = L["MAX_TRAIN_BATCH"]
            self.params = z(L["P_TOTAL"])
            self.mom = z(L["P_TOTAL"])
            self.pk = z(L["PK_TOTAL"], dt=torch.bfloat16)
            self.act2_rows = max(B, len(self.test_set))
            self.act2 = z(self.act2_rows, L["F0P"], dt=torch.bfloat16)   # eval activations (pool2 output)
            self.act2T = z(L["F0P"], B, dt=torch.bfloat16)               # KS1 -> KS2 operands
            self.h1 = z(B, 128, dt=torch.bfloat16)
            self.dact2 = z(B, L["F0"])                                  # KS1's FC side buffers
            self.dZ1T = z(L["DZ1_LD"], B, dt=torch.bfloat16)
            self.conv_slab = z(B, L["CS"])
            self.eval_part = z(2 * ((self.act2_rows + L["FC_SPW"] - 1) // L["FC_SPW"]))
            self.stats = z(2, 4, dt=torch.int32)       # [train, eval] x {loss_f32, correct, count, pad}
            self.round_ctr = z(4, dt=torch.int32)
        self._bufs = dict(
            train_images=_ptr(self.train_set.x), train_labels=_ptr(self.train_set.y), n_train=len(self.train_set),
            params=_ptr(self.params), mom=_ptr(self.mom), pk=_ptr(self.pk), act2=_ptr(self.act2),
            act2_rows=self.act2_rows, act2T=_ptr(self.act2T), h1=_ptr(self.h1), dact2=_ptr(self.dact2),
            dZ1T=_ptr(self.dZ1T), conv_slab=_ptr(self.conv_slab), eval_part=_ptr(self.eval_part),
            eval_part_floats=self.eval_part.numel(), train_stats=_ptr(self.stats[0]),
            eval_stats=_ptr(self.stats[1]), round_ctr=_ptr(self.round_ctr))
        self.engine = nat.LeNetEngine(self._bufs, cfg.lr, cfg.momentum, cfg.weight_decay, cfg.seed & 0xFFFFFFFF,
                                      bool(data.augment and cfg.augment))
        self._views = ordered_views(self.params, LENET_SPEC)
        if init_state is None:
            torch.manual_seed(cfg.seed)
            init_state = LeNet().state_dict()
        self.load_state_dict(init_state)
        self._starts: List[int] = []
        self._sizes: List[int] = []

    # ---- state -------------------------------------------------------------------
    @property
    def device(self) -> torch.device:
        return self._device

    def _stream(self) -> int:
        return native.stream_handle(self._device)

    def state_dict(self):
        return OrderedDict(self._views)

    def load_state_dict(self, sd) -> None:
        for name, _ in LENET_SPEC:
            src = sd[name]
            self._views[name].copy_(src.to(self._device, torch.float32).view(self._views[name].shape))
        self.after_aggregate()

    def float_state(self) -> torch.Tensor:
        return self.params

    def after_aggregate(self) -> None:
        self.engine.pack(self._stream())

    def momentum_state(self) -> torch.Tensor:
        return self.mom

    # ---- schedule -------------------------------------------------------------
    def set_schedule(self, starts, sizes) -> None:
        starts, sizes = list(map(int, starts)), list(map(int, sizes))
        if (starts, sizes) != (self._starts, self._sizes):
            self.engine.set_schedule(starts, sizes)
            self._starts, self._sizes = starts, sizes

    def set_train_data(self, data: ImageSet) -> None:
        """Replace the client's local training set (e.g. a non-IID shard); rebuilds the engine binding."""
        self.train_set = data.to(self._device)
        if self.train_set.y.dtype != torch.int32:
            self.train_set.y = self.train_set.y.to(torch.int32)
        self._bufs.update(train_images=_ptr(self.train_set.x), train_labels=_ptr(self.train_set.y),
                          n_train=len(self.train_set))
        self.engine = self._nat.LeNetEngine(self._bufs, self.cfg.lr, self.cfg.momentum, self.cfg.weight_decay,
                                            self.cfg.seed & 0xFFFFFFFF, bool(self.cfg.augment))
        self._starts, self._sizes = [], []

    # ---- compute ----------------------------------------------------------------
    def train_epoch(self) -> None:
        self.engine.run_epoch(self._stream(), bool(self.cfg.use_graph))
        if self._starts:
            self.round_idx += 1

    def train_step(self, start: int, nb: int, bump_round: bool = False) -> None:
        self.engine.step(self._stream(), int(start), int(nb), bool(bump_round))

    def _read_stats(self, i: int) -> EpochStats:
        return self.decode_stats(self.stats[i].cpu())

    def decode_stats(self, raw: torch.Tensor) -> EpochStats:
        # lenet::Stats: {float loss_sum, int correct, int count, pad} in an int32[4] row
        raw = raw.contiguous()
        return EpochStats(float(raw[0:1].view(torch.float32).item()), int(raw[1]), int(raw[2]))

    def eval_stats_raw(self) -> torch.Tensor:
        return self.stats[1]

    def train_stats(self) -> EpochStats:
        return self._read_stats(0)

    def evaluate(self) -> None:
        self.engine.eval(self._stream(), _ptr(self.test_set.x), _ptr(self.test_set.y), len(self.test_set))

    def eval_stats(self) -> EpochStats:
        return self._read_stats(1)

    def reset_momentum(self) -> None:
        self.mom.zero_()

    def set_lr(self, lr: float) -> None:
        """New learning rate (re-captures the epoch graph on the next train_epoch)."""
        self.cfg.lr = float(lr)
        self.engine.set_sgd(self.cfg.lr, self.cfg.momentum, self.cfg.weight_decay)
