"""LeNet local trainer on the fused HIP kernels + native hipGraph executor.

Device memory is allocated through PyTorch (caching allocator) and handed to
``_fedmi_native.LeNetEngine`` as raw pointers.  Per round the host issues:
one graph launch (the whole local epoch: 4 kernels x #owned batches), the
FedAvg all-reduce on :meth:`float_state`, one pack launch, and two eval
launches — no per-step host synchronisation (the reference syncs twice per
step via ``.item()``, src/main.py:153-156).
"""
from __future__ import annotations

from collections import OrderedDict
from typing import List, Optional

import dataclasses
import os

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
            self.act2 = z(self.act2_rows, L["F0P"], dt=torch.bfloat16)
            self.act2T = z(L["F0P"], B, dt=torch.bfloat16)
            self.h1 = z(self.act2_rows + 16, 128, dt=torch.bfloat16)
            self.pool1 = z(B, L["NP1"], dt=torch.bfloat16)
            self.am1 = z(B, L["NP1"], dt=torch.uint8)
            self.am2 = z(B, L["F0"], dt=torch.uint8)
            self.dact2 = z(B, L["F0"])
            self.dZ1T = z(L["DZ1_LD"], B, dt=torch.bfloat16)
            self.conv_slab = z(B, L["CS"])
            self.fc1w_grad = z(L["F1W_N"])
            self.fc_slab = z(L["MAX_FC_WG"], L["FS"])
            self.stats = z(2, 4, dt=torch.int32)       # [train, eval] x {loss_f32, correct, count, pad}
            self.round_ctr = z(4, dt=torch.int32)
            self.done_flags = z(B, dt=torch.int32)       # K12 conv -> FC-head hand-off flags (step generations)
            self.step_gen = z(4, dt=torch.int32)
            self.bwd_flags = z(B + L["N_DW1_WG"], dt=torch.int32)   # K34 producer -> SGD hand-off flags
            self.bwd_gen = z(4, dt=torch.int32)
        self._bufs = dict(
            train_images=_ptr(self.train_set.x), train_labels=_ptr(self.train_set.y), n_train=len(self.train_set),
            params=_ptr(self.params), mom=_ptr(self.mom), pk=_ptr(self.pk), act2=_ptr(self.act2),
            act2_rows=self.act2_rows, act2T=_ptr(self.act2T), h1=_ptr(self.h1), pool1=_ptr(self.pool1), am1=_ptr(self.am1),
            am2=_ptr(self.am2), dact2=_ptr(self.dact2), dZ1T=_ptr(self.dZ1T), conv_slab=_ptr(self.conv_slab),
            fc1w_grad=_ptr(self.fc1w_grad), fc_slab=_ptr(self.fc_slab), train_stats=_ptr(self.stats[0]), eval_stats=_ptr(self.stats[1]),
            round_ctr=_ptr(self.round_ctr), done_flags=_ptr(self.done_flags), step_gen=_ptr(self.step_gen),
            bwd_flags=_ptr(self.bwd_flags), bwd_gen=_ptr(self.bwd_gen))
        self.engine = nat.LeNetEngine(self._bufs, cfg.lr, cfg.momentum, cfg.weight_decay, cfg.seed & 0xFFFFFFFF,
                                      bool(data.augment and cfg.augment))
        self.fuse_fc1 = os.environ.get("FEDMI_LENET_FUSE_FC1", "1") == "1"
        self._configure_engine()
        self._views = ordered_views(self.params, LENET_SPEC)
        if init_state is None:
            torch.manual_seed(cfg.seed)
            init_state = LeNet().state_dict()
        self.load_state_dict(init_state)
        self._starts: List[int] = []
        self._sizes: List[int] = []
        # opt-in: measured slower (91-93 vs 99.5 rounds/s) -- the eval workgroups take CUs the 117 KB-LDS
        # training workgroups then wait for
        self._eval_overlap = os.environ.get("FEDMI_LENET_EVAL_OVERLAP", "0") == "1"
        self._ev_stream = self._ev_params = self._ev_pk = None

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
        self._configure_engine()
        self._starts, self._sizes = [], []

    def _configure_engine(self) -> None:
        """Launch-schedule switches of a (re)built engine binding (env overrides for A/B runs)."""
        self.engine.set_fuse_fc1(self.fuse_fc1)
        # K1 + K2 in one launch (FC-head weight prefetch overlapped with the conv stack)
        self.engine.set_fuse_head(os.environ.get("FEDMI_LENET_FUSE_HEAD", "1") == "1")
        # K3 + K4 in one launch (flag hand-off to SGD workgroups): opt-in -- measured 15.0 us vs 10.4 + 4.9,
        # the conv-param slab combine then trails the slowest sample (profiles/r2_lenet/experiments.md)
        self.engine.set_fuse_sgd(os.environ.get("FEDMI_LENET_FUSE_SGD", "0") == "1")
        # default: per-sample step kernel + batched FC-gradient GEMM/SGD kernel (2 launches, 10.45 vs
        # 12.95 ms per round, profiles/r2_lenet/experiments.md); FEDMI_LENET_PATH=head: K12 -> K3 -> K4
        self.engine.set_sample_path(os.environ.get("FEDMI_LENET_PATH", "sample") == "sample")

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
        # lenet::Stats: {float loss_sum, int correct, int count, flag} in an int32[4] row.  The flag word is
        # set by the cross-workgroup hand-off waits of the head path (K12 act2 wait: 1, K34 wait: 2) when
        # they time out and the kernel went on with stale rows -- never train on that silently.
        raw = raw.contiguous()
        flag = int(raw[3])
        if flag:
            what = {1: "conv -> FC-head act2 hand-off (K12)", 2: "K3 -> K4 gradient hand-off (K34)"}.get(flag, "?")
            raise RuntimeError(f"LeNet kernel hand-off timed out: {what} (stats flag {flag}); the step ran on "
                               "stale rows -- another process is starving this GPU, or a workgroup never ran")
        return EpochStats(float(raw[0:1].view(torch.float32).item()), int(raw[1]), int(raw[2]))

    def eval_stats_raw(self) -> torch.Tensor:
        return self.stats[1]

    def train_stats(self) -> EpochStats:
        return self._read_stats(0)

    def evaluate(self) -> None:
        """Eval of the current model.  Overlapped (opt-in, FEDMI_LENET_EVAL_OVERLAP=1): the weights
        are snapshotted on the current stream and the eval kernels run on a side stream, so they fill the
        CUs the next round's 128-workgroup training steps leave idle; the next round trains on the live
        buffers meanwhile.  Readers: :meth:`eval_stats` waits for it, device consumers use
        :meth:`eval_stream` (EvalHistory)."""
        if not self._eval_overlap:
            self.engine.eval(self._stream(), _ptr(self.test_set.x), _ptr(self.test_set.y), len(self.test_set))
            return
        main = torch.cuda.current_stream(self._device)
        if self._ev_stream is None:
            self._ev_stream = torch.cuda.Stream(self._device)
            self._ev_params = torch.empty_like(self.params)
            self._ev_pk = torch.empty_like(self.pk)
        main.wait_stream(self._ev_stream)          # the previous eval is done with the snapshot
        self._ev_params.copy_(self.params)
        self._ev_pk.copy_(self.pk)
        self._ev_stream.wait_stream(main)
        self.engine.eval(native.stream_handle_of(self._ev_stream), _ptr(self.test_set.x), _ptr(self.test_set.y),
                         len(self.test_set), _ptr(self._ev_pk), _ptr(self._ev_params))

    def eval_stream(self):
        return self._ev_stream if self._eval_overlap else None

    def eval_stats(self) -> EpochStats:
        if self._eval_overlap and self._ev_stream is not None:
            self._ev_stream.synchronize()
        return self._read_stats(1)

    def set_fuse_fc1(self, on: bool) -> None:
        """fc1 inside the FC-tail kernel (default) or as its own kernel (the graph is re-captured)."""
        self.fuse_fc1 = bool(on)
        self.engine.set_fuse_fc1(self.fuse_fc1)

    def reset_momentum(self) -> None:
        self.mom.zero_()

    def set_lr(self, lr: float) -> None:
        """New learning rate (re-captures the epoch graph on the next train_epoch)."""
        self.cfg.lr = float(lr)
        self.engine.set_sgd(self.cfg.lr, self.cfg.momentum, self.cfg.weight_decay)
