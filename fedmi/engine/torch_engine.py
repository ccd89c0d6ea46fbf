"""Generic local trainer for any model of the zoo (PyTorch autograd for the
layers, fedmi flat buffers + native fused SGD on GPU).

All parameters live in ONE flat fp32 buffer (``p.data`` are views), all
gradients in one flat grad buffer and all floating BN buffers in a second flat
buffer, so FedAvg is a single collective over :meth:`float_state` and the SGD
update is a single ``sgd_flat`` launch instead of 4 ops per tensor.
On CPU the identical update is done with torch ops (reference semantics).

``hybrid=True`` (GPU; what :func:`fedmi.engine.build_trainer` picks for zoo models without a
whole-network native engine): the step runs under :class:`fedmi.ops.native_mode.NativeMode`, so
every aten op of forward AND autograd backward executes on fedmi's HIP kernels (MFMA / depthwise /
grouped convs, BatchNorm, pooling, concat, SE gates, GEMM, loss) on channels-last bf16 activations
with fp32 master weights; the whole SGD step (zero-grad, forward, backward, fused SGD, loss /
accuracy statistics) is captured once into a HIP graph and replayed.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import List

import dataclasses
import os
import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

from .. import native
from ..models import build_model
from .base import EpochStats, LocalTrainer, TrainerConfig
from .data import FedDataset, ImageSet, augment_normalize


class FlatState:
    """Re-home a module's parameters / floating buffers into contiguous storage."""

    def __init__(self, model: nn.Module, device: torch.device):
        self.model = model
        params = [p for p in model.parameters()]
        n = sum(p.numel() for p in params)
        self.n_params = n
        fbufs = [(m, k, b) for m in model.modules() for k, b in m._buffers.items()
                 if b is not None and b.is_floating_point()]
        nb = sum(b.numel() for _, _, b in fbufs)
        # one storage: [params | float buffers]; params are aligned to 16 B for the vector kernels
        self.flat = torch.zeros(n + nb, dtype=torch.float32, device=device)
        self.grad = torch.zeros(n, dtype=torch.float32, device=device)
        self.mom = torch.zeros(n, dtype=torch.float32, device=device)
        off = 0
        self.offsets = []
        for p in params:
            k = p.numel()
            self.offsets.append(off)
            self.flat[off:off + k].copy_(p.data.reshape(-1))
            p.data = self.flat[off:off + k].view_as(p)
            p.grad = self.grad[off:off + k].view_as(p)
            off += k
        for m, key, b in fbufs:
            k = b.numel()
            self.flat[off:off + k].copy_(b.reshape(-1))
            m._buffers[key] = self.flat[off:off + k].view_as(b)
            off += k
        # integer buffers (BN num_batches_tracked) re-homed into ONE int64 vector as well: FedAvg averages
        # them in one collective instead of one per BatchNorm
        ibufs = [(m, k, b) for m in model.modules() for k, b in m._buffers.items()
                 if b is not None and not b.is_floating_point()]
        self.iflat = None
        if ibufs and all(b.dtype == torch.int64 for _, _, b in ibufs):
            self.iflat = torch.zeros(sum(b.numel() for _, _, b in ibufs), dtype=torch.int64, device=device)
            off = 0
            for m, key, b in ibufs:
                k = b.numel()
                self.iflat[off:off + k].copy_(b.reshape(-1))
                m._buffers[key] = self.iflat[off:off + k].view_as(b)
                off += k
        self.ibufs = [(m, k, m._buffers[k]) for m, k, _ in ibufs]

    def int_state(self) -> list:
        """The integer buffers as averaged by FedAvg: the one packed int64 vector (or the buffers themselves)."""
        if self.iflat is not None:
            return [self.iflat]
        return [b for _, _, b in self.ibufs]

    @property
    def params(self) -> torch.Tensor:
        return self.flat[:self.n_params]


class TorchTrainer(LocalTrainer):
    def __init__(self, model_name: str, data: FedDataset, device: torch.device,
                 cfg: TrainerConfig = TrainerConfig(), init_state=None, model_kwargs=None, hybrid: bool = False):
        self.model_name = model_name
        self.cfg = dataclasses.replace(cfg)   # private copy: set_lr mutates it
        self._device = torch.device(device)
        torch.manual_seed(cfg.seed)
        model = build_model(model_name, **(model_kwargs or {}))
        if init_state is not None:
            model.load_state_dict(init_state)
        self.model = model.to(self._device)
        self.fs = FlatState(self.model, self._device)
        self.train_set = data.train.to(self._device)
        self.test_set = data.test.to(self._device)
        self.mean, self.std = data.mean, data.std
        self.augment = bool(data.augment and cfg.augment)
        self.round_idx = 0
        self._starts: List[int] = []
        self._sizes: List[int] = []
        self._nat = native.require() if self._device.type == "cuda" and not native.force_torch_path() else None
        self.hybrid = bool(hybrid and self._nat is not None)
        # hybrid: the native ce_stats kernel accumulates fp32 (exact for counts < 2^24)
        sdt = torch.float32 if self.hybrid else torch.float64
        self._tstats = torch.zeros(3, dtype=sdt, device=self._device)
        self._estats = torch.zeros(3, dtype=sdt, device=self._device)
        self.mode = None
        self._flat_input = model_name.lower() == "mlp"     # flattens NCHW: keep the fp32 input as is
        if self.hybrid:
            from ..ops.native_mode import NativeMode

            # discard_unread: the step copies every p.grad inside the block, nothing reads a deferred tensor after it
            self.mode = NativeMode(strict=os.environ.get("FEDMI_NATIVE_STRICT", "0") == "1", seed=cfg.seed,
                                   discard_unread=True)
            self.mode.rng_ctr(self._device)      # allocated here, never inside a captured step
            self.mode.stable_storage = self.fs.flat.untyped_storage().data_ptr()   # weight images: batched packs
            # parameter gradients written straight into the flat gradient buffer (see native_mode._param_grad)
            self.mode.grad_flat = self.fs.grad
            self._params = list(self.model.parameters())
            self._grad_views = [self.fs.grad[o:o + p.numel()].view_as(p) for o, p in zip(self.fs.offsets, self._params)]
            off_of = {id(p): o for o, p in zip(self.fs.offsets, self._params)}
            for m in self.model.modules():
                w, b = getattr(m, "weight", None), getattr(m, "bias", None)
                if isinstance(w, nn.Parameter) and isinstance(b, nn.Parameter) and id(w) in off_of and id(b) in off_of:
                    self.mode.bias_of[off_of[id(w)]] = (off_of[id(b)], b.numel())
        # hybrid mode replays each full-batch SGD step (zero-grad + forward + autograd backward + SGD +
        # stats) from one captured HIP graph: the Python / launch overhead of ~10^3 small kernels per step
        # goes away.  Round 1's NaN-under-replay (autocast weight-cast cache, bf16 adaptive pooling, host
        # RNG state baked into the graph) is gone with the native backend: no autocast, fp32-accumulated
        # reductions, dropout masks keyed by a device counter the graph itself bumps.
        self.use_graph = bool(self.hybrid and cfg.use_graph and os.environ.get("FEDMI_HYBRID_GRAPH", "1") == "1")
        self._graph = None
        self._gx = self._gy = None

    @property
    def device(self) -> torch.device:
        return self._device

    # ---- state -------------------------------------------------------------------
    def state_dict(self):
        return OrderedDict(self.model.state_dict())

    def load_state_dict(self, sd) -> None:
        cleaned = OrderedDict((k[7:] if k.startswith("module.") else k, v) for k, v in sd.items())
        with torch.no_grad():
            own = self.model.state_dict()
            for k, v in cleaned.items():
                own[k].copy_(v.to(own[k].device, own[k].dtype))

    def float_state(self) -> torch.Tensor:
        return self.fs.flat

    def int_state(self) -> List[torch.Tensor]:
        return self.fs.int_state()

    def momentum_state(self) -> torch.Tensor:
        return self.fs.mom

    # ---- data ----------------------------------------------------------------------
    def set_schedule(self, starts, sizes) -> None:
        self._starts, self._sizes = list(map(int, starts)), list(map(int, sizes))

    def set_train_data(self, data: ImageSet) -> None:
        self.train_set = data.to(self._device)

    def _batch(self, start: int, nb: int):
        x = self.train_set.x[start:start + nb]
        gidx = np.arange(start, start + nb) if self.augment else None
        xin = augment_normalize(x, gidx, self.cfg.seed & 0xFFFFFFFF, self.round_idx, self.mean, self.std)
        return self._layout(xin), self.train_set.y[start:start + nb].long()

    def _layout(self, x: torch.Tensor) -> torch.Tensor:
        if self.hybrid and x.dim() == 4 and not self._flat_input:
            from ..ops.native_mode import EW_COPY, ew

            out = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
            return ew(out, [x], EW_COPY)
        return x

    def _run(self, x: torch.Tensor) -> torch.Tensor:
        return self.model(x)

    # ---- compute -------------------------------------------------------------------
    def _sgd(self) -> None:
        c = self.cfg
        fs = self.fs
        if self._nat is not None:
            self._nat.sgd_flat(native.stream_handle(self._device), fs.params.data_ptr(), fs.grad.data_ptr(),
                               fs.mom.data_ptr(), fs.n_params, c.lr, c.momentum, c.weight_decay, 0.0, False, False)
        else:
            with torch.no_grad():
                d = fs.grad.add(fs.params, alpha=c.weight_decay)
                fs.mom.mul_(c.momentum).add_(d)
                fs.params.sub_(fs.mom, alpha=c.lr)

    def train_step(self, start: int, nb: int) -> torch.Tensor:
        x, y = self._batch(start, nb)
        if self.use_graph and nb == self.cfg.batch_size:
            if self._graph is None:
                self._capture(x, y)
            self._gx.copy_(x)
            self._gy.copy_(y)
            self._graph.replay()
            return self._gloss
        return self._step_body(x, y)

    def _capture(self, x: torch.Tensor, y: torch.Tensor) -> None:
        """Capture one SGD step on static input buffers.  The warm-up step that precedes capture (it sizes
        the native workspaces and lets MIOpen pick its kernels) runs on a state snapshot that is restored
        afterwards, so capturing never changes the training trajectory."""
        fs = self.fs
        self._gx, self._gy = x.clone(), y.clone()
        snap = (fs.flat.clone(), fs.mom.clone(), [b.clone() for b in self.int_state()], self._tstats.clone())
        side = torch.cuda.Stream(self._device)
        side.wait_stream(torch.cuda.current_stream(self._device))
        with torch.cuda.stream(side):
            self._step_body(self._gx, self._gy)
        torch.cuda.current_stream(self._device).wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._gloss = self._step_body(self._gx, self._gy)
        with torch.no_grad():
            fs.flat.copy_(snap[0])
            fs.mom.copy_(snap[1])
            for b, v in zip(self.int_state(), snap[2]):
                b.copy_(v)
            self._tstats.copy_(snap[3])
        self._graph = g
        # the graph holds raw pointers into the shared conv workspace: keep that allocation alive even if a
        # later eager call (eval at a larger batch) grows the workspace and drops it from the cache
        from ..ops import conv as _conv

        self._graph_ws = _conv._WS.get(self._device)

    def _step_body(self, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        nb = x.shape[0]
        if self.mode is not None:
            from ..ops.native_mode import ce_stats_

            with self.mode:
                self.fs.grad.zero_()
                for p in self._params:        # AccumulateGrad adopts the native backward's flat-buffer gradients
                    p.grad = None
                out = self._run(x)
                loss = F.cross_entropy(out, y)
                loss.backward()
                for p, g in zip(self._params, self._grad_views):
                    if p.grad is not None and p.grad.data_ptr() != g.data_ptr():
                        g.copy_(p.grad)       # a gradient not produced in place (classifier GEMM, ATen op)
                    p.grad = g
            self._sgd()
            ce_stats_(out.detach(), y, self._tstats)
            return loss
        self.fs.grad.zero_()
        out = self._run(x)
        loss = F.cross_entropy(out, y)
        loss.backward()
        self._sgd()
        with torch.no_grad():
            self._tstats[0] += loss.detach().double() * nb
            self._tstats[1] += (out.argmax(1) == y).sum()
            self._tstats[2] += nb
        return loss

    def train_epoch(self) -> None:
        self.model.train()
        self._tstats.zero_()
        for s, n in zip(self._starts, self._sizes):
            self.train_step(s, n)
        if self._starts:
            self.round_idx += 1

    def train_stats(self) -> EpochStats:
        v = self._tstats.cpu().tolist()
        return EpochStats(v[0], int(v[1]), int(v[2]))

    @torch.no_grad()
    def evaluate(self) -> None:
        self.model.eval()
        self._estats.zero_()
        n = len(self.test_set)
        bs = self.cfg.eval_batch_size
        for s in range(0, n, bs):
            x = self._layout(augment_normalize(self.test_set.x[s:s + bs], None, 0, 0, self.mean, self.std))
            y = self.test_set.y[s:s + bs].long()
            if self.mode is not None:
                from ..ops.native_mode import ce_stats_

                with self.mode:
                    out = self._run(x)
                ce_stats_(out, y, self._estats)
                continue
            out = self._run(x)
            self._estats[0] += F.cross_entropy(out, y, reduction="sum").double()
            self._estats[1] += (out.argmax(1) == y).sum()
            self._estats[2] += y.numel()

    def eval_stats(self) -> EpochStats:
        return self.decode_stats(self._estats.cpu())

    def eval_stats_raw(self) -> torch.Tensor:
        return self._estats

    def decode_stats(self, raw: torch.Tensor) -> EpochStats:
        v = raw.tolist()
        return EpochStats(v[0], int(v[1]), int(v[2]))

    def set_lr(self, lr: float) -> None:
        if float(lr) != self.cfg.lr:
            self._graph = None           # the learning rate is a kernel argument baked into the graph
        self.cfg.lr = float(lr)
