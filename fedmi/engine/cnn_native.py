"""Native HIP engine for the BatchNorm CNN families of the zoo:

* ResNet-18/34 (BasicBlock) and ResNet-50/101/152 (Bottleneck), src/models/resnet.py:14-124
* MobileNet (depthwise-separable, the reference's default model), src/models/mobilenet.py:11-52
* MobileNetV2 (inverted residuals), src/models/mobilenetv2.py:11-77

The zoo ``nn.Module`` is only the parameter/buffer container (its
``state_dict`` keeps the reference key names and lives in fedmi's flat fp32
buffers); the training step is an explicit schedule of fedmi kernels on NHWC
bf16 activations.  A network is a list of *blocks*; a block is a chain of
*units* (conv or depthwise conv -> BatchNorm -> optional ReLU) whose last BN is
fused with the block's shortcut (none / identity residual / projection
conv+BN) and output ReLU in one ``bn_apply`` launch:

  forward   prep_input (crop/flip/normalize, device-side batch start)
            -> per unit: conv (implicit-GEMM MFMA, BN batch statistics summed in
               the epilogue) or depthwise conv (VALU, same fused statistics)
               -> bn_apply (+residual / +projection BN, +ReLU)
            -> head (global avgpool + linear + CE + dlogits)
  backward  per block, reversed: bn_bwd (ReLU mask, both BN branches, residual
            fan-in of two incoming grads) -> wgrad (split-K partials into a
            workspace, one reduce into the flat grad buffer) -> dgrad
  update    one multi-tensor SGD launch over the flat fp32 master, then the
            bf16 [O][R][S][C] weight images of the dense convs are repacked

Each training step is captured once per batch size into a HIP graph
(``torch.cuda.CUDAGraph``) and replayed for every batch of the epoch (the
batch start comes from a device-side schedule).  All activations stay
resident, sized for max(train batch, eval batch) rows.
"""
from __future__ import annotations

import dataclasses
import os
from collections import OrderedDict
from typing import Dict, List, Optional

import torch
from torch import nn

from .. import native
from ..models import build_model
from ..models.zoo.mobile import DWSeparable, InvertedResidual, MobileNet, MobileNetV2
from ..models.zoo.multibranch import VGG, GoogLeNet, Inception
from ..models.zoo.residual import BasicBlock, Bottleneck, PreActBlock, PreActBottleneck, PreActResNet, ResNet
from ..ops import cnn, conv
from .base import EpochStats, LocalTrainer, TrainerConfig
from .data import FedDataset, ImageSet
from .torch_engine import FlatState

BN_EPS = 1e-5
BN_MOM = 0.1


class _Unit:
    """conv (dense or depthwise, no bias) + BatchNorm2d (+ ReLU), with its device buffers."""

    def __init__(self, c: nn.Conv2d, bn: nn.BatchNorm2d, in_hw: int, relu: bool, rows: int, dev,
                 need_y: bool = True, c_in_pad: Optional[int] = None, act_dtype=torch.bfloat16):
        assert c.dilation == (1, 1)
        # a conv bias (VGG) stays out of z: train-mode BN cancels it exactly (its gradient is 0, the
        # flat grad entry is never written), it only enters running_mean / eval via BNParams.cbias
        self.conv, self.bn, self.relu = c, bn, relu
        self.depthwise = c.groups > 1
        if self.depthwise and not (c.groups == c.in_channels == c.out_channels):
            raise TypeError("grouped (non-depthwise) convolutions are not supported by the native engine")
        self.O, self.Cw, self.R, self.S = c.weight.shape
        if self.depthwise:
            self.Cw = c.in_channels
        self.C = c_in_pad or conv.pad8(self.Cw)
        self.stride, self.pad = c.stride[0], c.padding[0]
        self.H = in_hw
        self.P = (in_hw + 2 * self.pad - self.R) // self.stride + 1
        n_out = rows * self.P * self.P * self.O
        bf = dict(dtype=act_dtype, device=dev)
        self.wr = None if self.depthwise else torch.empty(self.O, self.R, self.S, self.C, dtype=torch.bfloat16,
                                                          device=dev)
        # flipped/transposed weight image for the tap-major DGRAD kernel (O % 64 == 0; stride 1: O % 8 == 0)
        self.wd = (torch.empty(conv.dgrad_image_numel(c.weight.shape, self.C), dtype=torch.bfloat16, device=dev)
                   if not self.depthwise and conv.dgrad_eligible(self.O, self.stride) else None)
        self.z = torch.empty(n_out, **bf)                            # conv output (pre-BN)
        self.y = torch.empty(n_out, **bf) if need_y else None        # BN(+ReLU) output inside a block
        self.dz = torch.empty(n_out, **bf)                           # grad wrt z
        self.dy = torch.empty(n_out, **bf) if need_y else None       # grad wrt y
        self.smean = torch.empty(self.O, device=dev)
        self.sinv = torch.empty(self.O, device=dev)
        self.shift = torch.zeros(self.O, device=dev)   # previous batch mean: stats are sums of (z - shift)
        self._fusable: Optional[bool] = None

    def view(self, t: torch.Tensor, nb: int) -> torch.Tensor:
        return t[: nb * self.P * self.P * self.O].view(nb, self.P, self.P, self.O)

    def bn_args(self, stats) -> dict:
        b = self.bn
        return cnn.bn_desc(stats, b.weight, b.bias, b.running_mean, b.running_var, b.num_batches_tracked,
                           self.smean, self.sinv, self.shift, cbias=self.conv.bias)

    def in_shape(self, nb: int):
        return (nb, self.H, self.H, self.C)

    def ws_floats(self, nb: int) -> int:
        if self.depthwise:
            return conv.dwconv_ws_floats(self.in_shape(nb), self.R, self.stride, self.pad)
        shp = (self.in_shape(nb), self.O, self.R, self.S, self.stride, self.pad, self.Cw)
        return max(conv.wgrad_ws_floats(*shp), conv.fd_ws_floats(*shp))

    # ---- launches (``ws``: the engine's shared split-K workspace; launches are stream-serial)
    def fwd(self, x: torch.Tensor, nb: int, stats, ws: Optional[torch.Tensor] = None,
            res: Optional[torch.Tensor] = None) -> None:
        sh = self.shift if stats is not None else None
        if self.depthwise:
            assert res is None
            conv.dwconv_fwd(x, self.conv.weight, self.stride, self.pad, stats=stats, out=self.view(self.z, nb),
                            shift=sh)
        else:
            conv.conv2d_fwd(x, self.wr, self.stride, self.pad, Cw=self.Cw, stats=stats, out=self.view(self.z, nb),
                            shift=sh, ws=ws, res=res)

    def wgrad_floats(self, nb: int) -> int:
        """Partial-sum floats this conv's WGRAD writes (its own buffer when the reduction is deferred)."""
        if self.depthwise:
            return conv.dwconv_ws_floats(self.in_shape(nb), self.R, self.stride, self.pad)
        return conv.wgrad_ws_floats(self.in_shape(nb), self.O, self.R, self.S, self.stride, self.pad, self.Cw)

    def wgrad(self, x: torch.Tensor, nb: int, ws: torch.Tensor, dz: Optional[torch.Tensor] = None,
              deferred: Optional[list] = None) -> None:
        dz = self.view(self.dz, nb) if dz is None else dz
        if self.depthwise:
            conv.dwconv_wgrad(x, dz, self.R, self.stride, self.pad, out=self.conv.weight.grad, ws=ws,
                              deferred=deferred)
        else:
            conv.conv2d_wgrad(x, dz, self.R, self.S, self.stride, self.pad, Cw=self.Cw, out=self.conv.weight.grad,
                              ws=ws, deferred=deferred)

    def dgrad(self, nb: int, out: torch.Tensor, ws: Optional[torch.Tensor] = None,
              dz: Optional[torch.Tensor] = None, accumulate: bool = False, add: Optional[torch.Tensor] = None,
              bn_sums: Optional[dict] = None) -> torch.Tensor:
        dz = self.view(self.dz, nb) if dz is None else dz
        if self.depthwise:
            assert not accumulate and add is None
            return conv.dwconv_dgrad(dz, self.conv.weight, self.in_shape(nb), self.stride, self.pad, out=out,
                                     bn_sums=bn_sums)
        return conv.conv2d_dgrad(dz, self.wr, self.in_shape(nb), self.stride, self.pad, Cw=self.Cw, out=out, ws=ws,
                                 wd=self.wd, accumulate=accumulate, add=add, bn_sums=bn_sums)

    def dgrad_fusable(self, add: bool = False) -> bool:
        """Whether this conv's DGRAD can take its producer BN's backward sums in the epilogue (dense tap
        path; the depthwise DGRAD with the sums measured slower, 846 vs 832 ms per MobileNet round, and with
        round 5's blocked depthwise DGRAD kernels a wash, 695.8 / 694.7 vs 695.9 / 693.5 ms) and,
        ``add``, a second incoming grad."""
        if self.depthwise:
            return False
        if self._fusable is None:
            self._fusable = (self.wd is not None and
                             conv.dgrad_fusable(self.in_shape(1), self.O, self.R, self.S, self.stride, self.pad,
                                                self.Cw, True))
        return self._fusable

    def pack_item(self):
        return None if self.depthwise else (self.conv.weight.data, self.wr)

    def dgrad_pack_item(self):
        return None if self.wd is None else (self.conv.weight.data, self.wd, self.stride, self.pad, self.C)


class _Block:
    """Chain of units; the last unit's BN is fused with the shortcut and the output ReLU, optionally
    followed by MaxPool2d(2, 2) (VGG)."""

    def __init__(self, pairs, relus, in_hw: int, cin: int, rows: int, dev, shortcut: str = "none",
                 proj=None, out_relu: bool = True, first: bool = False, act_dtype=torch.bfloat16, pool: bool = False):
        self.main: List[_Unit] = []
        hw = in_hw
        for i, ((c, bn), r) in enumerate(zip(pairs, relus)):
            last = i == len(pairs) - 1
            u = _Unit(c, bn, hw, relu=r, rows=rows, dev=dev, need_y=not last,
                      c_in_pad=8 if first and i == 0 else None, act_dtype=act_dtype)
            self.main.append(u)
            hw = u.P
        self.in_hw, self.cin = in_hw, cin
        self.pre_hw = hw                    # spatial size before the optional pool
        self.pool = pool
        if pool and (shortcut != "none" or hw % 2):
            raise TypeError("maxpool blocks: no shortcut, even spatial size")
        self.out_hw = hw // 2 if pool else hw
        self.cout = self.main[-1].O
        self.shortcut = shortcut            # "none" | "identity" | "proj"
        self.proj = (_Unit(proj[0], proj[1], in_hw, relu=False, rows=rows, dev=dev, need_y=False,
                           act_dtype=act_dtype) if proj else None)
        self.out_relu = out_relu
        self.first = first                  # network input block: no input gradient
        bf = dict(dtype=act_dtype, device=dev)
        self.pre = torch.empty(rows * hw * hw * self.cout, **bf)
        self.out = torch.empty(rows * self.out_hw * self.out_hw * self.cout, **bf) if pool else self.pre
        self.dpre = torch.empty(rows * hw * hw * self.cout, **bf) if pool else None
        n_in = rows * in_hw * in_hw * cin
        self.din_a = None if first else torch.empty(n_in, **bf)
        self.din_b = torch.empty(n_in, **bf) if shortcut != "none" else None

    def units(self) -> List[_Unit]:
        return self.main + ([self.proj] if self.proj else [])

    def out_view(self, nb: int) -> torch.Tensor:
        return self.out[: nb * self.out_hw * self.out_hw * self.cout].view(nb, self.out_hw, self.out_hw, self.cout)

    def pre_view(self, nb: int) -> torch.Tensor:
        return self.pre[: nb * self.pre_hw * self.pre_hw * self.cout].view(nb, self.pre_hw, self.pre_hw, self.cout)

    def dpre_view(self, nb: int) -> torch.Tensor:
        return self.dpre[: nb * self.pre_hw * self.pre_hw * self.cout].view(nb, self.pre_hw, self.pre_hw, self.cout)

    def in_view(self, t: torch.Tensor, nb: int) -> torch.Tensor:
        return t[: nb * self.in_hw * self.in_hw * self.cin].view(nb, self.in_hw, self.in_hw, self.cin)


# ---------------------------------------------------------------------------- network plans
def _plan_resnet(m: ResNet, rows, dev, dt) -> List[_Block]:
    blocks = [_Block([(m.conv1, m.bn1)], [True], 32, 8, rows, dev, first=True, act_dtype=dt)]
    hw, c = blocks[0].out_hw, blocks[0].cout
    for layer in (m.layer1, m.layer2, m.layer3, m.layer4):
        for blk in layer:
            if isinstance(blk, BasicBlock):
                pairs = [(blk.conv1, blk.bn1), (blk.conv2, blk.bn2)]
            elif isinstance(blk, Bottleneck):
                pairs = [(blk.conv1, blk.bn1), (blk.conv2, blk.bn2), (blk.conv3, blk.bn3)]
            else:
                raise TypeError(type(blk).__name__)
            relus = [True] * (len(pairs) - 1) + [False]
            proj = (blk.shortcut[0], blk.shortcut[1]) if len(blk.shortcut) else None
            b = _Block(pairs, relus, hw, c, rows, dev, shortcut="proj" if proj else "identity", proj=proj,
                       out_relu=True, act_dtype=dt)
            blocks.append(b)
            hw, c = b.out_hw, b.cout
    return blocks


def _plan_mobilenet(m: MobileNet, rows, dev, dt) -> List[_Block]:
    blocks = [_Block([(m.conv1, m.bn1)], [True], 32, 8, rows, dev, first=True, act_dtype=dt)]
    hw, c = blocks[0].out_hw, blocks[0].cout
    for blk in m.layers:
        assert isinstance(blk, DWSeparable)
        b = _Block([(blk.conv1, blk.bn1), (blk.conv2, blk.bn2)], [True, True], hw, c, rows, dev, out_relu=True,
                   act_dtype=dt)
        blocks.append(b)
        hw, c = b.out_hw, b.cout
    return blocks


def _plan_mobilenetv2(m: MobileNetV2, rows, dev, dt) -> List[_Block]:
    blocks = [_Block([(m.conv1, m.bn1)], [True], 32, 8, rows, dev, first=True, act_dtype=dt)]
    hw, c = blocks[0].out_hw, blocks[0].cout
    for blk in m.layers:
        assert isinstance(blk, InvertedResidual)
        pairs = [(blk.conv1, blk.bn1), (blk.conv2, blk.bn2), (blk.conv3, blk.bn3)]
        if blk.stride != 1:
            short, proj = "none", None
        elif len(blk.shortcut):
            short, proj = "proj", (blk.shortcut[0], blk.shortcut[1])
        else:
            short, proj = "identity", None
        b = _Block(pairs, [True, True, False], hw, c, rows, dev, shortcut=short, proj=proj, out_relu=False,
                   act_dtype=dt)
        blocks.append(b)
        hw, c = b.out_hw, b.cout
    blocks.append(_Block([(m.conv2, m.bn2)], [True], hw, c, rows, dev, out_relu=True, act_dtype=dt))
    return blocks


def _plan_vgg(m: VGG, rows, dev, dt) -> List[_Block]:
    """features = [Conv2d(bias), BN, ReLU | MaxPool2d(2)]..., AvgPool2d(1) (identity), classifier."""
    mods = list(m.features)
    blocks: List[_Block] = []
    hw, c = 32, 8
    i = 0
    while i < len(mods):
        mod = mods[i]
        if isinstance(mod, nn.Conv2d):
            bn = mods[i + 1]
            assert isinstance(bn, nn.BatchNorm2d) and isinstance(mods[i + 2], nn.ReLU)
            pool = i + 3 < len(mods) and isinstance(mods[i + 3], nn.MaxPool2d)
            b = _Block([(mod, bn)], [True], hw, c, rows, dev, out_relu=True, first=not blocks, act_dtype=dt,
                       pool=pool)
            blocks.append(b)
            hw, c = b.out_hw, b.cout
            i += 4 if pool else 3
        elif isinstance(mod, nn.AvgPool2d) and mod.kernel_size in (1, (1, 1)):
            i += 1
        else:
            raise TypeError(f"VGG plan: unexpected {type(mod).__name__}")
    return blocks


class _PABlock:
    """Pre-activation residual block (src/models/preact_resnet.py:12-62) as units.

    A unit is (conv, the BN that normalises its output).  Inside the block:
    (conv1, bn2) [, (conv2, bn3)], and the last conv pairs with the NEXT block's
    bn1 (None for the network's last block: its output goes to the head); its
    epilogue also adds the shortcut (identity x, or the 1x1 shortcut conv of the
    pre-activation, a BN-less unit) so the next bn1's statistics are of x + skip.
    """

    def __init__(self, blk, in_hw: int, cin: int, rows: int, dev, dt, next_bn):
        if isinstance(blk, PreActBlock):
            pairs = [(blk.conv1, blk.bn2), (blk.conv2, next_bn)]
        elif isinstance(blk, PreActBottleneck):
            pairs = [(blk.conv1, blk.bn2), (blk.conv2, blk.bn3), (blk.conv3, next_bn)]
        else:
            raise TypeError(type(blk).__name__)
        self.units: List[_Unit] = []
        hw = in_hw
        for c, bn in pairs:
            u = _Unit(c, bn, hw, relu=True, rows=rows, dev=dev, need_y=bn is not None, act_dtype=dt)
            self.units.append(u)
            hw = u.P
        self.sc = (_Unit(blk.shortcut[0], None, in_hw, relu=False, rows=rows, dev=dev, need_y=False, act_dtype=dt)
                   if hasattr(blk, "shortcut") else None)
        self.in_hw, self.cin, self.out_hw, self.cout = in_hw, cin, hw, self.units[-1].O
        self.da2 = torch.empty(rows * in_hw * in_hw * cin, dtype=dt, device=dev) if self.sc else None

    def all_units(self) -> List[_Unit]:
        return self.units + ([self.sc] if self.sc else [])

    def in_view(self, t: torch.Tensor, nb: int) -> torch.Tensor:
        return t[: nb * self.in_hw * self.in_hw * self.cin].view(nb, self.in_hw, self.in_hw, self.cin)


class _PreActPlan:
    def __init__(self, m: PreActResNet, rows, dev, dt):
        blks = [b for layer in (m.layer1, m.layer2, m.layer3, m.layer4) for b in layer]
        # stem conv (no BN of its own) pairs with the first block's bn1
        self.stem = _Unit(m.conv1, blks[0].bn1, 32, relu=True, rows=rows, dev=dev, need_y=True, c_in_pad=8,
                          act_dtype=dt)
        self.blocks: List[_PABlock] = []
        hw, c = self.stem.P, self.stem.O
        for i, b in enumerate(blks):
            nb = blks[i + 1].bn1 if i + 1 < len(blks) else None
            pb = _PABlock(b, hw, c, rows, dev, dt, nb)
            self.blocks.append(pb)
            hw, c = pb.out_hw, pb.cout

    def units(self) -> List[_Unit]:
        return [self.stem] + [u for b in self.blocks for u in b.all_units()]


def _plan_preact(m, rows, dev, dt):
    return _PreActPlan(m, rows, dev, dt)


def _nhwc(t: torch.Tensor, nb: int, hw: int, c: int) -> torch.Tensor:
    return t[: nb * hw * hw * c].view(nb, hw, hw, c)


class _Incep:
    """Inception module (src/models/googlenet.py:7-53) as four unit chains (1x1 | 1x1-3x3 |
    1x1-3x3-3x3 | maxpool3x3/1 -> 1x1).  Each chain's last BN+ReLU writes its channel slice of
    one concatenated NHWC output (strided ``bn_apply``), so ``torch.cat`` never runs; backward
    reads the slices of the output grad in place and the four input grads are summed by the
    first convs' DGRAD epilogues (accumulate) and the maxpool backward's gather."""

    def __init__(self, m: Inception, hw: int, cin: int, rows: int, dev, dt, pool_after: bool):
        self.branches: List[List[_Unit]] = []
        for k, seq in enumerate((m.b1, m.b2, m.b3, m.b4)):
            mods = list(seq)
            if k == 3:
                mp = mods.pop(0)
                if not (isinstance(mp, nn.MaxPool2d) and mp.kernel_size == 3 and mp.stride == 1 and mp.padding == 1):
                    raise TypeError("Inception pool branch: expected MaxPool2d(3, 1, 1)")
            pairs = [(mods[i], mods[i + 1]) for i in range(0, len(mods), 3)]
            us = []
            for i, (c, bn) in enumerate(pairs):
                assert isinstance(c, nn.Conv2d) and isinstance(bn, nn.BatchNorm2d)
                us.append(_Unit(c, bn, hw, relu=True, rows=rows, dev=dev, need_y=i < len(pairs) - 1, act_dtype=dt))
            self.branches.append(us)
        self.widths = [br[-1].O for br in self.branches]
        self.offs = [sum(self.widths[:k]) for k in range(4)]
        self.hw, self.cin, self.cout = hw, cin, sum(self.widths)
        bf = dict(dtype=dt, device=dev)
        n_in, n_out = rows * hw * hw * cin, rows * hw * hw * self.cout
        self.out = torch.empty(n_out, **bf)                  # concatenated branch outputs
        self.dout = torch.empty(n_out, **bf)                 # grad wrt out
        self.bp = torch.empty(n_in, **bf)                    # maxpool3/1 of the input (pool branch)
        self.bidx = torch.empty(n_in, dtype=torch.uint8, device=dev)
        self.dbp = torch.empty(n_in, **bf)
        self.pool_after = pool_after                         # MaxPool2d(3, 2, 1) after the module
        self.out_hw = (hw - 1) // 2 + 1 if pool_after else hw
        n_sp = rows * self.out_hw * self.out_hw * self.cout
        self.sp = torch.empty(n_sp, **bf) if pool_after else None
        self.sidx = torch.empty(n_sp, dtype=torch.uint8, device=dev) if pool_after else None
        self.dsp = torch.empty(n_sp, **bf) if pool_after else None
        self._bidx = self._sidx = None                       # argmax records of the current step

    def units(self) -> List[_Unit]:
        return [u for br in self.branches for u in br]

    def out_view(self, t, nb):
        return _nhwc(t, nb, self.hw, self.cout)

    def in_view(self, t, nb):
        return _nhwc(t, nb, self.hw, self.cin)

    def final_view(self, t, nb):                             # the module's result (after the stage pool)
        return _nhwc(t, nb, self.out_hw, self.cout)

    def slice(self, t4, k):
        return t4[..., self.offs[k]:self.offs[k] + self.widths[k]]


class _GoogPlan:
    """pre_layers (conv3x3+BN+ReLU) -> a3 b3 | pool | a4..e4 | pool | a5 b5 -> avgpool(8) + linear
    (src/models/googlenet.py:56-98)."""

    def __init__(self, m: GoogLeNet, rows, dev, dt):
        c0, bn0 = m.pre_layers[0], m.pre_layers[1]
        self.pre = _Unit(c0, bn0, 32, relu=True, rows=rows, dev=dev, need_y=True, c_in_pad=8, act_dtype=dt)
        hw, c = self.pre.P, self.pre.O
        mp = m.maxpool
        if not (mp.kernel_size == 3 and mp.stride == 2 and mp.padding == 1):
            raise TypeError("GoogLeNet plan: expected MaxPool2d(3, 2, 1) between stages")
        self.mods: List[_Incep] = []
        for name, _ in m.STAGES:
            I = _Incep(getattr(m, name), hw, c, rows, dev, dt, name in ("b3", "e4"))
            self.mods.append(I)
            hw, c = I.out_hw, I.cout
        if m.avgpool.kernel_size not in (hw, (hw, hw)):
            raise TypeError("GoogLeNet plan: the head must average the whole final map")
        self.head_hw, self.head_c = hw, c

    def units(self) -> List[_Unit]:
        return [self.pre] + [u for I in self.mods for u in I.units()]


def _plan_googlenet(m, rows, dev, dt):
    return _GoogPlan(m, rows, dev, dt)


PLANS = {ResNet: _plan_resnet, MobileNet: _plan_mobilenet, MobileNetV2: _plan_mobilenetv2, VGG: _plan_vgg,
         PreActResNet: _plan_preact, GoogLeNet: _plan_googlenet}


def supports(model: nn.Module) -> bool:
    return type(model) in PLANS


class CNNNativeTrainer(LocalTrainer):
    def __init__(self, model_name: str, data: FedDataset, device: torch.device, cfg: TrainerConfig = TrainerConfig(),
                 init_state=None, act_dtype=torch.bfloat16):
        """``act_dtype`` other than bf16 only works under the tests' kernel emulation (tests/emulate.py)."""
        self._nat = native.require()
        self._device = device = torch.device(device)
        self.cfg = dataclasses.replace(cfg)
        self.model_name = model_name
        torch.manual_seed(cfg.seed)
        model = build_model(model_name)
        if type(model) not in PLANS:
            raise TypeError(f"{model_name}: no native plan (ResNet, PreActResNet, MobileNet, MobileNetV2, VGG)")
        if init_state is not None:
            model.load_state_dict(init_state)
        self.model = model.to(device)
        self.fs = FlatState(self.model, device)
        self.train_set = data.train.to(device)
        self.test_set = data.test.to(device)
        self.augment = bool(data.augment and cfg.augment)
        if tuple(self.train_set.x.shape[1:]) != (3, 32, 32):
            raise ValueError("native CNN engine expects CIFAR-shaped uint8 [N,3,32,32] data")
        for s in (self.train_set, self.test_set):
            if s.y.dtype != torch.int32:
                s.y = s.y.to(torch.int32)
        self.eval_bs = min(cfg.eval_batch_size, 500)
        self.rows = R = max(cfg.batch_size, self.eval_bs)
        plan = PLANS[type(model)](self.model, R, device, act_dtype)
        self.preact = plan if isinstance(plan, _PreActPlan) else None
        self.goog = plan if isinstance(plan, _GoogPlan) else None
        if self.goog is not None:
            self.blocks = []
            self.head_hw, self.head_c = plan.head_hw, plan.head_c
            self.units: List[_Unit] = plan.units()
            self._no_dgrad = {id(plan.pre)}
        else:
            self.blocks = plan.blocks if self.preact else plan
            last = self.blocks[-1]
            self.head_hw, self.head_c = last.out_hw, last.cout
            self.units = plan.units() if self.preact else [u for b in self.blocks for u in b.units()]
            # units whose data gradient is never needed (they read the network input)
            self._no_dgrad = ({id(self.preact.stem)} if self.preact else
                              {id(u) for u in self.blocks[0].units()} if self.blocks[0].first else set())
        # per-step accumulators: BN batch stats [2][O] and BN-backward sums [3][O], one fill each
        # fp64 accumulators: the kernels add fp32 workgroup partials with fp64 atomics (order-independent sums)
        self.stats_all = torch.zeros(sum(conv.STAT_REP * 2 * u.O for u in self.units), dtype=torch.float64,
                                     device=device)
        self.red_all = torch.zeros(sum(3 * u.O for u in self.units), dtype=torch.float64, device=device)
        so = ro = 0
        for u in self.units:
            u.stats = self.stats_all[so:so + conv.STAT_REP * 2 * u.O].view(conv.STAT_REP, 2, u.O)
            u.red = self.red_all[ro:ro + 3 * u.O].view(3, u.O)
            so += conv.STAT_REP * 2 * u.O
            ro += 3 * u.O
        B = cfg.batch_size
        # one fp32 split-K workspace for every conv launch of a step (fwd / dgrad / wgrad)
        self.wgrad_ws = torch.empty(max(max(u.ws_floats(nb) for u in self.units) for nb in {B, self.eval_bs}),
                                    device=device)
        # (weight gradients on a side stream overlapping the dgrad chain measured slower -- ResNet-18 1036 vs
        # 983 ms per round, MobileNet 886 vs 832: the concurrent kernels compete for CUs / LDS and the split-K
        # sizing assumes the whole chip, profiles/r3_cnn.  Round 6 re-measured it as two graph branches with the
        # side stream's split count divided by 1 / 2 / 4 (sized for the CUs the DGRAD chain leaves): ResNet-18
        # 847 / 837 / 925 vs 823-827 ms, MobileNet 733 / 752 / 789 vs 690-692; and only for the small layers (<= 2048 /
        # 8192 output pixels per batch, whose kernels fill a fraction of the chip): ResNet-18 859 / 849 vs 826-829,
        # MobileNet 739 / 749 vs 691-692, profiles/r6_cnn/ -- one stream)
        # Deferred WGRAD reductions: every conv's WGRAD writes its split-K / depthwise partials into a buffer of its
        # own and ONE launch after the backward pass sums them all (conv.wgrad_reduce_multi; bit-identical to the
        # per-conv reduce launches it replaces, most of them latency-bound).  FEDMI_WRED_DEFER=0: per-conv
        # reductions in the shared workspace (A/B).
        self._wred: Optional[list] = None
        self._wpart = {}
        if os.environ.get("FEDMI_WRED_DEFER", "1") != "0":
            # sized for every batch size a schedule can hold: the automatic split count is capped by the
            # workspace, and it is not monotone in the batch (a partial last batch of 80 takes 160 splits of a
            # GoogLeNet 3x3 conv where 128 take 158) -- a binding cap would change the rounding.
            # FEDMI_WRED_DEFER_MB=n: defer only WGRADs with at most n MB of partials, reducing the larger sets right
            # away while they may still sit in the 256 MB infinity cache (ResNet-18's 3x3 halo WGRADs write ~38 MB
            # each, ~480 MB per step).  Measured a wash -- ResNet-18 816.6 / 819.2 ms at 8 MB, 815.3 at 64, 815.6 all
            # deferred; GoogLeNet 3338 vs 3325 (profiles/r6_cnn/wgrad_defer/cap_*) -- so everything is deferred.
            cap = float(os.environ.get("FEDMI_WRED_DEFER_MB", "inf")) * (1 << 20) / 4
            need = {id(u): max(u.wgrad_floats(nb) for nb in range(1, B + 1)) for u in self.units}
            units = [u for u in self.units if need[id(u)] <= cap]
            sizes = [(need[id(u)] + 63) // 64 * 64 for u in units]
            self.wgrad_parts = torch.empty(max(sum(sizes), 1), device=device)
            off = 0
            for u, n in zip(units, sizes):
                self._wpart[id(u)] = self.wgrad_parts[off:off + n]
                off += n
        # BN-backward two-level channel sums (replicated atomics + finalize; kept zero between uses)
        self.bn_ws = torch.zeros(max(cnn.bn_bwd_ws_floats(B * u.P * u.P, u.O) for u in self.units),
                                 dtype=torch.float64, device=device)
        # chained BN backward: every BN gets its own replica slice of one arena, the head launch clears the
        # arena each step and the apply kernels read the replicas directly (no finalize launch per BN)
        self.bn_chain = torch.zeros(sum((cnn.bn_bwd_chain_floats(u.O) + 3) // 4 * 4 for u in self.units) + 4,
                                    dtype=torch.float64, device=device)
        co = 0
        for u in self.units:
            nf = cnn.bn_bwd_chain_floats(u.O)
            n = (nf + 3) // 4 * 4
            u.bn_rep = self.bn_chain[co:co + n] if n else None
            u.bn_reps = nf // (3 * u.O)
            co += n
        # BN-backward channel sums taken in the epilogue of the DGRAD that writes the BN's output grad
        # (conv_igemm.hip BnSums): no separate reduce pass over (dy, z, y)
        self._fuse_bn_bwd = True
        # a ReLU'd BN inside a block (no residual): the forward stores its scale / shift, and the backward
        # derives the ReLU mask from z (z * sc + sh > 0) instead of re-reading the materialised y
        for u in self.units:
            u.zco = None
        if self._fuse_bn_bwd and self.preact is None and self.goog is None:
            for b in self.blocks:
                for v in b.main[:-1]:
                    if v.relu and v.bn_rep is not None:
                        v.zco = torch.empty(2, v.O, device=device)
        self.xin = torch.empty(R, 32, 32, 8, dtype=act_dtype, device=device)
        self.dhead = torch.empty(R * self.head_hw * self.head_hw * self.head_c, dtype=act_dtype, device=device)
        self.pooled = torch.empty(R, self.head_c, device=device)
        self.head_lin = getattr(self.model, "linear", None) or self.model.classifier
        self.dlog = torch.empty(R, self.head_lin.out_features, device=device)
        self.lossv = torch.empty(R, device=device)            # per-sample CE losses (ordered sum, no atomics)
        self.stats = torch.zeros(2, 4, device=device)        # [train, eval] x {loss, correct, count, pad}
        self.round_ctr = torch.zeros(4, dtype=torch.int32, device=device)
        self.sched = torch.zeros(1, dtype=torch.int32, device=device)
        self.counter = torch.zeros(1, dtype=torch.int32, device=device)
        self.cur = torch.zeros(1, dtype=torch.int32, device=device)
        self.ebase = torch.zeros(1, dtype=torch.int32, device=device)
        self._starts: List[int] = []
        self._sizes: List[int] = []
        self._graphs: Dict[tuple, torch.cuda.CUDAGraph] = {}
        self.round_idx = 0
        self.pack()
        # the step's tail in ONE launch: SGD on the flat master + every conv's forward / DGRAD image from the
        # updated weights (conv.SgdPack; FEDMI_SGD_PACK=0: sgd_flat, then the two pack launches)
        self._sgdpack = None
        if os.environ.get("FEDMI_SGD_PACK", "1") != "0":
            self._sgdpack = conv.SgdPack(
                self.fs.params, self.fs.grad, self.fs.mom,
                [(u.conv.weight.data, u.wr, None if id(u) in self._no_dgrad else u.wd, u.stride, u.pad, u.C)
                 for u in self.units if not u.depthwise])

    # ---- state ---------------------------------------------------------------------
    @property
    def device(self) -> torch.device:
        return self._device

    def state_dict(self):
        return OrderedDict((k, v.detach()) for k, v in self.model.state_dict().items())

    def load_state_dict(self, sd) -> None:
        with torch.no_grad():
            own = self.model.state_dict()
            for k, v in sd.items():
                own[k].copy_(v.to(own[k].device, own[k].dtype).view(own[k].shape))
        self.after_aggregate()

    def float_state(self) -> torch.Tensor:
        return self.fs.flat

    def int_state(self) -> List[torch.Tensor]:
        return self.fs.int_state()

    def momentum_state(self) -> torch.Tensor:
        return self.fs.mom

    def after_aggregate(self) -> None:
        self.pack()

    def set_lr(self, lr: float) -> None:
        self.cfg.lr = float(lr)
        self._graphs.clear()

    def pack(self) -> None:
        conv.pack_weights([it for it in (u.pack_item() for u in self.units) if it is not None])
        # the network input units never need a data gradient: skip their images
        conv.dgrad_pack_weights([it for u in self.units if id(u) not in self._no_dgrad
                                 for it in [u.dgrad_pack_item()] if it is not None])

    # ---- data ----------------------------------------------------------------------------
    def set_schedule(self, starts, sizes) -> None:
        starts, sizes = list(map(int, starts)), list(map(int, sizes))
        n = len(self.train_set)
        for s, b in zip(starts, sizes):
            if not (0 < b <= self.cfg.batch_size) or s < 0 or s + b > n:
                raise ValueError(f"schedule: batch ({s}, {b}) out of range")
        self._starts, self._sizes = starts, sizes
        self.sched = torch.tensor(starts or [0], dtype=torch.int32, device=self._device)
        self._graphs.clear()

    def set_train_data(self, data: ImageSet) -> None:
        self.train_set = data.to(self._device)
        if self.train_set.y.dtype != torch.int32:
            self.train_set.y = self.train_set.y.to(torch.int32)
        self._starts, self._sizes = [], []
        self._graphs.clear()

    def _act(self, b: "_Block", nb: int):
        return b.out_view(nb)

    # ---- kernel schedule ---------------------------------------------------------------------
    def _bn(self, u: _Unit, z: torch.Tensor, y: torch.Tensor, train: bool, relu: bool, **kw) -> torch.Tensor:
        return cnn.bn_apply(z, u.bn_args(u.stats), y, train, relu, eps=BN_EPS, momentum=BN_MOM, **kw)

    def _forward(self, nb: int, train: bool, images: torch.Tensor, labels: torch.Tensor, dbase, stats_row: int):
        if self.preact is not None:
            return self._forward_preact(nb, train, images, labels, dbase, stats_row)
        if self.goog is not None:
            return self._forward_goog(nb, train, images, labels, dbase, stats_row)
        x = cnn.prep_input(images, 0, nb, self.augment and train, self.cfg.seed, self.round_ctr,
                           out=self.xin[:nb], dbase=dbase)
        a = x
        for b in self.blocks:
            h = a
            ws = self.wgrad_ws
            for v in b.main[:-1]:
                v.fwd(h, nb, v.stats if train else None, ws)
                h = self._bn(v, v.view(v.z, nb), v.view(v.y, nb), train, v.relu,
                             co_out=v.zco if train else None)
            last = b.main[-1]
            last.fwd(h, nb, last.stats if train else None, ws)
            out = b.pre_view(nb)
            z = last.view(last.z, nb)
            if b.shortcut == "proj":
                p = b.proj
                p.fwd(a, nb, p.stats if train else None, ws)
                self._bn(last, z, out, train, b.out_relu, z2=p.view(p.z, nb), b=p.bn_args(p.stats))
            elif b.shortcut == "identity":
                self._bn(last, z, out, train, b.out_relu, res=a)
            else:
                self._bn(last, z, out, train, b.out_relu)
            if b.pool:
                cnn.maxpool2(out, out=b.out_view(nb))
            a = self._act(b, nb)
        lin = self.head_lin
        hd = self.dhead[: a.numel()].view_as(a)
        cnn.head(a, labels, 0, lin.weight, lin.bias, self.stats[stats_row], train, self.pooled[:nb], self.dlog[:nb],
                 hd if train else None, lin.weight.grad if train else None, lin.bias.grad if train else None,
                 dbase=dbase, zero=self.bn_chain if train else None, lossv=self.lossv[:nb])
        return x, hd

    def _sums(self, conv_u: _Unit, u: _Unit, nb: int, y, zb: Optional[_Unit] = None,
              add: bool = False) -> Optional[dict]:
        """BN-sums descriptor for ``u``'s BN, taken by ``conv_u``'s DGRAD epilogue (None: not fusable).
        ``add``: the DGRAD must also add a second incoming grad (a shortcut's)."""
        if not (self._fuse_bn_bwd and u.bn_rep is not None and u.bn_reps > 0 and conv_u.dgrad_fusable(add)):
            return None
        d = dict(rep=u.bn_rep, reps=u.bn_reps, z=u.view(u.z, nb), y=y, mean=u.smean, inv=u.sinv)
        if zb is not None:
            d.update(zb=zb.view(zb.z, nb), meanb=zb.smean, invb=zb.sinv)
        return d

    def _wgrad(self, u: _Unit, x, nb: int, dz=None) -> None:
        part = self._wpart.get(id(u)) if self._wred is not None else None
        if part is None:
            u.wgrad(x, nb, self.wgrad_ws, dz=dz)
        else:
            u.wgrad(x, nb, part, dz=dz, deferred=self._wred)

    def _bn_bwd(self, u: _Unit, nb: int, dya, dyb, y, zb: Optional[_Unit] = None, gout=None, dadd=None,
                mask_bn=None, presummed: bool = False) -> None:
        bn_ws = self.bn_ws if self.bn_ws.numel() else None
        chained = u.bn_rep is not None
        if chained:
            bn_ws = u.bn_rep
        kw = {}
        if zb is not None:
            kw = dict(zb=zb.view(zb.z, nb), b=zb.bn_args(None), dgamma_b=zb.bn.weight.grad,
                      dbeta_b=zb.bn.bias.grad, dzb=zb.view(zb.dz, nb))
        cnn.bn_bwd(dya, u.view(u.z, nb), u.bn_args(None), u.bn.weight.grad, u.bn.bias.grad, u.view(u.dz, nb), u.red,
                   dyb=dyb, y=y, gout=gout, ws=bn_ws, dadd=dadd, chained=chained, mask_bn=mask_bn,
                   presummed=presummed, **kw)

    def _backward(self, nb: int, x: torch.Tensor, dhead: torch.Tensor) -> None:
        if self.preact is not None:
            return self._backward_preact(nb, x, dhead)
        if self.goog is not None:
            return self._backward_goog(nb, x, dhead)
        dya, dyb, pres = dhead, None, False
        ws = self.wgrad_ws
        for i in range(len(self.blocks) - 1, -1, -1):
            b = self.blocks[i]
            prev = None if b.first else self.blocks[i - 1]
            a_in = x if b.first else self._act(prev, nb)
            last = b.main[-1]
            din_b = b.in_view(b.din_b, nb) if b.din_b is not None else None
            if b.pool:   # grad wrt the pooled output -> grad wrt the pre-pool activation
                dya = cnn.maxpool2_bwd(b.pre_view(nb), dya, out=b.dpre_view(nb))
            # pres: the next block's first DGRAD wrote dya = (its grad + the shortcut grad) and this BN's sums
            self._bn_bwd(last, nb, dya, dyb, b.pre_view(nb) if b.out_relu else None, zb=b.proj,
                         gout=din_b if b.shortcut == "identity" else None, presummed=pres)
            proj_done = False
            for j in range(len(b.main) - 1, -1, -1):
                v = b.main[j]
                xin = b.main[j - 1].view(b.main[j - 1].y, nb) if j > 0 else a_in
                self._wgrad(v, xin, nb)
                if j > 0:
                    w = b.main[j - 1]
                    wy = w.view(w.y, nb) if w.relu else None
                    bs = self._sums(v, w, nb, wy)
                    msc = None
                    if bs is not None and w.zco is not None:   # ReLU mask from z: y is not re-read
                        bs.update(y=None, msc=w.zco)
                        wy, msc = None, w.zco
                    v.dgrad(nb, w.view(w.dy, nb), ws, bn_sums=bs)
                    self._bn_bwd(w, nb, w.view(w.dy, nb), None, wy, presummed=bs is not None, mask_bn=msc)
                elif not b.first:
                    din_a = b.in_view(b.din_a, nb)
                    bs = None
                    if not prev.pool:
                        pl = prev.main[-1]
                        bs = self._sums(v, pl, nb, prev.pre_view(nb) if prev.out_relu else None, zb=prev.proj,
                                        add=din_b is not None)
                    if bs is not None:
                        # the shortcut's grad first, then conv1's DGRAD adds it and takes the previous
                        # block's BN-backward sums from the complete grad
                        if b.proj is not None:
                            self._wgrad(b.proj, a_in, nb)
                            b.proj.dgrad(nb, din_b, ws)
                            proj_done = True
                        v.dgrad(nb, din_a, ws, add=din_b, bn_sums=bs)   # add=None: no shortcut
                        dya, dyb, pres = din_a, None, True
                    else:
                        v.dgrad(nb, din_a, ws)
                        dya, dyb, pres = din_a, din_b, False
            if b.proj is not None and not proj_done:
                self._wgrad(b.proj, a_in, nb)
                b.proj.dgrad(nb, din_b, ws)

    # ---- pre-activation ResNets --------------------------------------------------------------
    def _head(self, a, nb, train, labels, dbase, stats_row):
        lin = self.head_lin
        hd = self.dhead[: a.numel()].view_as(a)
        cnn.head(a, labels, 0, lin.weight, lin.bias, self.stats[stats_row], train, self.pooled[:nb], self.dlog[:nb],
                 hd if train else None, lin.weight.grad if train else None, lin.bias.grad if train else None,
                 dbase=dbase, zero=self.bn_chain if train else None, lossv=self.lossv[:nb])
        return hd

    def _forward_preact(self, nb: int, train: bool, images, labels, dbase, stats_row: int):
        P, ws = self.preact, self.wgrad_ws
        x = cnn.prep_input(images, 0, nb, self.augment and train, self.cfg.seed, self.round_ctr,
                           out=self.xin[:nb], dbase=dbase)
        st = P.stem
        st.fwd(x, nb, st.stats if train else None, ws)
        self._bn(st, st.view(st.z, nb), st.view(st.y, nb), train, True)
        prev = st
        for b in P.blocks:
            a = prev.view(prev.y, nb)                      # relu(bn1(x_b))
            h = a
            for u in b.units[:-1]:
                u.fwd(h, nb, u.stats if train else None, ws)
                self._bn(u, u.view(u.z, nb), u.view(u.y, nb), train, True)
                h = u.view(u.y, nb)
            if b.sc is not None:
                b.sc.fwd(a, nb, None, ws)
                skip = b.sc.view(b.sc.z, nb)
            else:
                skip = prev.view(prev.z, nb)               # identity: x_b
            L = b.units[-1]
            L.fwd(h, nb, L.stats if (train and L.bn is not None) else None, ws, res=skip)
            if L.bn is not None:
                self._bn(L, L.view(L.z, nb), L.view(L.y, nb), train, True)
            prev = L
        return x, self._head(prev.view(prev.z, nb), nb, train, labels, dbase, stats_row)

    def _backward_preact(self, nb: int, x: torch.Tensor, dhead: torch.Tensor) -> None:
        P, ws = self.preact, self.wgrad_ws
        g = dhead                                          # dL / d x_{b+1} (= dz of the block's last unit)
        for bi in range(len(P.blocks) - 1, -1, -1):
            b = P.blocks[bi]
            prev = P.blocks[bi - 1].units[-1] if bi > 0 else P.stem
            a = prev.view(prev.y, nb)
            L = b.units[-1]
            pen = b.units[-2]
            self._wgrad(L, pen.view(pen.y, nb), nb, dz=g)
            L.dgrad(nb, pen.view(pen.dy, nb), ws, dz=g)
            for j in range(len(b.units) - 2, -1, -1):
                u = b.units[j]
                self._bn_bwd(u, nb, u.view(u.dy, nb), None, u.view(u.y, nb))
                if j > 0:
                    w = b.units[j - 1]
                    self._wgrad(u, w.view(w.y, nb), nb)
                    u.dgrad(nb, w.view(w.dy, nb), ws)
                else:
                    self._wgrad(u, a, nb)
                    u.dgrad(nb, prev.view(prev.dy, nb), ws)      # d a_b, conv1 branch
            da2 = None
            if b.sc is not None:                           # d a_b, shortcut-conv branch
                self._wgrad(b.sc, a, nb, dz=g)
                da2 = b.in_view(b.da2, nb)
                b.sc.dgrad(nb, da2, ws, dz=g)
            # bn1 of this block (prev's BN): dx_b = BN_bwd(relu mask) + identity-shortcut grad
            self._bn_bwd(prev, nb, prev.view(prev.dy, nb), da2, a, dadd=None if b.sc is not None else g)
            g = prev.view(prev.dz, nb)
        self._wgrad(P.stem, x, nb)

    # ---- GoogLeNet ----------------------------------------------------------------------------
    def _forward_goog(self, nb: int, train: bool, images, labels, dbase, stats_row: int):
        G, ws = self.goog, self.wgrad_ws
        x = cnn.prep_input(images, 0, nb, self.augment and train, self.cfg.seed, self.round_ctr,
                           out=self.xin[:nb], dbase=dbase)
        p = G.pre
        p.fwd(x, nb, p.stats if train else None, ws)
        a = self._bn(p, p.view(p.z, nb), p.view(p.y, nb), train, True)
        for I in G.mods:
            out = I.out_view(I.out, nb)
            for k, br in enumerate(I.branches):
                h = a
                if k == 3:
                    h, I._bidx = cnn.maxpool3(a, 1, out=I.in_view(I.bp, nb), idx=I.in_view(I.bidx, nb))
                for u in br[:-1]:
                    u.fwd(h, nb, u.stats if train else None, ws)
                    h = self._bn(u, u.view(u.z, nb), u.view(u.y, nb), train, True)
                L = br[-1]
                L.fwd(h, nb, L.stats if train else None, ws)
                self._bn(L, L.view(L.z, nb), I.slice(out, k), train, True)    # its channel slice of the concat
            a = out
            if I.pool_after:
                a, I._sidx = cnn.maxpool3(out, 2, out=I.final_view(I.sp, nb), idx=I.final_view(I.sidx, nb))
        return x, self._head(a, nb, train, labels, dbase, stats_row)

    def _backward_goog(self, nb: int, x: torch.Tensor, dhead: torch.Tensor) -> None:
        G, ws = self.goog, self.wgrad_ws
        p = G.pre
        g = dhead                                          # grad wrt the current module's result
        for i in range(len(G.mods) - 1, -1, -1):
            I = G.mods[i]
            if i > 0:                                      # the module input and where its grad goes
                J = G.mods[i - 1]
                a = J.final_view(J.sp if J.pool_after else J.out, nb)
                dx = J.final_view(J.dsp if J.pool_after else J.dout, nb)
            else:
                a, dx = p.view(p.y, nb), p.view(p.dy, nb)
            if I.pool_after:
                g = cnn.maxpool3_bwd(g, I._sidx, (nb, I.hw, I.hw, I.cout), 2, out=I.out_view(I.dout, nb))
            out = I.out_view(I.out, nb)
            for k, br in enumerate(I.branches):
                self._bn_bwd(br[-1], nb, I.slice(g, k), None, I.slice(out, k))
                for j in range(len(br) - 1, -1, -1):
                    v = br[j]
                    if j > 0:
                        w = br[j - 1]
                        wy = w.view(w.y, nb)
                        self._wgrad(v, wy, nb)
                        # the inner BN's backward sums in this DGRAD's epilogue where it runs on conv_tap
                        # (no separate reduce pass over (dy, z, y))
                        bs = self._sums(v, w, nb, wy)
                        v.dgrad(nb, w.view(w.dy, nb), ws, bn_sums=bs)
                        self._bn_bwd(w, nb, w.view(w.dy, nb), None, wy, presummed=bs is not None)
                    elif k < 3:                            # branch heads: the module input's grad fan-in
                        self._wgrad(v, a, nb)
                        v.dgrad(nb, dx, ws, accumulate=k > 0)
                    else:
                        self._wgrad(v, I.in_view(I.bp, nb), nb)
                        dbp = v.dgrad(nb, I.in_view(I.dbp, nb), ws)
                        cnn.maxpool3_bwd(dbp, I._bidx, (nb, I.hw, I.hw, I.cin), 1, out=dx, accumulate=True)
            g = dx
        self._bn_bwd(p, nb, p.view(p.dy, nb), None, p.view(p.y, nb))
        self._wgrad(p, x, nb)

    def _sgd(self) -> None:
        c, fs = self.cfg, self.fs
        if self._sgdpack is not None:
            self._sgdpack.step(c.lr, c.momentum, c.weight_decay)
            return
        self._nat.sgd_flat(native.stream_handle(self._device), fs.params.data_ptr(), fs.grad.data_ptr(),
                           fs.mom.data_ptr(), fs.n_params, c.lr, c.momentum, c.weight_decay, 0.0, False, False)
        self.pack()

    def _forward_backward(self, nb: int, zeroed: bool = False) -> None:
        # every gradient entry is overwritten (wgrad reduce, BN dgamma/dbeta, head): no grad zeroing;
        # the BN statistics accumulators are zeroed by the step's first kernel (sched_next) unless ``zeroed``
        if not zeroed:
            self.stats_all.zero_()
        if not self.bn_ws.numel():     # atomic BN-backward sums (emulation) need zeroed accumulators
            self.red_all.zero_()
        x, dh = self._forward(nb, True, self.train_set.x, self.train_set.y, self.cur, 0)
        self._wred = [] if self._wpart else None
        try:
            self._backward(nb, x, dh)
            if self._wred:      # the most recently written partials first (the likeliest still cache-resident)
                conv.wgrad_reduce_multi(self._wred[::-1], self._device)
        finally:
            self._wred = None

    def _train_step(self, nb: int) -> None:
        """One SGD step on the batch at sched[counter] (device-side)."""
        cnn.sched_next(self.sched, self.counter, self.cur, zero=self.stats_all)
        self._forward_backward(nb, zeroed=True)
        self._sgd()

    def grads_for_batch(self, start: int, nb: int) -> None:
        """Forward + backward of one batch WITHOUT the update (tests / diagnostics); grads in fs.grad."""
        self.model.train()
        self.cur.fill_(start)
        self._forward_backward(nb)

    # ---- compute ------------------------------------------------------------------------------
    def train_epoch(self) -> None:
        if not self._starts:
            return
        self.model.train()
        self.stats[0].zero_()
        self.counter.zero_()
        if not self.cfg.use_graph:
            for nb in self._sizes:
                self._train_step(nb)
        else:
            for nb in self._sizes:
                g = self._graphs.get(("train", nb))
                if g is None:
                    g = self._capture(nb)
                g.replay()
        self.round_ctr[0] += 1
        self.round_idx += 1

    def _capture(self, nb: int) -> torch.cuda.CUDAGraph:
        # a warm-up eager step precedes capture; snapshot and restore everything it touches
        saved = (self.fs.flat.clone(), self.fs.mom.clone(), [b.clone() for b in self.int_state()],
                 self.counter.clone(), self.stats.clone(), [u.shift.clone() for u in self.units])
        s = torch.cuda.Stream(self._device)
        s.wait_stream(torch.cuda.current_stream(self._device))
        with torch.cuda.stream(s):
            self._train_step(nb)
        torch.cuda.current_stream(self._device).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            self._train_step(nb)
        with torch.no_grad():
            self.fs.flat.copy_(saved[0])
            self.fs.mom.copy_(saved[1])
            for b, v in zip(self.int_state(), saved[2]):
                b.copy_(v)
            self.counter.copy_(saved[3])
            self.stats.copy_(saved[4])
            for u, v in zip(self.units, saved[5]):      # BN statistics shifts: the replay starts bit-identical
                u.shift.copy_(v)
        self.pack()
        self._graphs[("train", nb)] = g
        return g

    def train_stats(self) -> EpochStats:
        return self._read_stats(0)

    def _read_stats(self, i: int) -> EpochStats:
        return self.decode_stats(self.stats[i].cpu())

    def decode_stats(self, raw: torch.Tensor) -> EpochStats:
        # head kernel row: {float loss_sum, int correct, int count, pad} in a float32[4] row
        raw = raw.contiguous()
        iv = raw.view(torch.int32)
        return EpochStats(float(raw[0]), int(iv[1]), int(iv[2]))

    def eval_stats_raw(self) -> torch.Tensor:
        return self.stats[1]

    @torch.no_grad()
    def evaluate(self) -> None:
        self.model.eval()
        self.stats[1].zero_()
        n = len(self.test_set)
        bs = self.eval_bs
        for s in range(0, n, bs):
            nb = min(bs, n - s)
            self.ebase.fill_(s)
            self._forward(nb, False, self.test_set.x, self.test_set.y, self.ebase, 1)

    def eval_stats(self) -> EpochStats:
        return self._read_stats(1)


# backwards-compatible name
ResNetNativeTrainer = CNNNativeTrainer
