"""Depthwise / grouped / searched CIFAR families: MobileNet v1/v2, ShuffleNet v1/v2,
EfficientNet-B0, RegNet X/Y, PNASNet A/B.

Key-compatible with the reference zoo:
  MobileNet      src/models/mobilenet.py:11-52    (reference default model)
  MobileNetV2    src/models/mobilenetv2.py:11-77
  ShuffleNet     src/models/shufflenet.py:10-100  (G2/G3; the reference's float
                 mid_planes makes them unconstructible, quirk A12 — fixed with //)
  ShuffleNetV2   src/models/shufflenetv2.py:10-152
  EfficientNetB0 src/models/efficientnet.py:12-164 (swish, SE, drop-connect)
  RegNet         src/models/regnet.py:12-143
  PNASNet        src/models/pnasnet.py:10-116
"""
from __future__ import annotations

from typing import Dict, Sequence

import torch
import torch.nn.functional as F
from torch import nn

from .pool import global_avg_pool


def _bn(c: int) -> nn.BatchNorm2d:
    return nn.BatchNorm2d(c)


def _dw(c: int, k: int = 3, stride: int = 1, cout: int | None = None) -> nn.Conv2d:
    return nn.Conv2d(c, cout or c, k, stride=stride, padding=(k - 1) // 2, groups=c, bias=False)


def _pw(cin: int, cout: int, groups: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, 1, groups=groups, bias=False)


def channel_shuffle(x: torch.Tensor, groups: int) -> torch.Tensor:
    n, c, h, w = x.shape
    return x.view(n, groups, c // groups, h, w).transpose(1, 2).reshape(n, c, h, w)


class _Shuffle(nn.Module):
    def __init__(self, groups: int = 2):
        super().__init__()
        self.groups = groups

    def forward(self, x):
        return channel_shuffle(x, self.groups)


def swish(x: torch.Tensor) -> torch.Tensor:
    return x * torch.sigmoid(x)


# --------------------------------------------------------------------------- MobileNet v1
class DWSeparable(nn.Module):
    def __init__(self, cin: int, cout: int, stride: int = 1):
        super().__init__()
        self.conv1, self.bn1 = _dw(cin, 3, stride), _bn(cin)
        self.conv2, self.bn2 = _pw(cin, cout), _bn(cout)

    def forward(self, x):
        return F.relu(self.bn2(self.conv2(F.relu(self.bn1(self.conv1(x))))))


class MobileNet(nn.Module):
    PLAN = (64, (128, 2), 128, (256, 2), 256, (512, 2), 512, 512, 512, 512, 512, (1024, 2), 1024)

    def __init__(self, num_classes: int = 10):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 32, 3, padding=1, bias=False)
        self.bn1 = _bn(32)
        blocks, c = [], 32
        for item in self.PLAN:
            cout, stride = (item, 1) if isinstance(item, int) else item
            blocks.append(DWSeparable(c, cout, stride))
            c = cout
        self.layers = nn.Sequential(*blocks)
        self.linear = nn.Linear(1024, num_classes)

    def forward(self, x):
        y = self.layers(F.relu(self.bn1(self.conv1(x))))
        return self.linear(torch.flatten(F.avg_pool2d(y, 2), 1))


# --------------------------------------------------------------------------- MobileNet v2
class InvertedResidual(nn.Module):
    def __init__(self, cin: int, cout: int, expansion: int, stride: int):
        super().__init__()
        self.stride = stride
        mid = expansion * cin
        self.conv1, self.bn1 = _pw(cin, mid), _bn(mid)
        self.conv2, self.bn2 = _dw(mid, 3, stride), _bn(mid)
        self.conv3, self.bn3 = _pw(mid, cout), _bn(cout)
        self.shortcut = nn.Sequential()
        if stride == 1 and cin != cout:
            self.shortcut = nn.Sequential(_pw(cin, cout), _bn(cout))

    def forward(self, x):
        y = F.relu(self.bn1(self.conv1(x)))
        y = F.relu(self.bn2(self.conv2(y)))
        y = self.bn3(self.conv3(y))
        return y + self.shortcut(x) if self.stride == 1 else y


class MobileNetV2(nn.Module):
    # (expansion, out, blocks, stride) with CIFAR strides (stage 2 and the stem at stride 1)
    PLAN = ((1, 16, 1, 1), (6, 24, 2, 1), (6, 32, 3, 2), (6, 64, 4, 2), (6, 96, 3, 1), (6, 160, 3, 2),
            (6, 320, 1, 1))

    def __init__(self, num_classes: int = 10):
        super().__init__()
        self.conv1, self.bn1 = nn.Conv2d(3, 32, 3, padding=1, bias=False), _bn(32)
        blocks, c = [], 32
        for e, cout, n, s in self.PLAN:
            for st in [s] + [1] * (n - 1):
                blocks.append(InvertedResidual(c, cout, e, st))
                c = cout
        self.layers = nn.Sequential(*blocks)
        self.conv2, self.bn2 = _pw(320, 1280), _bn(1280)
        self.linear = nn.Linear(1280, num_classes)

    def forward(self, x):
        y = self.layers(F.relu(self.bn1(self.conv1(x))))
        y = F.relu(self.bn2(self.conv2(y)))
        return self.linear(torch.flatten(F.avg_pool2d(y, 4), 1))


# --------------------------------------------------------------------------- ShuffleNet v1
class ShuffleUnit(nn.Module):
    def __init__(self, cin: int, cout: int, stride: int, groups: int):
        super().__init__()
        self.stride = stride
        mid = cout // 4
        g = 1 if cin == 24 else groups
        self.conv1, self.bn1 = _pw(cin, mid, groups=g), _bn(mid)
        self.shuffle1 = _Shuffle(g)
        self.conv2, self.bn2 = _dw(mid, 3, stride), _bn(mid)
        self.conv3, self.bn3 = _pw(mid, cout, groups=groups), _bn(cout)
        self.shortcut = nn.Sequential(nn.AvgPool2d(3, stride=2, padding=1)) if stride == 2 else nn.Sequential()

    def forward(self, x):
        y = self.shuffle1(F.relu(self.bn1(self.conv1(x))))
        y = self.bn3(self.conv3(F.relu(self.bn2(self.conv2(y)))))
        r = self.shortcut(x)
        return F.relu(torch.cat([y, r], 1)) if self.stride == 2 else F.relu(y + r)


class ShuffleNet(nn.Module):
    def __init__(self, outs: Sequence[int], depths: Sequence[int], groups: int, num_classes: int = 10):
        super().__init__()
        self.conv1, self.bn1 = _pw(3, 24), _bn(24)
        c = 24
        stages = []
        for cout, n in zip(outs, depths):
            units = []
            for i in range(n):
                units.append(ShuffleUnit(c, cout - (c if i == 0 else 0), 2 if i == 0 else 1, groups))
                c = cout
            stages.append(nn.Sequential(*units))
        self.layer1, self.layer2, self.layer3 = stages
        self.linear = nn.Linear(outs[2], num_classes)

    def forward(self, x):
        y = F.relu(self.bn1(self.conv1(x)))
        y = self.layer3(self.layer2(self.layer1(y)))
        return self.linear(torch.flatten(F.avg_pool2d(y, 4), 1))


# --------------------------------------------------------------------------- ShuffleNet v2
class SplitUnit(nn.Module):
    def __init__(self, c: int, ratio: float = 0.5):
        super().__init__()
        self.ratio = ratio
        h = int(c * ratio)
        self.conv1, self.bn1 = _pw(h, h), _bn(h)
        self.conv2, self.bn2 = _dw(h, 3, 1), _bn(h)
        self.conv3, self.bn3 = _pw(h, h), _bn(h)
        self.shuffle = _Shuffle(2)

    def forward(self, x):
        k = int(x.size(1) * self.ratio)
        keep, work = x[:, :k], x[:, k:]
        y = F.relu(self.bn1(self.conv1(work)))
        y = F.relu(self.bn3(self.conv3(self.bn2(self.conv2(y)))))
        return self.shuffle(torch.cat([keep, y], 1))


class DownUnit(nn.Module):
    def __init__(self, cin: int, cout: int):
        super().__init__()
        mid = cout // 2
        self.conv1, self.bn1 = _dw(cin, 3, 2), _bn(cin)
        self.conv2, self.bn2 = _pw(cin, mid), _bn(mid)
        self.conv3, self.bn3 = _pw(cin, mid), _bn(mid)
        self.conv4, self.bn4 = _dw(mid, 3, 2), _bn(mid)
        self.conv5, self.bn5 = _pw(mid, mid), _bn(mid)
        self.shuffle = _Shuffle(2)

    def forward(self, x):
        left = F.relu(self.bn2(self.conv2(self.bn1(self.conv1(x)))))
        right = F.relu(self.bn3(self.conv3(x)))
        right = F.relu(self.bn5(self.conv5(self.bn4(self.conv4(right)))))
        return self.shuffle(torch.cat([left, right], 1))


SHUFFLEV2_CFG: Dict[float, tuple] = {
    0.5: ((48, 96, 192, 1024), (3, 7, 3)),
    1: ((116, 232, 464, 1024), (3, 7, 3)),
    1.5: ((176, 352, 704, 1024), (3, 7, 3)),
    2: ((224, 488, 976, 2048), (3, 7, 3)),
}


class ShuffleNetV2(nn.Module):
    def __init__(self, net_size: float = 1, num_classes: int = 10):
        super().__init__()
        outs, depths = SHUFFLEV2_CFG[net_size]
        self.conv1, self.bn1 = nn.Conv2d(3, 24, 3, padding=1, bias=False), _bn(24)
        c = 24
        stages = []
        for cout, n in zip(outs[:3], depths):
            stages.append(nn.Sequential(DownUnit(c, cout), *[SplitUnit(cout) for _ in range(n)]))
            c = cout
        self.layer1, self.layer2, self.layer3 = stages
        self.conv2, self.bn2 = _pw(outs[2], outs[3]), _bn(outs[3])
        self.linear = nn.Linear(outs[3], num_classes)

    def forward(self, x):
        y = F.relu(self.bn1(self.conv1(x)))
        y = self.layer3(self.layer2(self.layer1(y)))
        y = F.relu(self.bn2(self.conv2(y)))
        return self.linear(torch.flatten(F.avg_pool2d(y, 4), 1))


# --------------------------------------------------------------------------- EfficientNet-B0
class SqueezeExcite(nn.Module):
    def __init__(self, c: int, squeeze: int, act=swish):
        super().__init__()
        self.se1 = nn.Conv2d(c, squeeze, 1)
        self.se2 = nn.Conv2d(squeeze, c, 1)
        self.act = act

    def forward(self, x):
        s = self.act(self.se1(global_avg_pool(x)))
        return x * torch.sigmoid(self.se2(s))


def drop_connect(x: torch.Tensor, p: float) -> torch.Tensor:
    keep = 1.0 - p
    mask = torch.empty(x.shape[0], 1, 1, 1, dtype=x.dtype, device=x.device).bernoulli_(keep)
    return x / keep * mask


class MBConv(nn.Module):
    def __init__(self, cin: int, cout: int, k: int, stride: int, expand: int, se_ratio: float, drop: float):
        super().__init__()
        self.expand_ratio, self.drop_rate = expand, drop
        mid = expand * cin
        self.conv1, self.bn1 = _pw(cin, mid), _bn(mid)
        self.conv2, self.bn2 = _dw(mid, k, stride), _bn(mid)
        self.se = SqueezeExcite(mid, int(cin * se_ratio))
        self.conv3, self.bn3 = _pw(mid, cout), _bn(cout)
        self.has_skip = stride == 1 and cin == cout

    def forward(self, x):
        y = x if self.expand_ratio == 1 else swish(self.bn1(self.conv1(x)))
        y = self.se(swish(self.bn2(self.conv2(y))))
        y = self.bn3(self.conv3(y))
        if self.has_skip:
            if self.training and self.drop_rate > 0:
                y = drop_connect(y, self.drop_rate)
            y = y + x
        return y


class EfficientNet(nn.Module):
    def __init__(self, expansion, outs, depths, kernels, strides, dropout=0.2, drop_connect_rate=0.2,
                 num_classes: int = 10):
        super().__init__()
        self.dropout = dropout
        self.conv1, self.bn1 = nn.Conv2d(3, 32, 3, padding=1, bias=False), _bn(32)
        total = sum(depths)
        blocks, c, b = [], 32, 0
        for e, cout, n, k, s in zip(expansion, outs, depths, kernels, strides):
            for st in [s] + [1] * (n - 1):
                blocks.append(MBConv(c, cout, k, st, e, 0.25, drop_connect_rate * b / total))
                c = cout
        # (the reference never advances its block counter, so every drop rate is 0)
        self.layers = nn.Sequential(*blocks)
        self.linear = nn.Linear(outs[-1], num_classes)

    def forward(self, x):
        y = self.layers(swish(self.bn1(self.conv1(x))))
        y = torch.flatten(global_avg_pool(y), 1)
        if self.training and self.dropout > 0:
            y = F.dropout(y, p=self.dropout)
        return self.linear(y)


# --------------------------------------------------------------------------- RegNet
class RegBlock(nn.Module):
    def __init__(self, w_in: int, w_out: int, stride: int, group_width: int, bottleneck: float, se_ratio: float):
        super().__init__()
        wb = int(round(w_out * bottleneck))
        self.conv1, self.bn1 = _pw(w_in, wb), _bn(wb)
        self.conv2 = nn.Conv2d(wb, wb, 3, stride=stride, padding=1, groups=wb // group_width, bias=False)
        self.bn2 = _bn(wb)
        self.with_se = se_ratio > 0
        if self.with_se:
            self.se = SqueezeExcite(wb, int(round(w_in * se_ratio)), act=F.relu)
        self.conv3, self.bn3 = _pw(wb, w_out), _bn(w_out)
        self.shortcut = nn.Sequential()
        if stride != 1 or w_in != w_out:
            self.shortcut = nn.Sequential(nn.Conv2d(w_in, w_out, 1, stride=stride, bias=False), _bn(w_out))

    def forward(self, x):
        y = F.relu(self.bn1(self.conv1(x)))
        y = F.relu(self.bn2(self.conv2(y)))
        if self.with_se:
            y = self.se(y)
        y = self.bn3(self.conv3(y))
        return F.relu(y + self.shortcut(x))


class RegNet(nn.Module):
    def __init__(self, depths, widths, strides, group_width, bottleneck=1, se_ratio=0.0, num_classes: int = 10):
        super().__init__()
        self.conv1, self.bn1 = nn.Conv2d(3, 64, 3, padding=1, bias=False), _bn(64)
        c = 64
        stages = []
        for d, w, s in zip(depths, widths, strides):
            blocks = []
            for i in range(d):
                blocks.append(RegBlock(c, w, s if i == 0 else 1, group_width, bottleneck, se_ratio))
                c = w
            stages.append(nn.Sequential(*blocks))
        self.layer1, self.layer2, self.layer3, self.layer4 = stages
        self.linear = nn.Linear(widths[-1], num_classes)

    def forward(self, x):
        y = F.relu(self.bn1(self.conv1(x)))
        y = self.layer4(self.layer3(self.layer2(self.layer1(y))))
        return self.linear(torch.flatten(global_avg_pool(y), 1))


# --------------------------------------------------------------------------- PNASNet
class SepConv(nn.Module):
    def __init__(self, cin: int, cout: int, k: int, stride: int):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, k, stride, padding=(k - 1) // 2, bias=False, groups=cin)
        self.bn1 = _bn(cout)

    def forward(self, x):
        return self.bn1(self.conv1(x))


class CellA(nn.Module):
    def __init__(self, cin: int, cout: int, stride: int = 1):
        super().__init__()
        self.stride = stride
        self.sep_conv1 = SepConv(cin, cout, 7, stride)
        if stride == 2:
            self.conv1, self.bn1 = _pw(cin, cout), _bn(cout)

    def forward(self, x):
        y2 = F.max_pool2d(x, 3, stride=self.stride, padding=1)
        if self.stride == 2:
            y2 = self.bn1(self.conv1(y2))
        return F.relu(self.sep_conv1(x) + y2)


class CellB(nn.Module):
    def __init__(self, cin: int, cout: int, stride: int = 1):
        super().__init__()
        self.stride = stride
        self.sep_conv1 = SepConv(cin, cout, 7, stride)
        self.sep_conv2 = SepConv(cin, cout, 3, stride)
        self.sep_conv3 = SepConv(cin, cout, 5, stride)
        if stride == 2:
            self.conv1, self.bn1 = _pw(cin, cout), _bn(cout)
        self.conv2, self.bn2 = _pw(2 * cout, cout), _bn(cout)

    def forward(self, x):
        left = F.relu(self.sep_conv1(x) + self.sep_conv2(x))
        pooled = F.max_pool2d(x, 3, stride=self.stride, padding=1)
        if self.stride == 2:
            pooled = self.bn1(self.conv1(pooled))
        right = F.relu(pooled + self.sep_conv3(x))
        return F.relu(self.bn2(self.conv2(torch.cat([left, right], 1))))


class PNASNet(nn.Module):
    def __init__(self, cell, planes: int, cells: int = 6, num_classes: int = 10):
        super().__init__()
        self.conv1, self.bn1 = nn.Conv2d(3, planes, 3, padding=1, bias=False), _bn(planes)
        c = planes

        def run(width, n):
            nonlocal c
            seq = []
            for _ in range(n):
                seq.append(cell(c, width, 1))
                c = width
            return nn.Sequential(*seq)

        def down(width):
            nonlocal c
            m = cell(c, width, 2)
            c = width
            return m

        self.layer1 = run(planes, cells)
        self.layer2 = down(planes * 2)
        self.layer3 = run(planes * 2, cells)
        self.layer4 = down(planes * 4)
        self.layer5 = run(planes * 4, cells)
        self.linear = nn.Linear(planes * 4, num_classes)

    def forward(self, x):
        y = F.relu(self.bn1(self.conv1(x)))
        for m in (self.layer1, self.layer2, self.layer3, self.layer4, self.layer5):
            y = m(y)
        return self.linear(torch.flatten(F.avg_pool2d(y, 8), 1))


_B0 = dict(expansion=(1, 6, 6, 6, 6, 6, 6), outs=(16, 24, 40, 80, 112, 192, 320), depths=(1, 2, 2, 3, 3, 4, 1),
           kernels=(3, 3, 5, 3, 5, 5, 3), strides=(1, 2, 2, 2, 1, 2, 1))

FACTORIES = {
    "MobileNet": MobileNet,
    "MobileNetV2": MobileNetV2,
    "ShuffleNetG2": lambda: ShuffleNet((200, 400, 800), (4, 8, 4), 2),
    "ShuffleNetG3": lambda: ShuffleNet((240, 480, 960), (4, 8, 4), 3),
    "ShuffleNetV2": lambda net_size=1: ShuffleNetV2(net_size),
    "EfficientNetB0": lambda: EfficientNet(**_B0),
    "RegNetX_200MF": lambda: RegNet((1, 1, 4, 7), (24, 56, 152, 368), (1, 1, 2, 2), 8),
    "RegNetX_400MF": lambda: RegNet((1, 2, 7, 12), (32, 64, 160, 384), (1, 1, 2, 2), 16),
    "RegNetY_400MF": lambda: RegNet((1, 2, 7, 12), (32, 64, 160, 384), (1, 1, 2, 2), 16, se_ratio=0.25),
    "PNASNetA": lambda: PNASNet(CellA, 44),
    "PNASNetB": lambda: PNASNet(CellB, 32),
}
