"""Multi-branch / concatenating CIFAR families: VGG, GoogLeNet, DenseNet, DPN.

Key-compatible with the reference zoo:
  VGG        src/models/vgg.py:6-38          (features = Sequential[conv,bn,relu | pool]..., classifier)
  GoogLeNet  src/models/googlenet.py:7-98    (pre_layers, a3..b5 Inception b1..b4, linear)
  DenseNet   src/models/densenet.py:9-99     (conv1, dense1..4, trans1..3, bn, linear)
  DPN        src/models/dpn.py:7-89          (dual path: residual slice-add + dense concat)
"""
from __future__ import annotations

import math
from typing import Dict, List, Sequence

import torch
import torch.nn.functional as F
from torch import nn


def _cbr(cin: int, cout: int, k: int, pad: int = 0, bias: bool = True) -> List[nn.Module]:
    return [nn.Conv2d(cin, cout, k, padding=pad, bias=bias), nn.BatchNorm2d(cout), nn.ReLU(True)]


# --------------------------------------------------------------------------- VGG
VGG_CFG: Dict[str, Sequence] = {
    "VGG11": (64, "M", 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"),
    "VGG13": (64, 64, "M", 128, 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"),
    "VGG16": (64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"),
    "VGG19": (64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M",
              512, 512, 512, 512, "M"),
}


class VGG(nn.Module):
    def __init__(self, name: str = "VGG19", num_classes: int = 10):
        super().__init__()
        mods: List[nn.Module] = []
        c = 3
        for v in VGG_CFG[name.upper()]:
            if v == "M":
                mods.append(nn.MaxPool2d(2, 2))
            else:
                mods += _cbr(c, v, 3, pad=1)
                c = v
        mods.append(nn.AvgPool2d(1, 1))
        self.features = nn.Sequential(*mods)
        self.classifier = nn.Linear(512, num_classes)

    def forward(self, x):
        return self.classifier(torch.flatten(self.features(x), 1))


# --------------------------------------------------------------------------- GoogLeNet
class Inception(nn.Module):
    def __init__(self, cin: int, n1: int, r3: int, n3: int, r5: int, n5: int, npool: int):
        super().__init__()
        self.b1 = nn.Sequential(*_cbr(cin, n1, 1))
        self.b2 = nn.Sequential(*_cbr(cin, r3, 1), *_cbr(r3, n3, 3, 1))
        # the "5x5" branch is two stacked 3x3 convs
        self.b3 = nn.Sequential(*_cbr(cin, r5, 1), *_cbr(r5, n5, 3, 1), *_cbr(n5, n5, 3, 1))
        self.b4 = nn.Sequential(nn.MaxPool2d(3, stride=1, padding=1), *_cbr(cin, npool, 1))

    def forward(self, x):
        return torch.cat([b(x) for b in (self.b1, self.b2, self.b3, self.b4)], 1)


class GoogLeNet(nn.Module):
    STAGES = (
        ("a3", (192, 64, 96, 128, 16, 32, 32)), ("b3", (256, 128, 128, 192, 32, 96, 64)),
        ("a4", (480, 192, 96, 208, 16, 48, 64)), ("b4", (512, 160, 112, 224, 24, 64, 64)),
        ("c4", (512, 128, 128, 256, 24, 64, 64)), ("d4", (512, 112, 144, 288, 32, 64, 64)),
        ("e4", (528, 256, 160, 320, 32, 128, 128)), ("a5", (832, 256, 160, 320, 32, 128, 128)),
        ("b5", (832, 384, 192, 384, 48, 128, 128)),
    )

    def __init__(self, num_classes: int = 10):
        super().__init__()
        self.pre_layers = nn.Sequential(*_cbr(3, 192, 3, 1))
        for name, cfg in self.STAGES:
            setattr(self, name, Inception(*cfg))
        self.maxpool = nn.MaxPool2d(3, stride=2, padding=1)
        self.avgpool = nn.AvgPool2d(8, stride=1)
        self.linear = nn.Linear(1024, num_classes)

    def forward(self, x):
        y = self.pre_layers(x)
        for name, _ in self.STAGES:
            y = getattr(self, name)(y)
            if name in ("b3", "e4"):
                y = self.maxpool(y)
        return self.linear(torch.flatten(self.avgpool(y), 1))


# --------------------------------------------------------------------------- DenseNet
class DenseLayer(nn.Module):
    """BN-ReLU-1x1(4g) -> BN-ReLU-3x3(g), output concatenated in front of the input."""

    def __init__(self, cin: int, growth: int):
        super().__init__()
        self.bn1, self.conv1 = nn.BatchNorm2d(cin), nn.Conv2d(cin, 4 * growth, 1, bias=False)
        self.bn2, self.conv2 = nn.BatchNorm2d(4 * growth), nn.Conv2d(4 * growth, growth, 3, padding=1, bias=False)

    def forward(self, x):
        y = self.conv2(F.relu(self.bn2(self.conv1(F.relu(self.bn1(x))))))
        return torch.cat([y, x], 1)


class Transition(nn.Module):
    def __init__(self, cin: int, cout: int):
        super().__init__()
        self.bn, self.conv = nn.BatchNorm2d(cin), nn.Conv2d(cin, cout, 1, bias=False)

    def forward(self, x):
        return F.avg_pool2d(self.conv(F.relu(self.bn(x))), 2)


class DenseNet(nn.Module):
    def __init__(self, depths: Sequence[int], growth: int = 12, reduction: float = 0.5, num_classes: int = 10):
        super().__init__()
        c = 2 * growth
        self.conv1 = nn.Conv2d(3, c, 3, padding=1, bias=False)
        for i, n in enumerate(depths, start=1):
            setattr(self, f"dense{i}", nn.Sequential(*[DenseLayer(c + j * growth, growth) for j in range(n)]))
            c += n * growth
            if i < len(depths):
                cout = int(math.floor(c * reduction))
                setattr(self, f"trans{i}", Transition(c, cout))
                c = cout
        self.bn = nn.BatchNorm2d(c)
        self.linear = nn.Linear(c, num_classes)
        self._n = len(depths)

    def forward(self, x):
        y = self.conv1(x)
        for i in range(1, self._n):
            y = getattr(self, f"trans{i}")(getattr(self, f"dense{i}")(y))
        y = getattr(self, f"dense{self._n}")(y)
        y = F.avg_pool2d(F.relu(self.bn(y)), 4)
        return self.linear(torch.flatten(y, 1))


# --------------------------------------------------------------------------- DPN
class DualPathBlock(nn.Module):
    def __init__(self, cin: int, mid: int, out: int, dense: int, stride: int, first: bool):
        super().__init__()
        self.out_planes, self.dense_depth = out, dense
        self.conv1, self.bn1 = nn.Conv2d(cin, mid, 1, bias=False), nn.BatchNorm2d(mid)
        self.conv2 = nn.Conv2d(mid, mid, 3, stride=stride, padding=1, groups=32, bias=False)
        self.bn2 = nn.BatchNorm2d(mid)
        self.conv3, self.bn3 = nn.Conv2d(mid, out + dense, 1, bias=False), nn.BatchNorm2d(out + dense)
        self.shortcut = nn.Sequential()
        if first:
            self.shortcut = nn.Sequential(nn.Conv2d(cin, out + dense, 1, stride=stride, bias=False),
                                          nn.BatchNorm2d(out + dense))

    def forward(self, x):
        y = F.relu(self.bn1(self.conv1(x)))
        y = F.relu(self.bn2(self.conv2(y)))
        y = self.bn3(self.conv3(y))
        s = self.shortcut(x)
        d = self.out_planes
        return F.relu(torch.cat([s[:, :d] + y[:, :d], s[:, d:], y[:, d:]], 1))


class DPN(nn.Module):
    def __init__(self, mids, outs, depths, dense, num_classes: int = 10):
        super().__init__()
        self.conv1, self.bn1 = nn.Conv2d(3, 64, 3, padding=1, bias=False), nn.BatchNorm2d(64)
        last = 64
        stages = []
        for mid, out, n, dd, stride in zip(mids, outs, depths, dense, (1, 2, 2, 2)):
            blocks = []
            for i, s in enumerate([stride] + [1] * (n - 1)):
                blocks.append(DualPathBlock(last, mid, out, dd, s, i == 0))
                last = out + (i + 2) * dd
            stages.append(nn.Sequential(*blocks))
        self.layer1, self.layer2, self.layer3, self.layer4 = stages
        self.linear = nn.Linear(outs[3] + (depths[3] + 1) * dense[3], num_classes)

    def forward(self, x):
        y = F.relu(self.bn1(self.conv1(x)))
        y = self.layer4(self.layer3(self.layer2(self.layer1(y))))
        return self.linear(torch.flatten(F.avg_pool2d(y, 4), 1))


_DPN_MID, _DPN_OUT, _DPN_DENSE = (96, 192, 384, 768), (256, 512, 1024, 2048), (16, 32, 24, 128)

FACTORIES = {
    "VGG11": lambda: VGG("VGG11"), "VGG13": lambda: VGG("VGG13"),
    "VGG16": lambda: VGG("VGG16"), "VGG19": lambda: VGG("VGG19"),
    "GoogLeNet": GoogLeNet,
    "DenseNet121": lambda: DenseNet([6, 12, 24, 16], growth=32),
    "DenseNet169": lambda: DenseNet([6, 12, 32, 32], growth=32),
    "DenseNet201": lambda: DenseNet([6, 12, 48, 32], growth=32),
    "DenseNet161": lambda: DenseNet([6, 12, 36, 24], growth=48),
    "densenet_cifar": lambda: DenseNet([6, 12, 24, 16], growth=12),
    "DPN26": lambda: DPN(_DPN_MID, _DPN_OUT, (2, 2, 2, 2), _DPN_DENSE),
    "DPN92": lambda: DPN(_DPN_MID, _DPN_OUT, (3, 4, 20, 3), _DPN_DENSE),
}
