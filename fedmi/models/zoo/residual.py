"""Residual CIFAR families: ResNet, PreAct-ResNet, ResNeXt-29, SENet-18.

State-dict keys/shapes are identical to the reference zoo so checkpoints move
between fedmi and reference peers:
  ResNet          src/models/resnet.py:14-124      (conv1,bn1,layer1..4,linear)
  PreActResNet    src/models/preact_resnet.py:12-110
  ResNeXt29       src/models/resnext.py:10-87      (3 stages, grouped 3x3)
  SENet18         src/models/senet.py:45-109       (PreAct blocks + SE via 1x1 convs)
All take 3x32x32 inputs and produce 10 logits.
"""
from __future__ import annotations

from typing import List, Sequence

import torch
import torch.nn.functional as F
from torch import nn

from .pool import global_avg_pool


def _conv3(cin: int, cout: int, stride: int = 1, groups: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, 3, stride=stride, padding=1, groups=groups, bias=False)


def _conv1(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, 1, stride=stride, bias=False)


def _projection(cin: int, cout: int, stride: int, with_bn: bool = True) -> nn.Sequential:
    """1x1 (strided) projection used when a block changes shape; empty Sequential otherwise."""
    if stride == 1 and cin == cout:
        return nn.Sequential()
    mods: List[nn.Module] = [_conv1(cin, cout, stride)]
    if with_bn:
        mods.append(nn.BatchNorm2d(cout))
    return nn.Sequential(*mods)


# --------------------------------------------------------------------------- ResNet
class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin: int, planes: int, stride: int = 1):
        super().__init__()
        self.conv1, self.bn1 = _conv3(cin, planes, stride), nn.BatchNorm2d(planes)
        self.conv2, self.bn2 = _conv3(planes, planes), nn.BatchNorm2d(planes)
        self.shortcut = _projection(cin, planes, stride)

    def forward(self, x):
        y = self.bn2(self.conv2(F.relu(self.bn1(self.conv1(x)))))
        return F.relu(y + self.shortcut(x))


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin: int, planes: int, stride: int = 1):
        super().__init__()
        out = planes * self.expansion
        self.conv1, self.bn1 = _conv1(cin, planes), nn.BatchNorm2d(planes)
        self.conv2, self.bn2 = _conv3(planes, planes, stride), nn.BatchNorm2d(planes)
        self.conv3, self.bn3 = _conv1(planes, out), nn.BatchNorm2d(out)
        self.shortcut = _projection(cin, out, stride)

    def forward(self, x):
        y = F.relu(self.bn1(self.conv1(x)))
        y = F.relu(self.bn2(self.conv2(y)))
        y = self.bn3(self.conv3(y))
        return F.relu(y + self.shortcut(x))


def _stage(block, cin: int, planes: int, n: int, stride: int):
    blocks = []
    for s in [stride] + [1] * (n - 1):
        blocks.append(block(cin, planes, s))
        cin = planes * block.expansion
    return nn.Sequential(*blocks), cin


class ResNet(nn.Module):
    def __init__(self, block, depths: Sequence[int], num_classes: int = 10):
        super().__init__()
        self.conv1, self.bn1 = _conv3(3, 64), nn.BatchNorm2d(64)
        c = 64
        self.layer1, c = _stage(block, c, 64, depths[0], 1)
        self.layer2, c = _stage(block, c, 128, depths[1], 2)
        self.layer3, c = _stage(block, c, 256, depths[2], 2)
        self.layer4, c = _stage(block, c, 512, depths[3], 2)
        self.linear = nn.Linear(c, num_classes)

    def forward(self, x):
        y = F.relu(self.bn1(self.conv1(x)))
        y = self.layer4(self.layer3(self.layer2(self.layer1(y))))
        return self.linear(torch.flatten(F.avg_pool2d(y, 4), 1))


# --------------------------------------------------------------------------- PreAct
class PreActBlock(nn.Module):
    expansion = 1

    def __init__(self, cin: int, planes: int, stride: int = 1):
        super().__init__()
        self.bn1, self.conv1 = nn.BatchNorm2d(cin), _conv3(cin, planes, stride)
        self.bn2, self.conv2 = nn.BatchNorm2d(planes), _conv3(planes, planes)
        if stride != 1 or cin != planes:
            self.shortcut = nn.Sequential(_conv1(cin, planes, stride))

    def forward(self, x):
        pre = F.relu(self.bn1(x))
        skip = self.shortcut(pre) if hasattr(self, "shortcut") else x
        y = self.conv2(F.relu(self.bn2(self.conv1(pre))))
        return y + skip


class PreActBottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin: int, planes: int, stride: int = 1):
        super().__init__()
        out = planes * self.expansion
        self.bn1, self.conv1 = nn.BatchNorm2d(cin), _conv1(cin, planes)
        self.bn2, self.conv2 = nn.BatchNorm2d(planes), _conv3(planes, planes, stride)
        self.bn3, self.conv3 = nn.BatchNorm2d(planes), _conv1(planes, out)
        if stride != 1 or cin != out:
            self.shortcut = nn.Sequential(_conv1(cin, out, stride))

    def forward(self, x):
        pre = F.relu(self.bn1(x))
        skip = self.shortcut(pre) if hasattr(self, "shortcut") else x
        y = self.conv1(pre)
        y = self.conv2(F.relu(self.bn2(y)))
        y = self.conv3(F.relu(self.bn3(y)))
        return y + skip


class PreActResNet(nn.Module):
    def __init__(self, block, depths: Sequence[int], num_classes: int = 10):
        super().__init__()
        self.conv1 = _conv3(3, 64)
        c = 64
        self.layer1, c = _stage(block, c, 64, depths[0], 1)
        self.layer2, c = _stage(block, c, 128, depths[1], 2)
        self.layer3, c = _stage(block, c, 256, depths[2], 2)
        self.layer4, c = _stage(block, c, 512, depths[3], 2)
        self.linear = nn.Linear(c, num_classes)

    def forward(self, x):
        y = self.layer4(self.layer3(self.layer2(self.layer1(self.conv1(x)))))
        return self.linear(torch.flatten(F.avg_pool2d(y, 4), 1))


# --------------------------------------------------------------------------- ResNeXt
class ResNeXtBlock(nn.Module):
    expansion = 2

    def __init__(self, cin: int, cardinality: int, width: int, stride: int = 1):
        super().__init__()
        gw = cardinality * width
        out = self.expansion * gw
        self.conv1, self.bn1 = _conv1(cin, gw), nn.BatchNorm2d(gw)
        self.conv2, self.bn2 = _conv3(gw, gw, stride, groups=cardinality), nn.BatchNorm2d(gw)
        self.conv3, self.bn3 = _conv1(gw, out), nn.BatchNorm2d(out)
        self.shortcut = _projection(cin, out, stride)

    def forward(self, x):
        y = F.relu(self.bn1(self.conv1(x)))
        y = F.relu(self.bn2(self.conv2(y)))
        y = self.bn3(self.conv3(y))
        return F.relu(y + self.shortcut(x))


class ResNeXt(nn.Module):
    def __init__(self, depths: Sequence[int], cardinality: int, width: int, num_classes: int = 10):
        super().__init__()
        self.conv1, self.bn1 = _conv1(3, 64), nn.BatchNorm2d(64)
        c, w = 64, width
        stages = []
        for n, stride in zip(depths, (1, 2, 2)):
            blocks = []
            for s in [stride] + [1] * (n - 1):
                blocks.append(ResNeXtBlock(c, cardinality, w, s))
                c = ResNeXtBlock.expansion * cardinality * w
            stages.append(nn.Sequential(*blocks))
            w *= 2                                  # bottleneck width doubles per stage
        self.layer1, self.layer2, self.layer3 = stages
        self.linear = nn.Linear(cardinality * width * 8, num_classes)

    def forward(self, x):
        y = F.relu(self.bn1(self.conv1(x)))
        y = self.layer3(self.layer2(self.layer1(y)))
        return self.linear(torch.flatten(F.avg_pool2d(y, 8), 1))


# --------------------------------------------------------------------------- SENet
class SEPreActBlock(nn.Module):
    """Pre-activation basic block with squeeze-excitation (1x1 convs as FCs)."""

    def __init__(self, cin: int, planes: int, stride: int = 1):
        super().__init__()
        self.bn1, self.conv1 = nn.BatchNorm2d(cin), _conv3(cin, planes, stride)
        self.bn2, self.conv2 = nn.BatchNorm2d(planes), _conv3(planes, planes)
        if stride != 1 or cin != planes:
            self.shortcut = nn.Sequential(_conv1(cin, planes, stride))
        self.fc1 = nn.Conv2d(planes, planes // 16, 1)
        self.fc2 = nn.Conv2d(planes // 16, planes, 1)

    def forward(self, x):
        pre = F.relu(self.bn1(x))
        skip = self.shortcut(pre) if hasattr(self, "shortcut") else x
        y = self.conv2(F.relu(self.bn2(self.conv1(pre))))
        gate = torch.sigmoid(self.fc2(F.relu(self.fc1(global_avg_pool(y)))))
        return y * gate + skip


class SENet(nn.Module):
    def __init__(self, depths: Sequence[int], num_classes: int = 10):
        super().__init__()
        self.conv1, self.bn1 = _conv3(3, 64), nn.BatchNorm2d(64)
        c = 64
        stages = []
        for planes, n, stride in zip((64, 128, 256, 512), depths, (1, 2, 2, 2)):
            blocks = []
            for s in [stride] + [1] * (n - 1):
                blocks.append(SEPreActBlock(c, planes, s))
                c = planes
            stages.append(nn.Sequential(*blocks))
        self.layer1, self.layer2, self.layer3, self.layer4 = stages
        self.linear = nn.Linear(512, num_classes)

    def forward(self, x):
        y = F.relu(self.bn1(self.conv1(x)))
        y = self.layer4(self.layer3(self.layer2(self.layer1(y))))
        return self.linear(torch.flatten(F.avg_pool2d(y, 4), 1))


FACTORIES = {
    "ResNet18": lambda: ResNet(BasicBlock, [2, 2, 2, 2]),
    "ResNet34": lambda: ResNet(BasicBlock, [3, 4, 6, 3]),
    "ResNet50": lambda: ResNet(Bottleneck, [3, 4, 6, 3]),
    "ResNet101": lambda: ResNet(Bottleneck, [3, 4, 23, 3]),
    "ResNet152": lambda: ResNet(Bottleneck, [3, 8, 36, 3]),
    "PreActResNet18": lambda: PreActResNet(PreActBlock, [2, 2, 2, 2]),
    "PreActResNet34": lambda: PreActResNet(PreActBlock, [3, 4, 6, 3]),
    "PreActResNet50": lambda: PreActResNet(PreActBottleneck, [3, 4, 6, 3]),
    "PreActResNet101": lambda: PreActResNet(PreActBottleneck, [3, 4, 23, 3]),
    "PreActResNet152": lambda: PreActResNet(PreActBottleneck, [3, 8, 36, 3]),
    "ResNeXt29_2x64d": lambda: ResNeXt([3, 3, 3], 2, 64),
    "ResNeXt29_4x64d": lambda: ResNeXt([3, 3, 3], 4, 64),
    "ResNeXt29_8x64d": lambda: ResNeXt([3, 3, 3], 8, 64),
    "ResNeXt29_32x4d": lambda: ResNeXt([3, 3, 3], 32, 4),
    "SENet18": lambda: SENet([2, 2, 2, 2]),
}
