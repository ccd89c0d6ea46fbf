"""Deep Layer Aggregation CIFAR models: DLA and SimpleDLA.

Key-compatible with src/models/dla.py:11-123 and src/models/dla_simple.py:16-116
(base/layer1/layer2 stems, hierarchical Trees of residual blocks joined by
1x1 "Root" aggregation nodes, linear head).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

from .residual import BasicBlock


def _stem(cin: int, cout: int) -> nn.Sequential:
    return nn.Sequential(nn.Conv2d(cin, cout, 3, padding=1, bias=False), nn.BatchNorm2d(cout), nn.ReLU(True))


class Root(nn.Module):
    """Aggregation node: concat -> 1x1 conv -> BN -> ReLU."""

    def __init__(self, cin: int, cout: int, kernel_size: int = 1):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, kernel_size, padding=(kernel_size - 1) // 2, bias=False)
        self.bn = nn.BatchNorm2d(cout)

    def forward(self, xs):
        return F.relu(self.bn(self.conv(torch.cat(xs, 1))))


class Tree(nn.Module):
    """DLA tree: level-1 = two blocks + root; level-L adds nested subtrees and a prev_root block."""

    def __init__(self, cin: int, cout: int, level: int = 1, stride: int = 1):
        super().__init__()
        self.level = level
        self.root = Root((2 if level == 1 else level + 2) * cout, cout)
        if level > 1:
            for i in range(level - 1, 0, -1):
                setattr(self, f"level_{i}", Tree(cin, cout, level=i, stride=stride))
            self.prev_root = BasicBlock(cin, cout, stride)
            self.left_node = BasicBlock(cout, cout, 1)
        else:
            self.left_node = BasicBlock(cin, cout, stride)
        self.right_node = BasicBlock(cout, cout, 1)

    def forward(self, x):
        outs = [self.prev_root(x)] if self.level > 1 else []
        for i in range(self.level - 1, 0, -1):
            x = getattr(self, f"level_{i}")(x)
            outs.append(x)
        x = self.left_node(x)
        outs.append(x)
        outs.append(self.right_node(x))
        return self.root(outs)


class SimpleTree(nn.Module):
    """Binary tree: left subtree -> right subtree, root joins the two."""

    def __init__(self, cin: int, cout: int, level: int = 1, stride: int = 1):
        super().__init__()
        self.root = Root(2 * cout, cout)
        if level == 1:
            self.left_tree = BasicBlock(cin, cout, stride)
            self.right_tree = BasicBlock(cout, cout, 1)
        else:
            self.left_tree = SimpleTree(cin, cout, level - 1, stride)
            self.right_tree = SimpleTree(cout, cout, level - 1, 1)

    def forward(self, x):
        a = self.left_tree(x)
        return self.root([a, self.right_tree(a)])


class _DLABase(nn.Module):
    tree = Tree

    def __init__(self, num_classes: int = 10):
        super().__init__()
        self.base = _stem(3, 16)
        self.layer1 = _stem(16, 16)
        self.layer2 = _stem(16, 32)
        t = self.tree
        self.layer3 = t(32, 64, level=1, stride=1)
        self.layer4 = t(64, 128, level=2, stride=2)
        self.layer5 = t(128, 256, level=2, stride=2)
        self.layer6 = t(256, 512, level=1, stride=2)
        self.linear = nn.Linear(512, num_classes)

    def forward(self, x):
        y = self.base(x)
        for m in (self.layer1, self.layer2, self.layer3, self.layer4, self.layer5, self.layer6):
            y = m(y)
        return self.linear(torch.flatten(F.avg_pool2d(y, 4), 1))


class DLA(_DLABase):
    tree = Tree


class SimpleDLA(_DLABase):
    tree = SimpleTree


FACTORIES = {"DLA": DLA, "SimpleDLA": SimpleDLA}
