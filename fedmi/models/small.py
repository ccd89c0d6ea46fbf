"""Small federated models: the 2-conv CNN ("LeNet", the headline config) and the
2-layer MLP plumbing model.

State-dict keys and shapes are identical to the reference LeNet
(src/models/lenet.py:5-23: conv1 [6,3,5,5] ... fc3 [10,84]) so checkpoints are
interchangeable with reference peers (``torch.save({'net','acc','epoch'})``).
On GPU the LeNet step does not run through this module: the fused HIP kernels
(csrc/kernels/lenet_kernels.hip) implement it; this module is the fp32
reference the kernels are tested against and the CPU engine's model.
"""
from __future__ import annotations

import torch
from torch import nn
import torch.nn.functional as F


class LeNet(nn.Module):
    """conv(3->6,k5) relu pool2 -> conv(6->16,k5) relu pool2 -> 400 -> 120 -> 84 -> 10."""

    feature_shape = (16, 5, 5)

    def __init__(self, num_classes: int = 10, in_channels: int = 3):
        super().__init__()
        self.conv1 = nn.Conv2d(in_channels, 6, kernel_size=5)
        self.conv2 = nn.Conv2d(6, 16, kernel_size=5)
        self.fc1 = nn.Linear(400, 120)
        self.fc2 = nn.Linear(120, 84)
        self.fc3 = nn.Linear(84, num_classes)

    def features(self, x: torch.Tensor) -> torch.Tensor:
        for conv in (self.conv1, self.conv2):
            x = F.max_pool2d(F.relu(conv(x)), 2)
        return torch.flatten(x, 1)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        h = self.features(x)
        h = F.relu(self.fc1(h))
        h = F.relu(self.fc2(h))
        return self.fc3(h)


class MLP(nn.Module):
    """2-layer perceptron for the CPU plumbing config (synthetic MNIST, BASELINE.json configs[0])."""

    def __init__(self, in_features: int = 784, hidden: int = 200, num_classes: int = 10):
        super().__init__()
        self.fc1 = nn.Linear(in_features, hidden)
        self.fc2 = nn.Linear(hidden, num_classes)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.fc2(F.relu(self.fc1(torch.flatten(x, 1))))
