"""Dataset statistics and layer initialisation helpers.

Working versions of the reference's dead helpers (src/utils.py:15-42, quirk
A11): ``get_mean_and_std`` there lacks ``import torch`` and ``init_params``
uses the removed ``init.kaiming_normal`` and tests a tensor's truthiness
(``if m.bias:``).  Here both run, on any device, without a DataLoader.
"""
from __future__ import annotations

from typing import Tuple

import torch
from torch import nn


@torch.no_grad()
def get_mean_and_std(images: torch.Tensor, chunk: int = 4096) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per-channel mean/std of an [N, C, H, W] image tensor (uint8 or float).

    The reference averages per-IMAGE standard deviations (batch size 1); this
    returns the same quantity: mean over images of each image's channel std.
    """
    n, c = images.shape[:2]
    mean = torch.zeros(c, dtype=torch.float64, device=images.device)
    std = torch.zeros(c, dtype=torch.float64, device=images.device)
    for i in range(0, n, chunk):
        x = images[i:i + chunk].double()
        if images.dtype == torch.uint8:
            x = x / 255.0
        flat = x.flatten(2)
        mean += flat.mean(2).sum(0)
        std += flat.std(2, unbiased=False).sum(0)
    return (mean / n).float(), (std / n).float()


@torch.no_grad()
def init_params(net: nn.Module) -> nn.Module:
    """Kaiming-normal conv weights, unit/zero BN, N(0, 1e-3) linear weights, zero biases."""
    for m in net.modules():
        if isinstance(m, nn.Conv2d):
            nn.init.kaiming_normal_(m.weight, mode="fan_out")
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, nn.BatchNorm2d):
            nn.init.ones_(m.weight)
            nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Linear):
            nn.init.normal_(m.weight, std=1e-3)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
    return net


def make_deterministic() -> None:
    """Run-to-run deterministic PyTorch reference (the fp32 / autocast-bf16 engines that the native engine is
    compared against): deterministic algorithms only (an op without one warns instead of failing), the
    deterministic MIOpen convolution solvers (``cudnn.deterministic`` selects them on ROCm, no benchmark
    search) and a fixed rocBLAS / hipBLASLt workspace.  Without this the fp32 reference differs between runs
    by more than the native-vs-fp32 gap being tested."""
    import os

    os.environ.setdefault("CUBLAS_WORKSPACE_CONFIG", ":4096:8")
    torch.use_deterministic_algorithms(True, warn_only=True)
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
