"""Local training engines (one per federated client)."""
from __future__ import annotations

import torch

from .. import native
from .base import EpochStats, LocalTrainer, TrainerConfig
from .data import FedDataset


def build_trainer(model: str, data: FedDataset, device, cfg: TrainerConfig = TrainerConfig(),
                  init_state=None) -> LocalTrainer:
    """LeNet on a GPU -> fused HIP engine (mandatory, no silent fallback); else PyTorch engine."""
    device = torch.device(device)
    from ..models import _canon

    if _canon(model) == "lenet" and device.type == "cuda" and not native.force_torch_path():
        from .lenet_native import LeNetNativeTrainer

        return LeNetNativeTrainer(data, device, cfg, init_state=init_state)
    from .torch_engine import TorchTrainer

    kw = {}
    if _canon(model) in ("lenet", "mlp"):
        c, h, w = data.train.x.shape[1:]
        kw = {"in_channels": c} if _canon(model) == "lenet" else {"in_features": c * h * w}
    return TorchTrainer(model, data, device, cfg, init_state=init_state, model_kwargs=kw)


__all__ = ["build_trainer", "EpochStats", "LocalTrainer", "TrainerConfig", "FedDataset"]
