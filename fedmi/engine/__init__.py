"""Local training engines (one per federated client)."""
from __future__ import annotations


import torch

from .. import native
from .base import EpochStats, LocalTrainer, TrainerConfig
from .data import FedDataset


# zoo models with a native (hand-written HIP) training engine on the GPU
NATIVE_CNNS = ("resnet18", "resnet34", "resnet50", "resnet101", "resnet152", "mobilenet", "mobilenetv2", "vgg11",
               "vgg13", "vgg16", "vgg19", "preactresnet18", "preactresnet34", "preactresnet50", "preactresnet101",
               "preactresnet152", "googlenet")


def build_trainer(model: str, data: FedDataset, device, cfg: TrainerConfig = TrainerConfig(),
                  init_state=None) -> LocalTrainer:
    """On a GPU: LeNet -> fused HIP engine; ResNet / MobileNet / MobileNetV2 -> the implicit-GEMM +
    BN-fused HIP engine (mandatory, no silent fallback).  Other zoo models -> the generic engine with
    every aten op of the step on fedmi's HIP kernels (:class:`fedmi.ops.native_mode.NativeMode`, bf16
    channels-last activations, graph-replayed; ``FEDMI_TORCH_PATH=1``: plain PyTorch fp32); CPU runs -> the
    generic PyTorch engine."""
    device = torch.device(device)
    from ..models import _canon

    if device.type == "cuda" and not native.force_torch_path():
        if _canon(model) == "lenet":
            from .lenet_native import LeNetNativeTrainer

            return LeNetNativeTrainer(data, device, cfg, init_state=init_state)
        if _canon(model) in NATIVE_CNNS and tuple(data.train.x.shape[1:]) == (3, 32, 32):
            from .cnn_native import CNNNativeTrainer

            return CNNNativeTrainer(model, data, device, cfg, init_state=init_state)
    from .torch_engine import TorchTrainer

    kw = {}
    if _canon(model) in ("lenet", "mlp"):
        c, h, w = data.train.x.shape[1:]
        kw = {"in_channels": c} if _canon(model) == "lenet" else {"in_features": c * h * w}
    # zoo models without a whole-network engine: PyTorch autograd over the native aten backend
    hybrid = device.type == "cuda" and not native.force_torch_path() and _canon(model) != "lenet"
    return TorchTrainer(model, data, device, cfg, init_state=init_state, model_kwargs=kw, hybrid=hybrid)


__all__ = ["build_trainer", "EpochStats", "LocalTrainer", "TrainerConfig", "FedDataset"]
