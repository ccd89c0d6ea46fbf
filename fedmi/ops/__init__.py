"""Torch-facing wrappers over fedmi's hand-written HIP/CDNA4 kernels.

* :mod:`fedmi.ops.conv` — implicit-GEMM MFMA convolution fwd / dgrad / wgrad (NHWC bf16)
* :mod:`fedmi.ops.cnn`  — BatchNorm (+ReLU, +residual) fwd/bwd, classifier head + CE, input prep
* :mod:`fedmi.ops.flat` — flat-buffer SGD / FedAvg reduce / scale, compression kernels

Every wrapper launches on torch's current stream (graph-capturable) and raises
if the native extension is missing: there is no silent PyTorch fallback.
"""
from . import cnn, conv, flat  # noqa: F401
