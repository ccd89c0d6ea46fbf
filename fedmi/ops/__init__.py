"""Torch-facing wrappers over fedmi's hand-written HIP/CDNA4 kernels.

* :mod:`fedmi.ops.conv` — implicit-GEMM MFMA convolution fwd / dgrad / wgrad (NHWC bf16), depthwise
* :mod:`fedmi.ops.cnn`  — BatchNorm (+ReLU, +residual) fwd/bwd, classifier head + CE, input prep, pooling
* :mod:`fedmi.ops.native_mode` — the aten backend (TorchDispatchMode) for the zoo families without a
  whole-network engine

Every wrapper launches on torch's current stream (graph-capturable) and raises
if the native extension is missing: there is no silent PyTorch fallback.
"""
from . import cnn, conv  # noqa: F401
