"""Global average pooling shared by the squeeze-excite blocks and 1x1 heads of the zoo.

``F.adaptive_avg_pool2d(x, (1, 1))`` / ``F.avg_pool2d(x, x.size(2))`` in the reference
(src/models/efficientnet.py:36, :145; regnet.py:21, :104; senet.py:34, :69) is the spatial mean;
it is computed here as an fp32 mean so that bf16 channels-last
activations (hybrid engine) reduce in fp32.  It also replaces PyTorch-ROCm's bf16 adaptive pool
kernel, which produced NaNs under HIP-graph replay of a training step
(profiles/hybrid_graph_nan_diag_r1.txt).  For fp32 inputs the result equals the adaptive pool.
"""
import torch


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    return x.float().mean((2, 3), keepdim=True).to(x.dtype)
