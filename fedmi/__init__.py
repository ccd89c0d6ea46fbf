"""fedmi — an MI355X-native federated-learning engine.

Same capabilities as the gRPC FedAvg system amolahinge/739-839-federated-learning-using-grpc
(primary/backup coordinator, N clients, ``federated.proto`` Trainer service,
``{'net','acc','epoch'}`` checkpoints, ``-c Y`` compression), re-designed for
AMD Instinct MI355X (gfx950):

* one client = one GPU process; local SGD epochs run as hand-written CDNA4 HIP
  kernels (MFMA/LDS) replayed from a hipGraph by a native C++ executor;
* FedAvg is an RCCL all-reduce over xGMI instead of a gRPC parameter server;
* gRPC (unchanged wire schema) stays as the control plane.

Import order matters on ROCm: ``torch`` is imported first so its bundled HIP
runtime is the one the native extension binds to.
"""
import torch  # noqa: F401  (must precede the native extension)

__version__ = "0.1.0"

__all__ = ["__version__"]
