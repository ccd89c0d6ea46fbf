"""Coverage of the native aten backend (fedmi/ops/native_mode.py) on the CPU.

Every aten op a training step (forward + autograd backward) of each zoo family without a
whole-network engine dispatches must have a native implementation (or be a pure metadata op):
the census runs each model's step on the CPU under a recording dispatch mode and checks the
op set against NativeMode's tables.  The numerics of those implementations are GPU tests
(tests/test_native_mode_gpu.py).
"""
import collections

import pytest
import torch
import torch.nn.functional as F
from torch.utils._python_dispatch import TorchDispatchMode

from fedmi.models import build_model
from fedmi.ops import native_mode as nm

# one (small) member per family; the GPU tests train them under the native mode
HYBRID_MODELS = ["densenet_cifar", "DenseNet121", "ResNeXt29_2x64d", "ResNeXt29_32x4d", "DPN26", "ShuffleNetG2",
                 "ShuffleNetG3", "ShuffleNetV2", "SENet18", "EfficientNetB0", "RegNetX_200MF", "RegNetY_400MF",
                 "PNASNetA", "PNASNetB", "DLA", "SimpleDLA"]

# ops the CPU trace shows that the GPU trace does not (CPU-only dropout decomposition is covered:
# bernoulli_ / div_ / mul are native too)
_CPU_ONLY = set()


class _Census(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.ops = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        self.ops[func] += 1
        return func(*args, **(kwargs or {}))


def _step_ops(name):
    torch.manual_seed(0)
    m = build_model(name)
    m.train()
    x = torch.randn(2, 3, 32, 32)
    y = torch.tensor([1, 3])
    with _Census() as c:
        out = m(x)
        F.cross_entropy(out, y).backward()
        m.eval()
        with torch.no_grad():
            m(x)
    return c.ops


@pytest.mark.parametrize("name", HYBRID_MODELS)
def test_every_step_op_is_native(name):
    ops = _step_ops(name)
    known = set(nm._IMPL) | nm._PASSTHROUGH | _CPU_ONLY
    missing = sorted(str(f) for f in ops if f not in known)
    assert not missing, f"{name}: aten ops without a native implementation: {missing}"


def test_tables_disjoint_and_named():
    assert not (set(nm._IMPL) & nm._PASSTHROUGH)
    assert len(nm._IMPL) >= 40
    # every elementwise op code the Python side uses exists in the kernel's enum
    src = open(nm.__file__.replace("fedmi/ops/native_mode.py", "csrc/kernels/zoo_ops.hip")).read()
    for code in ("EW_COPY", "EW_ADD", "EW_MULS", "EW_BNB", "EW_BERN", "EW_ADDS", "EW_DIV"):
        assert code in src


def test_conv_kind_routing():
    k3, s1, s2, p1, d1 = (3, 3), (1, 1), (2, 2), (1, 1), (1, 1)
    assert nm._conv_kind(64, 128, 1, k3, s1, p1, d1) == "mfma"
    assert nm._conv_kind(64, 64, 64, k3, s2, p1, d1) == "dw"
    assert nm._conv_kind(128, 128, 2, k3, s1, p1, d1) == "mfma"         # one MFMA GEMM per group
    assert nm._conv_kind(3, 64, 1, k3, s1, p1, d1) == "mfma"            # stem: C zero-padded to 8
    assert nm._conv_kind(36, 12, 1, (1, 1), s1, (0, 0), d1) == "mfma"   # DenseNet growth widths
    assert nm._conv_kind(128, 128, 32, k3, s1, p1, d1) == "gdense"      # many narrow groups: block-diagonal MFMA
    assert nm._conv_kind(2048, 2048, 32, k3, s1, p1, d1) == "gconv"     # wide groups / channels: direct kernel
    assert nm._conv_kind(60, 60, 12, k3, s1, p1, d1) == "gconv"         # channels off the 8-grid
    assert nm._conv_kind(44, 44, 44, (7, 7), s1, (3, 3), d1) == "dwpad"  # PNASNetA: depthwise on padded channels
    assert nm._conv_kind(60, 60, 3, (1, 1), s1, (0, 0), d1) == "mfma"   # ShuffleNet g3 widths, padded
    assert nm._conv_kind(96, 96, 32, k3, s1, p1, d1) == "gdense"        # DPN cardinality 32
    assert nm._conv_kind(64, 64, 1, k3, (3, 3), p1, d1) == "gconv"      # stride 3


def test_mode_is_transparent_on_cpu():
    """Under the mode, CPU tensors take ATen: same numbers, nothing counted as a fallback."""
    torch.manual_seed(0)
    m = build_model("SimpleDLA")
    x = torch.randn(2, 3, 32, 32)
    ref = m(x)
    mode = nm.NativeMode(strict=True)
    with mode:
        out = m(x)
    assert torch.equal(out, ref)
    assert not mode.fallbacks and not mode.native_ops


def test_hybrid_is_gpu_only():
    from fedmi.engine import build_trainer
    from fedmi.engine.data import make_dataset

    data = make_dataset("synthetic-cifar10", device="cpu", n_train=64, n_test=32, seed=0)
    tr = build_trainer("SimpleDLA", data, "cpu")
    assert not tr.hybrid and tr.mode is None


def test_native_mode_api_used_by_the_trainer():
    """TorchTrainer allocates the dropout RNG counter before capture and reads the fusion counters."""
    mode = nm.NativeMode(fuse=True)
    ctr = mode.rng_ctr("cpu")
    assert ctr.dtype == torch.int32 and ctr.numel() == 4 and mode.rng_ctr("cpu") is ctr
    assert mode.fuse and not mode.fused and not mode.fallbacks
