"""The kernels a training step launches are fedmi's own ("assert a kernel list").

torch.profiler records every GPU kernel of an eager step; the step of the flagship LeNet engine and
of a native-mode zoo model (the aten backend) must launch no ATen, MIOpen or rocBLAS/hipBLASLt kernel -- except the
library GEMM of a 1x1 / stride-1 weight gradient over <= 2048 pixels, a plain GEMM where one library launch beats
split-K + reduce (fedmi/ops/conv.py WGRAD_GEMM_PIXELS).
"""
import pytest
import torch
from torch.profiler import ProfilerActivity, profile

from fedmi.engine import build_trainer
from fedmi.engine.base import TrainerConfig
from fedmi.engine.data import contiguous_schedule, make_dataset
from fedmi.ops import conv

pytestmark = pytest.mark.gpu

FOREIGN = ("at::native", "miopen", "MIOpen", "Cijk_", "rocblas", "hipblaslt", "igemm_", "naive_conv")


def _kernels(fn):
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        fn()
        torch.cuda.synchronize()
    names = [e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA]
    return [n for n in names if "memcpy" not in n.lower() and "memset" not in n.lower()
            and "copyBuffer" not in n and "fillBuffer" not in n]


def _library_gemm(name: str) -> bool:
    return name.startswith("Cijk_") or "hipblaslt" in name.lower()


def test_lenet_step_launches_only_fedmi_kernels(gpu_device):
    data = make_dataset("synthetic-cifar10", device=gpu_device, n_train=256, n_test=128, seed=0)
    tr = build_trainer("lenet", data, gpu_device, TrainerConfig(seed=1, use_graph=False))
    tr.set_schedule(*contiguous_schedule(256, 128))
    tr.train_epoch()                                   # warm-up (packing, first-touch)
    names = _kernels(tr.train_epoch)
    assert names, "profiler saw no kernels"
    bad = [n for n in names if any(f in n for f in FOREIGN)]
    assert not bad, bad[:10]
    assert any("lenet_sample_step" in n for n in names) and any("lenet_sgd2" in n for n in names), set(names)


@pytest.mark.parametrize("name", ["SimpleDLA", "RegNetX_200MF"])
def test_native_mode_step_launches_only_fedmi_kernels(gpu_device, name):
    data = make_dataset("synthetic-cifar10", device=gpu_device, n_train=256, n_test=64, seed=0)
    tr = build_trainer(name, data, gpu_device, TrainerConfig(batch_size=128, seed=1, augment=False))
    tr.use_graph = False
    x, y = tr._batch(0, 128)                           # input prep (augment / layout) outside the step
    tr.model.train()
    tr._step_body(x, y)                                # warm-up
    names = _kernels(lambda: tr._step_body(x, y))
    # library GEMM kernels only for the plain-GEMM 1x1 / stride-1 WGRADs over <= 2048 pixels (conv.WGRAD_GEMM_PIXELS)
    bad = [n for n in names if any(f in n for f in FOREIGN) and not _library_gemm(n)]
    assert not bad, sorted(set(bad))[:10]
    assert not tr.mode.fallbacks
    assert any("conv_igemm" in n or "conv_tap" in n for n in names)


@pytest.mark.parametrize("name", ["resnet18", "mobilenet"])
def test_cnn_engine_step_launches_only_fedmi_kernels(gpu_device, name):
    """the whole-network CNN engines' captured step (eager here, same launches) is fedmi
    kernels only -- the per-step BN-statistics zeroing rides in sched_next, no ATen fill."""
    data = make_dataset("synthetic-cifar10", device=gpu_device, n_train=256, n_test=128, seed=0)
    tr = build_trainer(name, data, gpu_device, TrainerConfig(seed=1, use_graph=False))
    tr.set_schedule(*contiguous_schedule(256, 128))
    tr.train_epoch()                                   # warm-up (weight images, first-touch)
    tr.counter.zero_()                                 # (epoch bookkeeping fills stay outside the profiled step)
    torch.cuda.synchronize()
    names = _kernels(lambda: tr._train_step(128))      # exactly what one graph replay launches
    assert names, "profiler saw no kernels"
    # the one library call allowed: the plain GEMM of a 1x1 / stride-1 WGRAD over <= 2048 pixels
    # (conv.WGRAD_GEMM_PIXELS: MobileNet's 4x4 / 2x2 pointwise layers), at most one kernel per such conv
    lib = [n for n in names if _library_gemm(n)]
    n_lib = sum(1 for u in tr.units if not u.depthwise and u.R == 1 and u.stride == 1 and u.C == u.Cw
                and 128 * u.P * u.P <= conv.WGRAD_GEMM_PIXELS)
    assert len(lib) <= n_lib, (len(lib), n_lib, sorted(set(lib))[:5])
    bad = [n for n in names if any(f in n for f in FOREIGN) and n not in lib]
    assert not bad, sorted(set(bad))[:10]
    assert any("conv_tap" in n for n in names) and any("sgd_pack" in n for n in names), sorted(set(names))[:20]
    assert sum("wgrad_reduce_multi" in n for n in names) == 1, "deferred WGRAD reductions: one launch per step"
