"""Hybrid-engine wiring on the CPU: which convs the native MFMA path takes, and that installing it
leaves the reference state dict untouched (fedmi/ops/native_layers.py)."""
import torch
from torch import nn

from fedmi.models import build_model
from fedmi.ops import native_layers


def test_eligibility_rules():
    ok = [nn.Conv2d(64, 128, 3, 1, 1), nn.Conv2d(24, 48, 1), nn.Conv2d(64, 64, 3, 2, 1, bias=False),
          nn.Conv2d(16, 32, 7, 2, 3)]
    bad = [nn.Conv2d(3, 64, 3, 1, 1),                 # stem: C % 8
           nn.Conv2d(64, 64, 3, 1, 1, groups=16),     # grouped, many narrow groups (RegNet)
           nn.Conv2d(64, 64, 3, 1, 1, groups=64),     # depthwise
           nn.Conv2d(64, 64, 3, 1, 2, dilation=2),    # dilated
           nn.Conv2d(36, 48, 1),                      # DenseNet growth-12 widths
           nn.Conv2d(64, 64, 3, 3, 1)]                # stride 3
    assert all(native_layers.conv_eligible(m) for m in ok)
    assert native_layers.grouped_eligible(nn.Conv2d(128, 128, 3, 1, 1, groups=2))
    assert native_layers.dw_eligible(nn.Conv2d(64, 64, 3, 1, 1, groups=64))
    assert not any(native_layers.conv_eligible(m) for m in bad)


def test_install_keeps_state_dict():
    m = build_model("SENet18")
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    names = native_layers.install(m)
    cov = native_layers.coverage(m)
    assert len(names) == cov["native"] > 0 and cov["native_weight_frac"] > 0.99
    assert list(m.state_dict()) == list(sd)
    assert all(torch.equal(m.state_dict()[k], v) for k, v in sd.items())


def test_hybrid_is_gpu_only():
    from fedmi.engine import build_trainer
    from fedmi.engine.data import make_dataset

    data = make_dataset("synthetic-cifar10", device="cpu", n_train=64, n_test=32, seed=0)
    tr = build_trainer("SimpleDLA", data, "cpu")
    assert not tr.hybrid and tr.native_convs == []
