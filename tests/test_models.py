"""Model zoo: every reference factory exists, forwards 3x32x32 -> 10 logits, and
has EXACTLY the reference state-dict keys and shapes (checkpoint interchange
with reference peers).  The reference model sources are imported read-only
from /root/reference/src/models when present."""
import importlib.util
from pathlib import Path

import pytest
import torch

from fedmi.models import build_model, list_models

REF = Path("/root/reference/src/models")

# (our registry name, reference file, reference factory expression)
CASES = [
    ("LeNet", "lenet", "LeNet()"),
    ("VGG11", "vgg", "VGG('VGG11')"), ("VGG19", "vgg", "VGG('VGG19')"),
    ("ResNet18", "resnet", "ResNet18()"), ("ResNet50", "resnet", "ResNet50()"),
    ("PreActResNet18", "preact_resnet", "PreActResNet18()"), ("PreActResNet50", "preact_resnet", "PreActResNet50()"),
    ("GoogLeNet", "googlenet", "GoogLeNet()"),
    ("DenseNet121", "densenet", "DenseNet121()"), ("densenet_cifar", "densenet", "densenet_cifar()"),
    ("ResNeXt29_2x64d", "resnext", "ResNeXt29_2x64d()"), ("ResNeXt29_32x4d", "resnext", "ResNeXt29_32x4d()"),
    ("MobileNet", "mobilenet", "MobileNet()"), ("MobileNetV2", "mobilenetv2", "MobileNetV2()"),
    ("DPN26", "dpn", "DPN26()"),
    ("ShuffleNetV2", "shufflenetv2", "ShuffleNetV2(1)"),
    ("SENet18", "senet", "SENet18()"),
    ("EfficientNetB0", "efficientnet", "EfficientNetB0()"),
    ("RegNetX_200MF", "regnet", "RegNetX_200MF()"), ("RegNetY_400MF", "regnet", "RegNetY_400MF()"),
    ("PNASNetA", "pnasnet", "PNASNetA()"), ("PNASNetB", "pnasnet", "PNASNetB()"),
    ("DLA", "dla", "DLA()"), ("SimpleDLA", "dla_simple", "SimpleDLA()"),
]

# parameter counts of the reference zoo (exact for LeNet, 3 s.f. otherwise)
PARAMS = {"LeNet": 62006, "VGG11": 9.23e6, "VGG19": 20.04e6, "ResNet18": 11.17e6, "ResNet50": 23.52e6,
          "PreActResNet18": 11.17e6, "GoogLeNet": 6.17e6, "DenseNet121": 6.96e6, "densenet_cifar": 1.00e6,
          "ResNeXt29_2x64d": 9.13e6, "MobileNet": 3.22e6, "MobileNetV2": 2.30e6, "DPN26": 11.57e6,
          "DPN92": 34.24e6, "ShuffleNetV2": 1.26e6, "SENet18": 11.26e6, "EfficientNetB0": 3.60e6,
          "RegNetX_200MF": 2.32e6, "RegNetY_400MF": 5.71e6, "PNASNetA": 0.13e6, "PNASNetB": 0.45e6,
          "DLA": 16.29e6, "SimpleDLA": 15.14e6}


def _ref_model(fname, expr):
    if not (REF / f"{fname}.py").exists():
        pytest.skip("reference model sources not mounted")
    spec = importlib.util.spec_from_file_location(f"_ref_{fname}", REF / f"{fname}.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return eval(expr, vars(mod))  # noqa: S307  (reference factory call, e.g. "ResNet18()")


@pytest.mark.parametrize("name,fname,expr", CASES, ids=[c[0] for c in CASES])
def test_state_dict_matches_reference(name, fname, expr):
    torch.manual_seed(0)
    ours = build_model(name)
    ref = _ref_model(fname, expr)
    so, sr = ours.state_dict(), ref.state_dict()
    assert list(so) == list(sr) or set(so) == set(sr), set(so) ^ set(sr)
    for k in sr:
        assert so[k].shape == sr[k].shape, k
    # weights are interchangeable: load the reference's and reproduce its outputs
    ours.load_state_dict(sr)
    ours.eval()
    ref.eval()
    x = torch.randn(2, 3, 32, 32)
    with torch.no_grad():
        assert torch.allclose(ours(x), ref(x), atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("name", sorted(PARAMS))
def test_param_counts(name):
    n = sum(p.numel() for p in build_model(name).parameters())
    assert abs(n - PARAMS[name]) <= max(0.0, 0.006 * PARAMS[name]) if name != "LeNet" else n == 62006


def test_registry_covers_reference_factories():
    names = set(list_models())
    for n in ["lenet", "vgg11", "vgg13", "vgg16", "vgg19", "resnet18", "resnet34", "resnet50", "resnet101",
              "resnet152", "preactresnet18", "preactresnet152", "googlenet", "densenet121", "densenet169",
              "densenet201", "densenet161", "densenetcifar", "resnext292x64d", "resnext294x64d",
              "resnext298x64d", "resnext2932x4d", "mobilenet", "mobilenetv2", "dpn26", "dpn92",
              "shufflenetg2", "shufflenetg3", "shufflenetv2", "senet18", "efficientnetb0", "regnetx200mf",
              "regnetx400mf", "regnety400mf", "pnasneta", "pnasnetb", "dla", "simpledla", "mlp"]:
        assert n in names, n


def test_shufflenet_v1_constructs_and_trains_a_step():
    """Reference ShuffleNetG2/G3 cannot be built (float channels, quirk A12); ours can."""
    for name in ("ShuffleNetG2", "ShuffleNetG3"):
        m = build_model(name)
        out = m(torch.randn(2, 3, 32, 32))
        assert out.shape == (2, 10)
        out.sum().backward()


def test_mlp_forward():
    m = build_model("mlp")
    assert m(torch.randn(4, 1, 28, 28)).shape == (4, 10)
