"""Model registry (explicit, no star-import shadowing — reference quirk A21,
src/models/__init__.py:1-18).

``build_model(name)`` accepts the reference's factory spellings
(``LeNet``, ``VGG('VGG19')`` -> ``vgg19``, ``ResNet18``, ``MobileNet`` ...),
case-insensitively.
"""
from __future__ import annotations

from typing import Callable, Dict

from torch import nn

from .small import LeNet, MLP

_REGISTRY: Dict[str, Callable[..., nn.Module]] = {}


def register(name: str, fn: Callable[..., nn.Module]) -> None:
    _REGISTRY[name.lower()] = fn


def _canon(name: str) -> str:
    n = name.strip().lower().replace("-", "").replace("_", "")
    aliases = {"cnn": "lenet", "2convcnn": "lenet", "twoconvcnn": "lenet", "mobilenetv1": "mobilenet"}
    return aliases.get(n, n)


def build_model(name: str, **kw) -> nn.Module:
    key = _canon(name)
    if key not in _REGISTRY:
        raise KeyError(f"unknown model {name!r}; known: {', '.join(sorted(_REGISTRY))}")
    return _REGISTRY[key](**kw)


def list_models():
    return sorted(_REGISTRY)


register("lenet", LeNet)
register("mlp", MLP)

from . import zoo as _zoo  # noqa: E402,F401  (registers the CIFAR zoo)
