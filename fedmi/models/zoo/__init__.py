"""CIFAR model zoo (reference src/models/*), registered by their reference
factory names (case/underscore-insensitive in ``fedmi.models.build_model``)."""
from __future__ import annotations

from .. import register, _canon
from . import aggregation, mobile, multibranch, residual

FACTORIES = {}
for _mod in (residual, multibranch, mobile, aggregation):
    FACTORIES.update(_mod.FACTORIES)

for _name, _fn in FACTORIES.items():
    register(_canon(_name), _fn)

__all__ = ["FACTORIES"]
