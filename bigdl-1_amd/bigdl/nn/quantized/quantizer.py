"""Model → int8 model rewrite (``DL/nn/quantized/Quantizer.scala:27-133``, entry
``Quantization.quantize`` :168-179): clone the model, then replace every registered float layer
(SpatialConvolution, SpatialDilatedConvolution, Linear) by its quantized twin, walking containers,
graphs and recurrent cells."""
from __future__ import annotations

from typing import Callable, Dict

from .. import layers as L
from . import layers as Q

_REGISTRY: Dict[type, Callable] = {}


def register(float_cls: type, convert: Callable):
    if float_cls in _REGISTRY:
        raise ValueError(f"Module: {float_cls.__name__} has been registered.")
    _REGISTRY[float_cls] = convert


register(L.SpatialConvolution, Q.SpatialConvolution.from_float)
register(L.SpatialShareConvolution, Q.SpatialConvolution.from_float)
register(L.SpatialDilatedConvolution, Q.SpatialDilatedConvolution.from_float)
register(L.Linear, Q.Linear.from_float)


def _convert(m):
    conv = _REGISTRY.get(type(m))
    if conv is not None:
        return conv(m)
    from ..graph import Graph
    if isinstance(m, Graph):
        for node in m.forward_order:
            node.element = _convert(node.element)
        m.modules = [n.element for n in m.forward_order]
        return m
    if hasattr(m, "cell") and getattr(m, "cell") is not None and not hasattr(m, "modules"):
        m.cell = _convert(m.cell)
        return m
    mods = getattr(m, "modules", None)
    if isinstance(mods, list):
        for i, c in enumerate(mods):
            mods[i] = _convert(c)
    return m


def quantize(model):
    """Deep-copy ``model`` and return its int8 version (evaluation mode)."""
    from ..fusion import unfuse
    clone = model.cloneModule()
    unfuse(clone)
    q = _convert(clone)
    q.evaluate()
    return q
