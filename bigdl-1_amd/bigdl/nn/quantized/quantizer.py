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
        from ...utils import config
        if type(m) is L.Linear and not config.get_property("bigdl.int8.quantizeLinear"):
            return m
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


def _link_int8_chains(model):
    """Quantised convs with calibrated scales that feed each other through ReLU / max pooling /
    (evaluation) dropout only, inside a Sequential: the producer writes the consumer's int8 input
    directly (requantised with the consumer's static scale, the ReLU fused into its epilogue), the
    pooling runs on int8, and no bf16 activation or per-image scale pass sits between them — the
    MKL-DNN int8 pipeline of ``MklInt8Convertible`` (scales from ``calcScales``)."""
    from ..containers import Sequential
    from ..layers.activation import Threshold
    from ..layers.pooling import SpatialMaxPooling
    from ..layers.dropout import Dropout
    from ...ops import native_ops as NO
    from ...utils import config
    for s in model.flattened_modules():
        if not isinstance(s, Sequential):
            continue
        mods = s.modules
        for i, a in enumerate(mods):
            if not (isinstance(a, Q.SpatialConvolution) and a.nGroup == 1 and a.nOutputPlane % 16 == 0):
                continue
            j, relu = i + 1, None
            while j < len(mods) and isinstance(mods[j], (Threshold, SpatialMaxPooling, Dropout)):
                m = mods[j]
                if isinstance(m, Threshold):
                    if not (m.threshold == 0.0 and m.value == 0.0):
                        break
                    if j == i + 1:
                        relu = m
                j += 1
            if j >= len(mods) or not isinstance(mods[j], Q.SpatialConvolution):
                continue
            b = mods[j]
            if b.static_scale is None or b.nGroup != 1 or not NO.conv_i8_supported(a.nOutputPlane, b.kernelH,
                                                                                   b.kernelW):
                continue
            if any(isinstance(m, Threshold) and not (m.threshold == 0.0 and m.value == 0.0) for m in mods[i + 1:j]):
                continue
            a._out_qscale = b.static_scale
            if relu is not None:
                a._relu_fused = True
                relu._i8_fused = True
                if config.get_property("bigdl.int8.unsignedActivations"):
                    # a ReLU'd tensor is non-negative: the unsigned code (offset −128) spends all
                    # 256 levels on [0, clip], halving the step of the signed clip / 127 scale
                    a._out_u8 = True
                    a._out_qscale = b.static_scale * 127.0 / 255.0


def quantize(model):
    """Deep-copy ``model`` and return its int8 version (evaluation mode).  Layers calibrated with
    ``calcScales`` quantise their input statically and chain int8 activations between quantised
    convs (:func:`_link_int8_chains`); uncalibrated ones use per-image dynamic scales."""
    from ..fusion import unfuse
    clone = model.cloneModule()
    unfuse(clone)
    q = _convert(clone)
    _link_int8_chains(q)
    q.evaluate()
    return q
