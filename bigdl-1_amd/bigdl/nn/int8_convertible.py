"""Int8 calibration state of a module (``DL/nn/MklInt8Convertible.scala``): input / output /
weight dimension masks and the per-mask max-abs scales collected by ``calcScales``, serialised in
the ``.bigdl`` fields 17-23 (``isMklInt8Enabled``, ``{input,output,weight}DimMasks`` /
``…Scales``).

``calcScales(input)`` is called after a forward on calibration data: it reads the module's
current ``output`` (no extra forward), appends the scales of input and output (and the weight, for
conv / linear) and recurses through Sequential / ConcatTable / Graph children exactly as the
reference.  A dimension mask selects the dimensions kept separate (bit i = dimension i): mask 0 is
one max over the whole tensor, all bits set is the element-wise |x|.  The int8 kernels of
``bigdl.nn.quantized`` use per-output-channel weight scales (mask 1 on the weight) computed
internally; these recorded scales are what an int8 deployment (or another runtime) consumes.
"""
from __future__ import annotations

from typing import List

import torch

from ..utils.table import Table


def calc_tensor_scale(t: torch.Tensor, mask: int) -> List[float]:
    """Max |x| per index of the masked dimensions (row-major), ``nn/Utils.calcScales``."""
    t = t.detach().float()
    nd = t.dim()
    if mask < 0 or mask > (1 << max(nd, 1)) - 1:
        raise ValueError(f"mask should between [0, {(1 << nd) - 1}]")
    if mask == 0:
        return [float(t.abs().max())] if t.numel() else [0.0]
    keep = [i for i in range(nd) if (mask >> i) & 1]
    red = [i for i in range(nd) if i not in keep]
    a = t.abs()
    if red:
        a = a.amax(dim=red)
    return [float(v) for v in a.reshape(-1).tolist()]


PERCENTILES = (99.9, 99.99, 99.999)


def abs_percentiles(t: torch.Tensor, cap: int = 1 << 22) -> List[float]:
    """|x| at :data:`PERCENTILES` (a strided sample of at most ``cap`` elements for big tensors)."""
    a = t.detach().float().abs().reshape(-1)
    if a.numel() > cap:
        a = a[:: (a.numel() + cap - 1) // cap]
    if a.numel() == 0:
        return [0.0 for _ in PERCENTILES]
    out = []
    for p in PERCENTILES:
        k = min(a.numel(), max(1, int(round(p / 100.0 * a.numel()))))
        out.append(float(a.kthvalue(k).values))
    return out


def _tensors(act):
    if isinstance(act, torch.Tensor):
        return [act]
    if isinstance(act, Table):
        return [v for v in act.values() if isinstance(v, torch.Tensor)]
    return []


class MklInt8Convertible:
    """Mixed into :class:`~bigdl.nn.abstractnn.AbstractModule`."""

    def _i8(self):
        st = self.__dict__.get("_int8_state")
        if st is None:
            st = {"inMask": 0, "outMask": 0, "wMask": 0, "in": [], "out": [], "w": []}
            self.__dict__["_int8_state"] = st
        return st

    # ---- masks -------------------------------------------------------------------------------
    def getInputDimMask(self):
        return self._i8()["inMask"]

    def getOutputDimMask(self):
        return self._i8()["outMask"]

    def getWeightDimMask(self):
        return self._i8()["wMask"]

    def _set_mask(self, key, mask, override):
        self._i8()[key] = int(mask)
        if override:
            for c in self.children():
                c._set_mask(key, mask, override)

    def setInputDimMask(self, mask: int, override_submodules: bool = False):
        self._set_mask("inMask", mask, override_submodules)

    def setOutputDimMask(self, mask: int, override_submodules: bool = False):
        self._set_mask("outMask", mask, override_submodules)

    def setWeightDimMask(self, mask: int, override_submodules: bool = False):
        self._set_mask("wMask", mask, override_submodules)

    # ---- scales ------------------------------------------------------------------------------
    def getInputScales(self):
        return [list(s) for s in self._i8()["in"]]

    def getOutputScales(self):
        return [list(s) for s in self._i8()["out"]]

    def getWeightScales(self):
        return [list(s) for s in self._i8()["w"]]

    def setInputScales(self, scales):
        self._i8()["in"] = [list(map(float, s)) for s in scales]

    def setOutputScales(self, scales):
        self._i8()["out"] = [list(map(float, s)) for s in scales]

    def setWeightScales(self, scales):
        self._i8()["w"] = [list(map(float, s)) for s in scales]

    def appendInputScales(self, s):
        self._i8()["in"].append(list(s))

    def appendOutputScales(self, s):
        self._i8()["out"].append(list(s))

    def appendWeightScales(self, s):
        self._i8()["w"].append(list(s))

    def updateInputScales(self, s, index):
        self._i8()["in"][index] = list(s)

    def updateOutputScales(self, s, index):
        self._i8()["out"][index] = list(s)

    def updateWeightScales(self, s, index):
        self._i8()["w"][index] = list(s)

    def flushWeightScales(self, weight):
        st = self._i8()
        st["w"] = [calc_tensor_scale(weight, st["wMask"])]

    def hasInt8Scales(self) -> bool:
        st = self.__dict__.get("_int8_state")
        return bool(st and (st["in"] or st["out"] or st["w"]))

    # ---- calibration -------------------------------------------------------------------------
    def _module_scales(self, inp, out, weight=None):
        st = self._i8()
        for t in _tensors(inp):
            st["in"].append(calc_tensor_scale(t, st["inMask"]))
            if st["inMask"] == 0:
                # clipping candidates for static int8 activation scales (nn/quantized: the
                # bigdl.int8.calibration rule), beside the reference's max|x|
                st.setdefault("in_pct", []).append(abs_percentiles(t))
        for t in _tensors(out):
            st["out"].append(calc_tensor_scale(t, st["outMask"]))
        if weight is not None:
            st["w"].append(calc_tensor_scale(weight, st["wMask"]))

    def calcScales(self, input):
        """Collect scales from ``input`` and this module's current ``output`` (run a forward on the
        calibration batch first)."""
        if input is None:
            return
        from .containers import Sequential, ConcatTable
        from .graph import Graph
        from .layers.activation import ReLU
        from .layers.conv import SpatialConvolution
        from .layers.linear import Linear
        from .layers.normalization import SpatialBatchNormalization
        from .layers.table_ops import CAddTable
        out = self.output
        if isinstance(self, Graph):
            self._module_scales(input, out)
            for n in self.forward_order:
                x = self._node_inputs.get(n._id) if hasattr(self, "_node_inputs") else None
                if x is not None and isinstance(n.element, _CONVERTIBLE()):
                    n.element.calcScales(x)
        elif isinstance(self, (Linear, SpatialConvolution)):
            w = self.weight
            if isinstance(self, SpatialConvolution) and w.dim() == 5 and w.shape[0] == 1:
                w = w[0]  # nGroup == 1: the 4-D (out, in, kh, kw) weight, as the reference's getWeight
            self._module_scales(input, out, w)
        elif isinstance(self, (ReLU, CAddTable, SpatialBatchNormalization)):
            self._module_scales(input, out)
        elif isinstance(self, Sequential):
            self._module_scales(input, out)
            prev = input
            for m in self.modules:
                if isinstance(m, _CONVERTIBLE()):
                    m.calcScales(prev)
                prev = m.output
        elif isinstance(self, ConcatTable):
            self._module_scales(input, out)
            for m in self.modules:
                if isinstance(m, _CONVERTIBLE()):
                    m.calcScales(input)
        else:
            raise NotImplementedError(f"Int8 conversion is not supported for module: {self.get_name()}")


def _CONVERTIBLE():
    from .containers import Sequential, ConcatTable
    from .graph import Graph
    from .layers.activation import ReLU
    from .layers.conv import SpatialConvolution
    from .layers.linear import Linear
    from .layers.normalization import SpatialBatchNormalization
    from .layers.table_ops import CAddTable
    return (Sequential, ConcatTable, Graph, ReLU, SpatialConvolution, Linear, SpatialBatchNormalization, CAddTable)


def install():
    from .abstractnn import AbstractModule
    for k, v in vars(MklInt8Convertible).items():
        if callable(v) and not k.startswith("__"):
            setattr(AbstractModule, k, v)
