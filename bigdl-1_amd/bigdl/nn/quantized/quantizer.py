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


def _fold_bn(model):
    """Fold every evaluation-mode BatchNormalization that directly follows a convolution inside a
    Sequential into that convolution's weights and bias (the reference's int8 pipeline fuses conv + BN
    before quantising, DL/nn/mkldnn/Fusion.scala:79-118): w' = w·γ/√(σ²+ε), b' = (b − μ)·γ/√(σ²+ε) + β.
    The BN becomes an Identity.  Calibrated input scales are unaffected (a conv's input does not change)."""
    import torch
    from ..containers import Sequential
    from ..layers.normalization import BatchNormalization
    from ..layers.shape import Identity
    for s in model.flattened_modules():
        if not isinstance(s, Sequential):
            continue
        mods = s.modules
        for i in range(len(mods) - 1):
            a, b = mods[i], mods[i + 1]
            if type(a) not in _REGISTRY or type(a) is L.Linear or not isinstance(b, BatchNormalization):
                continue
            if b.runningMean is None or b.runningVar is None or b.runningMean.numel() != a.nOutputPlane:
                continue
            with torch.no_grad():
                inv = (b.runningVar.float() + b.eps).rsqrt()
                g = b.weight.detach().float().reshape(-1) * inv if getattr(b, "affine", True) and b.weight is not None \
                    else inv
                beta = b.bias.detach().float().reshape(-1) if getattr(b, "affine", True) and b.bias is not None \
                    else torch.zeros_like(inv)
                w = a.weight
                shape = [1] * w.dim()
                if w.dim() == 5:  # (groups, out/groups, in/groups, kh, kw)
                    gs = g.reshape(w.shape[0], w.shape[1], 1, 1, 1)
                else:
                    shape[0] = -1
                    gs = g.reshape(shape)
                w.mul_(gs.to(w.dtype))
                b0 = a.bias.detach().float().reshape(-1) if (a.withBias and a.bias is not None) \
                    else torch.zeros_like(inv)
                a._folded_bias = ((b0 - b.runningMean.float()) * g + beta).clone()
            bst = b.__dict__.get("_int8_state")
            if bst and bst.get("out") and bst.get("outMask", 0) == 0:
                # the calibrated output range of the folded pair (the BN's output): a projection
                # shortcut writes its int8 residual with it
                a.__dict__["_folded_out_amax"] = max(float(v[0]) for v in bst["out"] if v)
            mods[i + 1] = Identity().set_name(b.get_name())
    return model


from ..containers import Container as _Container  # noqa: E402


class Int8ResidualBlock(_Container):
    """A residual block ``ReLU(branch(x) + shortcut(x))`` of a quantised model whose branch ends in a
    calibrated int8 convolution: the shortcut runs first, then the branch, and its last convolution sums
    the shortcut in its epilogue before the ReLU and requantises for the next block (conv + sum,
    DL/nn/mkldnn/Fusion.scala:120-165) — the sum and the ReLU never exist as separate passes.  An
    identity shortcut passes the block's int8 input itself (read with its scale); a projection shortcut
    writes bf16.  ``_out_qscale`` / ``_out_u8`` (set by the linker) make the block's output int8 for the
    next quantised layer."""
    SCALA_PACKAGE = "com.intel.analytics.bigdl.nn.quantized"
    _out_qscale = None
    _out_u8 = False

    def __init__(self, branch=None, shortcut=None, name=None):
        super().__init__()
        self.modules = [branch, shortcut]
        if name:
            self.set_name(name)

    @property
    def branch(self):
        return self.modules[0]

    @property
    def shortcut(self):
        return self.modules[1]

    @property
    def tail(self):
        return [m for m in self.branch.modules if not isinstance(m, L.Identity)][-1]

    def head(self):
        return _first_conv(self.branch)

    def updateOutput(self, input):
        import torch
        res = self.shortcut.forward(input)
        h = input
        tail = self.tail
        for m in self.branch.modules:
            if m is tail:
                break
            h = m.forward(h)
        y = tail.forward_residual(h, res, self._out_qscale, self._out_u8)
        if y is NotImplemented:  # dynamic-scale tail: sum + ReLU on the dequantised tensors
            yt = tail.forward(h)
            yt = Q.dequant(yt) if yt.dtype == torch.int8 else yt
            r = Q.dequant(res) if res.dtype == torch.int8 else res
            y = torch.relu(yt.float() + r.float()).to(yt.dtype)
            if self._out_qscale is not None and y.is_cuda:
                from ...ops import native_ops as NO
                yq = NO.quant_static(y.contiguous(memory_format=torch.channels_last), self._out_qscale,
                                     u8=self._out_u8)
                if yq is not NotImplemented:
                    y = yq
        return y

    def updateGradInput(self, input, gradOutput):
        raise NotImplementedError("Doesn't updateGradInput for quantized model (Int8ResidualBlock)")

    def parameters(self):
        return None

    def __repr__(self):
        return f"quantized.Int8ResidualBlock[{self.get_name()}]"


def _first_conv(seq):
    for m in getattr(seq, "modules", []):
        if isinstance(m, Q.SpatialConvolution):
            return m
        if isinstance(m, L.Identity):
            continue
        return None
    return None


def _fuse_residual_blocks(model):
    """Sequential [ConcatTable(branch, shortcut), CAddTable, ReLU] whose branch ends in a quantised conv
    → :class:`Int8ResidualBlock`."""
    from ..containers import Sequential, ConcatTable
    from ..layers.table_ops import CAddTable
    from ..layers.activation import Threshold
    for s in model.flattened_modules():
        if not isinstance(s, Sequential):
            continue
        mods = s.modules
        if not (len(mods) == 3 and isinstance(mods[0], ConcatTable) and isinstance(mods[1], CAddTable)
                and isinstance(mods[2], Threshold) and mods[2].threshold == 0.0 and mods[2].value == 0.0
                and len(mods[0].modules) == 2):
            continue
        branch, short = mods[0].modules
        if not isinstance(branch, Sequential):
            continue
        eff = [m for m in branch.modules if not isinstance(m, L.Identity)]
        if not eff or not isinstance(eff[-1], Q.SpatialConvolution) or eff[-1].nGroup != 1:
            continue
        s.modules = [Int8ResidualBlock(branch, short, name=s.get_name() + "_int8")]
    return model


def _exec_units(seq):
    """The modules of a Sequential in execution order, nested Sequentials flattened (a residual block
    and any other container stay one unit)."""
    from ..containers import Sequential
    out = []
    for m in seq.modules:
        if isinstance(m, Sequential):
            out += _exec_units(m)
        else:
            out.append(m)
    return out


def _link_units(units):
    """Producer → consumer links over one execution sequence: a quantised conv (or a residual block)
    followed — through ReLU / max pooling / eval dropout / Identity only — by a quantised conv with a
    static scale or by a residual block whose branch starts with one writes that consumer's int8 input
    (the ReLU fused into its epilogue, the unsigned code after a ReLU)."""
    from ..layers.activation import Threshold
    from ..layers.pooling import SpatialMaxPooling
    from ..layers.dropout import Dropout
    from ...ops import native_ops as NO
    from ...utils import config
    from ..layers.shape import View, Reshape, InferReshape
    u8 = bool(config.get_property("bigdl.int8.unsignedActivations"))
    flat = (View, Reshape, InferReshape)
    for i, a in enumerate(units):
        is_block = isinstance(a, Int8ResidualBlock)
        is_fc = isinstance(a, Q.Linear)
        if not (is_block or is_fc or (isinstance(a, Q.SpatialConvolution) and a.nGroup == 1
                                      and a.nOutputPlane % 16 == 0)):
            continue
        j, relu = i + 1, None
        while j < len(units) and isinstance(units[j], (Threshold, SpatialMaxPooling, Dropout, L.Identity) + flat):
            m = units[j]
            if isinstance(m, Threshold):
                if not (m.threshold == 0.0 and m.value == 0.0):
                    break
                if relu is None and all(isinstance(units[k], L.Identity) for k in range(i + 1, j)):
                    relu = m
            j += 1
        if j >= len(units):
            continue
        b = units[j]
        head = b.head() if isinstance(b, Int8ResidualBlock) else b
        if isinstance(head, Q.Linear):
            # the classifier head: conv / pool → flatten → FC, FC → ReLU → dropout → FC (int8 FC head)
            if head.static_scale is None or (is_fc and any(isinstance(m, SpatialMaxPooling) for m in units[i + 1:j])):
                continue
        elif not isinstance(head, Q.SpatialConvolution) or is_fc or any(isinstance(m, flat) for m in units[i + 1:j]):
            continue
        elif head.static_scale is None or head.nGroup != 1 or not NO.conv_i8_supported(
                a.tail.nOutputPlane if is_block else a.nOutputPlane, head.kernelH, head.kernelW):
            continue
        if any(isinstance(m, Threshold) and not (m.threshold == 0.0 and m.value == 0.0) for m in units[i + 1:j]):
            continue
        if isinstance(b, Int8ResidualBlock):
            sc = b.shortcut
            # the shortcut reads the same tensor: an identity or a quantised conv (any scale tag)
            if not (isinstance(sc, L.Identity) or isinstance(_first_conv(sc) if hasattr(sc, "modules") else sc,
                                                              Q.SpatialConvolution)):
                continue
        a._out_qscale = head.static_scale
        if is_block:
            if u8:  # the block output is ReLU(…) ≥ 0
                a._out_u8 = True
                a._out_qscale = head.static_scale * 127.0 / 255.0
            continue
        if relu is not None:
            a._relu_fused = True
            relu._i8_fused = True
            if u8:
                a._out_u8 = True
                a._out_qscale = head.static_scale * 127.0 / 255.0


def _link_all(model):
    from ..containers import Sequential
    seqs = [s for s in model.flattened_modules() if isinstance(s, Sequential)]
    if isinstance(model, Sequential):
        _link_units(_exec_units(model))
    for s in seqs:
        _link_units(list(s.modules))
    for blk in [m for m in model.flattened_modules() if isinstance(m, Int8ResidualBlock)]:
        _link_units(_exec_units(blk.branch))
        if hasattr(blk.shortcut, "modules"):
            _link_units(_exec_units(blk.shortcut))
            # a projection shortcut (conv + folded BN) with a calibrated output range writes the tail's
            # residual as int8 (signed, clip = the calibrated max) instead of bf16: half the bytes the
            # conv + sum epilogue reads
            eff = [m for m in _exec_units(blk.shortcut) if not isinstance(m, L.Identity)]
            if (len(eff) == 1 and isinstance(eff[0], Q.SpatialConvolution) and eff[0]._out_qscale is None
                    and getattr(eff[0], "static_out_scale", None) and eff[0].nOutputPlane % 16 == 0
                    and isinstance(blk.tail, Q.SpatialConvolution) and blk.tail.static_scale is not None):
                eff[0]._out_qscale = eff[0].static_out_scale
                eff[0]._out_u8 = False


def _graph_pass(e):
    """Single-tensor layers an int8 activation of a quantised chain passes through unchanged in
    scale (ReLU(0, 0), max pooling, evaluation dropout, Identity)."""
    from ..layers.activation import Threshold
    from ..layers.pooling import SpatialMaxPooling
    from ..layers.dropout import Dropout
    if isinstance(e, Threshold):
        return e.threshold == 0.0 and e.value == 0.0
    return isinstance(e, (SpatialMaxPooling, Dropout, L.Identity))


def _graph_consumers(node):
    """The quantised convs that read ``node``'s output through pass-through layers only (fan-out
    allowed): list of conv elements, or None when any path reaches something else."""
    out, todo, seen = [], list(node.next_nodes), set()
    while todo:
        n = todo.pop()
        if n._id in seen:
            continue
        seen.add(n._id)
        e = n.element
        if len(n.prev_nodes) != 1:
            return None
        if isinstance(e, Q.SpatialConvolution):
            out.append(e)
        elif _graph_pass(e) and n.next_nodes:
            todo.extend(n.next_nodes)
        else:
            return None
    return out or None


def _graph_producer(p):
    """(quantised conv, its ReLU or None) whose output reaches node ``p``'s output through at most one
    ReLU (a single-consumer chain), else None."""
    from ..layers.activation import Threshold
    relu = None
    if isinstance(p.element, Threshold) and _graph_pass(p.element) and len(p.prev_nodes) == 1:
        relu = p.element
        if len(p.prev_nodes[0].next_nodes) != 1:
            return None
        p = p.prev_nodes[0]
    e = p.element
    if isinstance(e, Q.SpatialConvolution) and e.nGroup == 1 and e.nOutputPlane % 16 == 0:
        return e, relu
    return None


def _link_graph(g):
    """int8 chains of a Graph model (node topology instead of Sequential order):

    * a calibrated int8 conv (optionally through its ReLU) whose consumers — through ReLU / max pooling
      / eval dropout / Identity, fan-out allowed — are all calibrated int8 convs writes their int8
      input directly, at ONE scale (the largest of the consumers' calibrated input scales; they read
      the same tensor, so they agree);
    * a channel JoinTable whose every input is such a producer and whose consumers are all int8 convs:
      every producer writes at the common scale and the concat runs on the int8 codes — the
      reference's input-scale unification ahead of a JoinTable (``setScalesPrevousJoinTable``,
      DL/nn/mkldnn/Fusion.scala:240-290)."""
    from ..layers.table_ops import JoinTable
    from ...ops import native_ops as NO
    from ...utils import config
    u8ok = bool(config.get_property("bigdl.int8.unsignedActivations"))

    def link(producers, consumers, in_channels):
        scales = [c.static_scale for c in consumers]
        if any(s is None for s in scales) or any(c.nGroup != 1 or not NO.conv_i8_supported(
                in_channels, c.kernelH, c.kernelW) for c in consumers):
            return False
        sc = max(scales)
        all_relu = all(r is not None for _c, r in producers)
        for conv, relu in producers:
            conv._out_qscale = sc
            if relu is not None:
                conv._relu_fused = True
                relu._i8_fused = True
            if u8ok and all_relu:  # every input of the tensor is ReLU'd: the unsigned code
                conv._out_u8 = True
                conv._out_qscale = sc * 127.0 / 255.0
        return True

    for n in g.forward_order:
        e = n.element
        if isinstance(e, JoinTable):
            if e.dimension != 2 or len(n.prev_nodes) < 2:
                continue
            prods = [_graph_producer(p) for p in n.prev_nodes]
            if any(x is None for x in prods) or len({id(c) for c, _r in prods}) != len(prods):
                continue
            if any(len(p.next_nodes) != 1 for p in n.prev_nodes):
                continue
            cons = _graph_consumers(n)
            if cons and link(prods, cons, sum(c.nOutputPlane for c, _r in prods)):
                e._i8_join = True
                # zero-copy concat: each producer writes its channel slice of the join's output
                ctot, off = sum(c.nOutputPlane for c, _r in prods), 0
                for c, _r in prods:
                    c._cat_join = (e, off, ctot)
                    off += c.nOutputPlane
            continue
        if not (isinstance(e, Q.SpatialConvolution) and e.nGroup == 1 and e.nOutputPlane % 16 == 0
                and len(n.next_nodes) == 1):
            continue
        nxt = n.next_nodes[0]
        from ..layers.activation import Threshold
        relu = nxt.element if (isinstance(nxt.element, Threshold) and _graph_pass(nxt.element)) else None
        src = nxt if relu is not None else n
        if relu is not None and len(nxt.prev_nodes) != 1:
            continue
        if any(isinstance(m.element, JoinTable) for m in src.next_nodes):
            continue  # (the join's pass decides)
        cons = _graph_consumers(src)
        if cons:
            link([(e, relu)], cons, e.nOutputPlane)
    # a conv whose only consumer is a ReLU but whose output does not chain on in int8 (an LRN, a
    # float layer follows): the ReLU still runs in the conv's epilogue, the ReLU node passes through
    from ..layers.activation import Threshold
    for n in g.forward_order:
        e = n.element
        if not (isinstance(e, Q.SpatialConvolution) and len(n.next_nodes) == 1) or e._relu_fused:
            continue
        nxt = n.next_nodes[0]
        if (isinstance(nxt.element, Threshold) and _graph_pass(nxt.element) and len(nxt.prev_nodes) == 1
                and not getattr(nxt.element, "_i8_fused", False)):
            e._relu_fused = True
            nxt.element._passthrough = True


def quantize(model):
    """Deep-copy ``model`` and return its int8 version (evaluation mode).  Evaluation BatchNorms after a
    convolution are folded into it first; layers calibrated with ``calcScales`` quantise their input
    statically and chain int8 activations between quantised convs (:func:`_link_int8_chains`), through
    residual blocks (conv + sum epilogues, :class:`Int8ResidualBlock`); uncalibrated ones use per-image
    dynamic scales."""
    from ..fusion import unfuse
    from ...utils import config
    clone = model.cloneModule()
    unfuse(clone)
    clone.evaluate()
    if config.get_property("bigdl.int8.foldBN"):
        _fold_bn(clone)
    q = _convert(clone)
    if config.get_property("bigdl.int8.residual"):
        _fuse_residual_blocks(q)
        _link_all(q)
    else:
        _link_int8_chains(q)
    from ..graph import Graph
    for g in [m for m in ([q] + list(q.flattened_modules())) if isinstance(m, Graph)]:
        _link_graph(g)
    q.evaluate()
    return q
