"""Intermediate representation for device graph planning: ``IROperator``s, ``IRElement``,
``IRGraph``, the module→IR (``BlasToIR``) and IR→device-graph (``IRConverter``) conversions and
``ConversionUtils.convert``.

Reference: ``DL/utils/intermediate/IRElement.scala:27-182`` (operator case classes),
``IRGraph.scala:41-220`` (build → converted graph, forward/backward delegation),
``BlasToIR.scala`` / ``IRToBlas.scala`` / ``IRToDnn.scala`` / ``IRConverter.scala:37-130`` and
``ConversionUtils.scala:31-95`` (``convert(model[, needQuantize])``).

The reference lowers the IR to MKL-DNN primitives with layout reorders.  Here there is one
backend: the IR is lowered to a device :class:`~bigdl.nn.Graph` of our modules (whose hot layers
are the HIP kernels, NHWC bf16 on the GPU) after the inference-time rewrites the primitives layer
would otherwise do:

* conv → BatchNorm (eval): the BN is folded into the conv weights/bias (``W·γ/σ``,
  ``(b−μ)·γ/σ + β``) and disappears — K6 of the kernel inventory;
* Linear → BatchNormalization (eval): same fold for fully-connected layers;
* conv → ReLU: ReLU in the conv epilogue; Inception-style concats of conv branches become
  zero-copy writes into the concat output (``bigdl.nn.fusion``);
* Dropout (eval) → identity.

Training graphs are lowered without folding (the BN statistics are live), reusing the original
modules and therefore the same parameters.  An inference graph is re-folded from the current
weights every time the IRGraph switches to evaluate mode.
"""
from __future__ import annotations

import copy
from typing import Dict, List, Optional, Sequence

import torch

from ..nn.abstractnn import AbstractModule


# ---------------------------------------------------------------------------------- operators
class IROperator:
    """One operation of the IR; ``module`` is the source layer (weights, hyper-parameters)."""

    def __init__(self, module: Optional[AbstractModule] = None, **attrs):
        self.module = module
        self.attrs = attrs

    @property
    def name(self) -> str:
        return type(self).__name__

    def __repr__(self):
        return f"{self.name}({', '.join(f'{k}={v}' for k, v in self.attrs.items())})"


def _op(name):
    return type(name, (IROperator,), {})


IRSpatialConvolution = _op("IRSpatialConvolution")
IRSpatialShareConvolution = _op("IRSpatialShareConvolution")
IRSpatialBatchNormalization = _op("IRSpatialBatchNormalization")
IRSpatialMaxPooling = _op("IRSpatialMaxPooling")
IRSpatialAveragePooling = _op("IRSpatialAveragePooling")
IRSpatialCrossMapLRN = _op("IRSpatialCrossMapLRN")
IRLinear = _op("IRLinear")
IRReLU = _op("IRReLU")
IRSoftMax = _op("IRSoftMax")
IRDropout = _op("IRDropout")
IRIdentity = _op("IRIdentity")
IRInput = _op("IRInput")
IRSqueeze = _op("IRSqueeze")
IRCAddTable = _op("IRCAddTable")
IRJoinTable = _op("IRJoinTable")
IRConcatTable = _op("IRConcatTable")
IRSelectTable = _op("IRSelectTable")
IRGeneralModule = _op("IRGeneralModule")


class IRElement:
    """A named IR operator with its (weights, gradWeights) (``IRElement.scala:142-182``)."""

    def __init__(self, name: str, op: IROperator, weights=None, grad_weights=None):
        self.name, self.op = name, op
        self.weights, self.gradWeights = weights, grad_weights

    def getName(self):
        return self.name

    def getOp(self):
        return self.op

    def getParameters(self):
        return self.weights, self.gradWeights

    def setWeights(self, w):
        self.weights = w

    def setGradWeights(self, g):
        self.gradWeights = g

    def __repr__(self):
        return f"IRElement({self.name}: {self.op})"


class IRNode:
    def __init__(self, element: IRElement):
        self.element = element
        self.prev_nodes: List["IRNode"] = []
        self.prev_index: List[int] = []
        self.next_nodes: List["IRNode"] = []


# ---------------------------------------------------------------------------------- module → IR
def _classify(m) -> IROperator:
    from ..nn import (SpatialConvolution, SpatialShareConvolution, SpatialBatchNormalization, SpatialMaxPooling,
                      SpatialAveragePooling, SpatialCrossMapLRN, Linear, ReLU, SoftMax, Dropout, Identity, Squeeze,
                      CAddTable, JoinTable, ConcatTable, SelectTable, BatchNormalization)
    from ..nn.graph import _InputLayer
    table = [
        (_InputLayer, IRInput), (SpatialShareConvolution, IRSpatialShareConvolution),
        (SpatialConvolution, IRSpatialConvolution), (SpatialBatchNormalization, IRSpatialBatchNormalization),
        (BatchNormalization, IRSpatialBatchNormalization), (SpatialMaxPooling, IRSpatialMaxPooling),
        (SpatialAveragePooling, IRSpatialAveragePooling), (SpatialCrossMapLRN, IRSpatialCrossMapLRN),
        (Linear, IRLinear), (ReLU, IRReLU), (SoftMax, IRSoftMax), (Dropout, IRDropout), (Squeeze, IRSqueeze),
        (CAddTable, IRCAddTable), (JoinTable, IRJoinTable), (ConcatTable, IRConcatTable),
        (SelectTable, IRSelectTable), (Identity, IRIdentity),
    ]
    for cls, op in table:
        if type(m) is cls:
            return op(m)
    for cls, op in table:  # subclasses (e.g. SpatialDilatedConvolution) keep their own module
        if isinstance(m, cls) and op not in (IRSpatialConvolution, IRLinear):
            return op(m)
    return IRGeneralModule(m)


class _Flattener:
    """Expand Sequential / ConcatTable / Concat containers into IR nodes so the lowering sees the
    conv → BN → ReLU chains inside residual and Inception blocks.  A list of several nodes stands
    for a Table activity (the next node takes them as its inputs, in order)."""

    def __init__(self):
        self.order: List[IRNode] = []

    def node(self, m, prevs):
        n = IRNode(IRElement(m.get_name(), _classify(m), *(m.parameters() if m.parameters() else (None, None))))
        for p in prevs:
            p, i = p if isinstance(p, tuple) else (p, 0)
            n.prev_nodes.append(p)
            n.prev_index.append(i)
            p.next_nodes.append(n)
        self.order.append(n)
        return n

    def expand(self, m, ins):
        from ..nn import Sequential, ConcatTable, Concat, JoinTable
        if type(m) is Sequential and m.modules:
            cur = ins
            for sub in m.modules:
                cur = self.expand(sub, cur)
            return cur
        if type(m) is ConcatTable and len(m.modules) > 1 and len(ins) == 1:
            outs = [self.expand(b, ins) for b in m.modules]
            if all(len(o) == 1 for o in outs):
                return [o[0] for o in outs]
            self.order = [n for n in self.order if n not in sum(outs, [])]  # pragma: no cover
        if type(m) is Concat and len(m.modules) > 1 and len(ins) == 1:
            outs = [self.expand(b, ins) for b in m.modules]
            if all(len(o) == 1 for o in outs):
                j = JoinTable(m.dimension, 0)
                j.set_name(m.get_name() + "/join")
                return [self.node(j, [o[0] for o in outs])]
        return [self.node(m, ins)]


def to_ir(model, input_formats=("nchw",), output_formats=("nc",)) -> "IRGraph":
    """``BlasToIR``: a module (Graph, Sequential, …) → IRGraph, containers expanded."""
    from ..nn.graph import Graph, _InputLayer
    from ..nn.fusion import unfuse
    unfuse(model)  # training-fusion flags describe container-level execution the IR flattens away
    f = _Flattener()
    if isinstance(model, Graph):
        made: Dict[int, list] = {}
        for n in model.forward_order:
            if not n.prev_nodes:
                made[n._id] = [f.node(n.element, [])]
                continue
            prevs = []
            for p, i in zip(n.prev_nodes, n.prev_index):
                src = made[p._id]
                prevs.append(src[i - 1] if (i and len(src) > 1) else ((src[0], i) if i else src[0]))
                if not i and len(src) > 1:
                    prevs[-1:] = src
            made[n._id] = f.expand(n.element, prevs)
        ins = [made[n._id][0] for n in model.inputs]
        outs = [made[n._id][0] for n in model.outputs_nodes]
    else:
        inp = _InputLayer()
        i0 = f.node(inp, [])
        outs = f.expand(model, [i0])
        ins = [i0]
    nin, nout = len(ins), len(outs)
    fi = list(input_formats) if len(input_formats) == nin else [input_formats[0]] * nin
    fo = list(output_formats) if len(output_formats) == nout else [output_formats[0]] * nout
    return IRGraph(ins, outs, None, True, fi, fo, _order=f.order)


# ---------------------------------------------------------------------------------- BN folding
def _bn_affine(bn):
    """Per-channel (scale, shift) of an eval-mode BN: y = x·scale + shift."""
    inv = torch.rsqrt(bn.runningVar.float() + bn.eps)
    g = bn.weight.float() if bn.affine and bn.weight is not None else torch.ones_like(inv)
    b = bn.bias.float() if bn.affine and bn.bias is not None else torch.zeros_like(inv)
    scale = g * inv
    return scale, b - bn.runningMean.float() * scale


def fold_conv_bn(conv, bn):
    """A new conv computing BN(conv(x)) in eval mode (weights (g, o/g, i/g, kh, kw))."""
    scale, shift = _bn_affine(bn)
    new = copy.deepcopy(conv)
    new._arena = None
    new._shadow_views, new._shadow_cache = {}, {}
    w = conv.weight.detach().float()
    g, og = w.shape[0], w.shape[1]
    s = scale.to(w.device).view(g, og, 1, 1, 1)
    b0 = conv.bias.detach().float() if conv.withBias and conv.bias is not None else torch.zeros(
        conv.nOutputPlane, device=w.device)
    new_b = b0 * scale.to(w.device) + shift.to(w.device)
    if not new.withBias:
        new.withBias = True
        new.register_parameter("bias", new_b.clone())
    new.weight.copy_(w * s)
    new.bias.copy_(new_b)
    new._bias_folded_into = None
    new.set_name(conv.get_name())
    return new


def fold_linear_bn(lin, bn):
    scale, shift = _bn_affine(bn)
    new = copy.deepcopy(lin)
    new._arena = None
    new._shadow_views, new._shadow_cache = {}, {}
    w = lin.weight.detach().float()
    b0 = lin.bias.detach().float() if lin.withBias and lin.bias is not None else torch.zeros(w.shape[0], device=w.device)
    if not new.withBias:
        new.withBias = True
        new.register_parameter("bias", torch.zeros(w.shape[0], device=w.device))
    new.weight.copy_(w * scale.to(w.device)[:, None])
    new.bias.copy_(b0 * scale.to(w.device) + shift.to(w.device))
    new.set_name(lin.get_name())
    return new


def _private_copy(m):
    """A copy of ``m`` for the inference graph that shares its tensors but not its fusion flags
    (leaf layers: shallow copy; containers: deep copy, their children get flagged too)."""
    if m.children():
        c = copy.deepcopy(m)
    else:
        c = copy.copy(m)
        c.__dict__ = dict(m.__dict__)
    for x in c.flattened_modules():
        x._arena = None
        if hasattr(x, "_shadow_views"):
            x._shadow_views, x._shadow_cache = {}, {}
    return c


# ---------------------------------------------------------------------------------- IR → device graph
class IRConverter:
    """Lower an IRGraph to an executable Graph (``IRConverter.toGraph``)."""

    def __init__(self, ir: "IRGraph"):
        self.ir = ir

    def to_graph(self, training: bool):
        from ..nn.graph import Graph, ModuleNode
        from ..nn import Identity
        order = self.ir.order
        alias: Dict[int, int] = {}        # IR node id → id of the IR node whose module produces its value
        replaced: Dict[int, AbstractModule] = {}
        fused_sum: Dict[int, tuple] = {}  # CAddTable node id → (conv node, shortcut node, relu node|None)
        absorbed = set()                  # nodes whose work moved into another node
        if not training:
            for n in order:
                op = n.element.op
                nxt = n.next_nodes
                if isinstance(op, (IRSpatialConvolution, IRSpatialShareConvolution, IRLinear)) and len(nxt) == 1 \
                        and isinstance(nxt[0].element.op, IRSpatialBatchNormalization) \
                        and len(nxt[0].prev_nodes) == 1:
                    bn = nxt[0].element.op.module
                    src = replaced.get(id(n), op.module)
                    if isinstance(op, IRLinear):
                        if bn.runningMean.dim() != 1 or getattr(bn, "dataFormat", "NCHW") != "NCHW":
                            continue
                        replaced[id(n)] = fold_linear_bn(src, bn)
                    elif getattr(src, "format", "NCHW") == "NCHW" and getattr(bn, "dataFormat", "NCHW") == "NCHW":
                        replaced[id(n)] = fold_conv_bn(src, bn)
                    else:
                        continue
                    alias[id(nxt[0])] = id(n)
                    absorbed.add(id(nxt[0]))
            by_id = {id(n): n for n in order}

            def value_src(n):
                while id(n) in alias:
                    n = by_id[alias[id(n)]]
                return n

            def sole_consumer(n):
                """The single consumer of n's value (through a folded BN), else None."""
                cur = n
                nxt = cur.next_nodes
                if len(nxt) == 1 and id(nxt[0]) in alias and alias[id(nxt[0])] == id(n):
                    cur = nxt[0]
                    nxt = cur.next_nodes
                return nxt[0] if len(nxt) == 1 else None

            # residual tail: ReLU(conv(x) [+BN] + shortcut) → one conv with the sum and ReLU in its epilogue
            for n in order:
                if not isinstance(n.element.op, IRCAddTable) or len(n.prev_nodes) != 2 or any(n.prev_index):
                    continue
                for k in (0, 1):
                    c = value_src(n.prev_nodes[k])
                    other = n.prev_nodes[1 - k]
                    cm = replaced.get(id(c), c.element.op.module)
                    if not (isinstance(c.element.op, (IRSpatialConvolution, IRSpatialShareConvolution))
                            and type(cm).__name__ in ("SpatialConvolution", "SpatialShareConvolution")
                            and cm.format == "NCHW" and sole_consumer(c) is n and len(c.prev_nodes) == 1
                            and value_src(other) is not c):
                        continue
                    relu = None
                    if len(n.next_nodes) == 1 and isinstance(n.next_nodes[0].element.op, IRReLU) \
                            and len(n.next_nodes[0].prev_nodes) == 1:
                        relu = n.next_nodes[0]
                    fused_sum[id(n)] = (c, other, relu)
                    absorbed.add(id(c))
                    if relu is not None:
                        alias[id(relu)] = id(n)
                        absorbed.add(id(relu))
                    break
        nodes: Dict[int, ModuleNode] = {}

        def node_of(n):
            while id(n) in alias and id(n) not in nodes:
                n = next(q for q in order if id(q) == alias[id(n)])
            return nodes[id(n)]
        for n in order:
            if id(n) in absorbed:
                continue
            op = n.element.op
            if id(n) in fused_sum:
                c, other, relu = fused_sum[id(n)]
                from ..nn.layers.conv import FusedConvSum
                m = FusedConvSum(replaced.get(id(c), c.element.op.module), relu is not None)
                mn = ModuleNode(m)
                cp, ci = c.prev_nodes[0], c.prev_index[0]
                mn((node_of(cp), ci) if ci else node_of(cp), node_of(other))
                nodes[id(n)] = mn
                continue
            m = replaced.get(id(n), op.module)
            if not training and isinstance(op, IRDropout):
                m = Identity().set_name(m.get_name())
            elif not training and id(n) not in replaced:
                m = _private_copy(m)
            mn = ModuleNode(m)
            for p, i in zip(n.prev_nodes, n.prev_index):
                src = node_of(p)
                mn(*[(src, i) if i else src])
            nodes[id(n)] = mn
        g = Graph([node_of(n) for n in self.ir.inputs], [node_of(n) for n in self.ir.outputs])
        from ..nn.fusion import fuse
        fuse(g)
        return g

    toGraph = to_graph


class IRGraph(AbstractModule):
    """Executable IR graph: ``build()`` lowers it; forward/backward delegate to the lowered graph."""

    SCALA_NAME = "IRGraph"

    def __init__(self, inputs: Sequence[IRNode], outputs: Sequence[IRNode], variables=None,
                 generate_backward: bool = True, input_formats=("nchw",), output_formats=("nc",), _order=None):
        super().__init__()
        if len(input_formats) != len(inputs):
            raise ValueError(f"IRGraph: inputFormats length {len(input_formats)} != inputs {len(inputs)}")
        if len(output_formats) != len(outputs):
            raise ValueError(f"IRGraph: outputFormats length {len(output_formats)} != outputs {len(outputs)}")
        self.inputs, self.outputs = list(inputs), list(outputs)
        self.variables, self.generateBackward = variables, generate_backward
        self.inputFormats, self.outputFormats = list(input_formats), list(output_formats)
        self.order = _order if _order is not None else self._topo()
        self.graph = None
        self._train_graph = None

    def _topo(self):
        seen, order = set(), []

        def visit(n):
            if id(n) in seen:
                return
            seen.add(id(n))
            for p in n.prev_nodes:
                visit(p)
            order.append(n)
        for o in self.outputs:
            visit(o)
        return order

    def isBuild(self) -> bool:
        return self.graph is not None

    def build(self):
        self._train_graph = IRConverter(self).to_graph(training=True)
        self.graph = self._train_graph if self.train else IRConverter(self).to_graph(training=False)
        return self

    def _need(self):
        if self.graph is None:
            raise RuntimeError("IRGraph: build() the graph first")
        return self.graph

    def updateOutput(self, input):
        return self._need().forward(input)

    def updateGradInput(self, input, gradOutput):
        if not self.train:
            raise RuntimeError("IRGraph: backward needs training mode (an inference graph has folded BNs)")
        return self._need().updateGradInput(input, gradOutput)

    def accGradParameters(self, input, gradOutput):
        self._need().accGradParameters(input, gradOutput)

    def backward(self, input, gradOutput):
        if not self.train:
            raise RuntimeError("IRGraph: backward needs training mode (an inference graph has folded BNs)")
        self.gradInput = self._need().backward(input, gradOutput)
        return self.gradInput

    def training(self, is_training: bool = True):
        if not is_training and not self.train and self.graph is not None and self.graph is not self._train_graph:
            return self  # already an inference graph: re-fold only on a training → inference switch
        self.train = is_training
        if self._train_graph is not None:
            self._train_graph.training(is_training)
            if is_training:
                self.graph = self._train_graph
            else:  # re-fold from the current weights
                self.graph = IRConverter(self).to_graph(training=False)
                self.graph.training(False)
        return self

    def parameters(self):
        g = self._train_graph or self._need()
        return g.parameters()

    def getParametersTable(self):
        return (self._train_graph or self._need()).getParametersTable()

    def getExtraParameter(self):
        return (self._train_graph or self._need()).getExtraParameter()

    def children(self):
        return [self._train_graph] if self._train_graph is not None else []

    def to(self, device=None, dtype=None):
        if self._train_graph is not None:
            self._train_graph.to(device, dtype)
            if not self.train:
                self.graph = IRConverter(self).to_graph(training=False)
                self.graph.evaluate()
        return self

    def __repr__(self):
        return f"IRGraph({len(self.order)} ops, built={self.isBuild()})"


class ConversionUtils:
    """``ConversionUtils.convert``: a model → a device-planned IRGraph (or the model itself when it is
    already one); ``need_quantize`` additionally swaps in the int8 layers."""

    @staticmethod
    def convert(model, need_quantize: bool = False):
        if isinstance(model, IRGraph):
            return model if model.isBuild() else model.build()
        if need_quantize:
            model = model.quantize()
        ir = to_ir(model)
        if not model.isTraining():
            ir.evaluate()
        return ir.build()


def _to_ir_graph(self, input_formats=("nchw",), output_formats=("nc",)):
    """``StaticGraph.toIRgraph``: this module as a built IRGraph."""
    ir = to_ir(self, input_formats, output_formats)
    ir.training(self.isTraining())
    return ir.build()


AbstractModule.toIRgraph = _to_ir_graph
