"""ONNX GraphProto → BigDL ``Graph`` (``pyspark/bigdl/contrib/onnx/onnx_loader.py``; op converters
``ops_converter.py`` — the reference maps 14 ops, this maps the common CNN/MLP inference set).

Each ONNX node becomes one module node fed by the modules producing its non-initializer inputs;
initializer inputs are bound into the module (weights, shapes, axes).  Constant subgraphs
(``Constant``, ``Shape`` of a known input, …) are folded while loading.
"""
from __future__ import annotations

from typing import Dict, List

import numpy as np
import torch
import torch.nn.functional as F

from ... import nn
from ...nn.graph import ModuleNode
from ...nn.onnx import Gemm as OnnxGemm, Reshape as OnnxReshape, Shape as OnnxShape
from ...nn.ops import Operation
from ...utils.table import Table
from . import _attrs, onnx_classes, to_array


class _Fn(Operation):
    def __init__(self, fn, op=""):
        super().__init__()
        self.fn, self.op = fn, op

    def updateOutput(self, input):
        args = input.values() if isinstance(input, Table) else [input]
        return self.fn(*args)


def _pads2(a, k):
    """ONNX pads [x1_begin, x2_begin, x1_end, x2_end] → symmetric (padH, padW) or None."""
    p = a.get("pads", [0] * (2 * k))
    begin, end = p[:k], p[k:]
    return (begin[0], begin[1]) if begin == end else None


def _conv(a, ins, consts):
    w = consts[1]
    b = consts[2] if len(ins) > 2 else None
    K, Cg, kh, kw = w.shape
    g = int(a.get("group", 1))
    s = a.get("strides", [1, 1])
    d = a.get("dilations", [1, 1])
    auto = a.get("auto_pad", "NOTSET")
    if auto in ("SAME_UPPER", "SAME_LOWER"):
        ph = pw = -1
    else:
        pp = _pads2(a, 2)
        if pp is None:
            raise NotImplementedError("asymmetric Conv pads")
        ph, pw = pp
    if d != [1, 1]:
        m = nn.SpatialDilatedConvolution(Cg * g, K, kw, kh, s[1], s[0], pw, ph, d[1], d[0])
    else:
        m = nn.SpatialConvolution(Cg * g, K, kw, kh, s[1], s[0], pw, ph, n_group=g, with_bias=b is not None)
    m.weight.data.copy_(torch.from_numpy(np.ascontiguousarray(w)).float().reshape(m.weight.shape))
    if b is not None:
        m.bias.data.copy_(torch.from_numpy(b).float())
    elif getattr(m, "bias", None) is not None:
        m.bias.data.zero_()
    return m, [0]


def _conv_t(a, ins, consts):
    w = consts[1]
    b = consts[2] if len(ins) > 2 else None
    Cin, Kg, kh, kw = w.shape
    s = a.get("strides", [1, 1])
    pp = _pads2(a, 2) or (0, 0)
    op = a.get("output_padding", [0, 0])
    m = nn.SpatialFullConvolution(Cin, Kg, kw, kh, s[1], s[0], pp[1], pp[0], op[1], op[0], no_bias=b is None)
    m.weight.data.copy_(torch.from_numpy(np.ascontiguousarray(w)).float().reshape(m.weight.shape))
    if b is not None:
        m.bias.data.copy_(torch.from_numpy(b).float())
    return m, [0]


def _bn(a, ins, consts):
    scale, bias, mean, var = (consts[i] for i in (1, 2, 3, 4))
    m = nn.SpatialBatchNormalization(scale.shape[0], eps=float(a.get("epsilon", 1e-5)),
                                     momentum=1 - float(a.get("momentum", 0.9)))
    m.weight.data.copy_(torch.from_numpy(scale).float())
    m.bias.data.copy_(torch.from_numpy(bias).float())
    m.runningMean.copy_(torch.from_numpy(mean).float())
    m.runningVar.copy_(torch.from_numpy(var).float())
    return m, [0]


def _gemm(a, ins, consts):
    alpha, beta = float(a.get("alpha", 1.0)), float(a.get("beta", 1.0))
    ta, tb = int(a.get("transA", 0)), int(a.get("transB", 0))
    B = consts.get(1)
    C = consts.get(2)
    if B is not None and not ta and (C is None or C.ndim <= 1):
        Wm = B.T if not tb else B  # Linear weight is [out, in]
        lin = nn.Linear(Wm.shape[1], Wm.shape[0], with_bias=C is not None)
        lin.weight.data.copy_(torch.from_numpy(np.ascontiguousarray(Wm)).float() * alpha)
        if C is not None:
            lin.bias.data.copy_(torch.from_numpy(np.broadcast_to(C, (Wm.shape[0],)).copy()).float() * beta)
        return lin, [0]
    return OnnxGemm(alpha, beta, ta, tb, B, C), [i for i in range(len(ins)) if i not in consts]


def _pool(kind):
    def conv(a, ins, consts):
        k = a["kernel_shape"]
        s = a.get("strides", [1, 1])
        pp = _pads2(a, 2)
        if pp is None:
            raise NotImplementedError("asymmetric pool pads")
        ceil = bool(a.get("ceil_mode", 0))
        if kind == "max":
            m = nn.SpatialMaxPooling(k[1], k[0], s[1], s[0], pp[1], pp[0], to_ceil=ceil)
        else:
            m = nn.SpatialAveragePooling(k[1], k[0], s[1], s[0], pp[1], pp[0], ceil_mode=ceil,
                                         count_include_pad=bool(a.get("count_include_pad", 0)))
        return m, [0]
    return conv


def _unary(fn):
    return lambda a, ins, consts: (_Fn(fn), [0])


def _binary(fn):
    def conv(a, ins, consts):
        if 1 in consts:
            c = torch.from_numpy(np.ascontiguousarray(consts[1]))
            return _Fn(lambda x: fn(x, c.to(x.device, x.dtype if c.is_floating_point() else c.dtype))), [0]
        if 0 in consts:
            c = torch.from_numpy(np.ascontiguousarray(consts[0]))
            return _Fn(lambda x: fn(c.to(x.device, x.dtype if c.is_floating_point() else c.dtype), x)), [1]
        return _Fn(fn), [0, 1]
    return conv


def _reshape(a, ins, consts):
    shape = consts.get(1)
    if shape is None:
        shape = a.get("shape")
    return OnnxReshape([int(v) for v in np.asarray(shape).flatten()]), [0]


def _flatten(a, ins, consts):
    ax = int(a.get("axis", 1))
    return _Fn(lambda x: x.reshape(int(np.prod(x.shape[:ax])) if ax else 1, -1)), [0]


def _axes(a, consts):
    ax = a.get("axes")
    if ax is None and 1 in consts:
        ax = [int(v) for v in consts[1].flatten()]
    return ax


def _unsqueeze(a, ins, consts):
    ax = _axes(a, consts)

    def f(x):
        for d in sorted(ax):
            x = x.unsqueeze(d)
        return x
    return _Fn(f), [0]


def _squeeze(a, ins, consts):
    ax = _axes(a, consts)

    def f(x):
        if ax is None:
            return x.squeeze()
        for d in sorted([d % x.dim() for d in ax], reverse=True):
            x = x.squeeze(d)
        return x
    return _Fn(f), [0]


def _concat(a, ins, consts):
    ax = int(a.get("axis", 1))
    live = [i for i in range(len(ins)) if i not in consts]
    cvals = {i: torch.from_numpy(consts[i]) for i in consts}

    def f(*xs):
        it = iter(xs)
        parts = [cvals[i].to(xs[0].device, xs[0].dtype) if i in cvals else next(it) for i in range(len(ins))]
        return torch.cat(parts, ax)
    return _Fn(f), live


def _softmax(log):
    def conv(a, ins, consts):
        ax = int(a.get("axis", 1))

        def f(x):
            shp = x.shape
            y = x.reshape(int(np.prod(shp[:ax])) if ax else 1, -1)
            y = torch.log_softmax(y.float(), -1) if log else torch.softmax(y.float(), -1)
            return y.reshape(shp).to(x.dtype)
        return _Fn(f), [0]
    return conv


def _reduce(fn):
    def conv(a, ins, consts):
        ax = _axes(a, consts)
        keep = bool(a.get("keepdims", 1))

        def f(x):
            axes = list(range(x.dim())) if ax is None else [d % x.dim() for d in ax]
            return fn(x, axes, keep)
        return _Fn(f), [0]
    return conv


def _pad(a, ins, consts):
    pads = a.get("pads") if "pads" in a else [int(v) for v in consts[1].flatten()]
    value = float(a.get("value", 0.0)) if 2 not in consts else float(consts[2])
    mode = a.get("mode", "constant")
    k = len(pads) // 2
    flat = []
    for d in range(k - 1, -1, -1):
        flat += [pads[d], pads[d + k]]

    def f(x):
        if mode == "constant":
            return F.pad(x, flat, value=value)
        return F.pad(x, flat[:2 * (x.dim() - 2)], mode={"reflect": "reflect", "edge": "replicate"}[mode])
    return _Fn(f), [0]


def _clip(a, ins, consts):
    lo = a.get("min", float(consts[1]) if 1 in consts else -float("inf"))
    hi = a.get("max", float(consts[2]) if 2 in consts else float("inf"))
    return _Fn(lambda x: x.clamp(lo, hi)), [0]


def _gather(a, ins, consts):
    ax = int(a.get("axis", 0))
    if 1 in consts:
        idx = torch.from_numpy(consts[1].astype(np.int64))
        return _Fn(lambda x: torch.index_select(x, ax, idx.flatten().to(x.device)).reshape(
            tuple(x.shape[:ax]) + tuple(idx.shape) + tuple(x.shape[ax + 1:]))), [0]
    return _Fn(lambda x, i: torch.index_select(x, ax, i.long().flatten()).reshape(
        tuple(x.shape[:ax]) + tuple(i.shape) + tuple(x.shape[ax + 1:]))), [0, 1]


_CONVERT = {
    "Conv": _conv, "ConvTranspose": _conv_t, "BatchNormalization": _bn, "Gemm": _gemm,
    "MatMul": lambda a, ins, consts: _gemm({}, ins, consts) if 1 in consts and consts[1].ndim == 2 else
    _binary(torch.matmul)(a, ins, consts),
    "MaxPool": _pool("max"), "AveragePool": _pool("avg"),
    "GlobalAveragePool": lambda a, ins, consts: (_Fn(lambda x: x.mean((2, 3), keepdim=True)), [0]),
    "GlobalMaxPool": lambda a, ins, consts: (_Fn(lambda x: x.amax((2, 3), keepdim=True)), [0]),
    "Relu": lambda a, ins, consts: (nn.ReLU(), [0]),
    "LeakyRelu": lambda a, ins, consts: (nn.LeakyReLU(float(a.get("alpha", 0.01))), [0]),
    "Elu": lambda a, ins, consts: (nn.ELU(float(a.get("alpha", 1.0))), [0]),
    "Sigmoid": lambda a, ins, consts: (nn.Sigmoid(), [0]), "Tanh": lambda a, ins, consts: (nn.Tanh(), [0]),
    "Softplus": lambda a, ins, consts: (nn.SoftPlus(), [0]),
    "Softmax": _softmax(False), "LogSoftmax": _softmax(True),
    "Dropout": lambda a, ins, consts: (nn.Identity(), [0]), "Identity": lambda a, ins, consts: (nn.Identity(), [0]),
    "Add": _binary(torch.add), "Sub": _binary(torch.sub), "Mul": _binary(torch.mul), "Div": _binary(torch.div),
    "Pow": _binary(torch.pow), "Max": _binary(torch.maximum), "Min": _binary(torch.minimum),
    "Sum": lambda a, ins, consts: (nn.CAddTable(), list(range(len(ins)))),
    "Exp": _unary(torch.exp), "Log": _unary(torch.log), "Sqrt": _unary(torch.sqrt), "Abs": _unary(torch.abs),
    "Neg": _unary(torch.neg), "Ceil": _unary(torch.ceil), "Floor": _unary(torch.floor),
    "Reciprocal": _unary(torch.reciprocal), "Erf": _unary(torch.erf),
    "Clip": _clip, "Reshape": _reshape, "Flatten": _flatten, "Unsqueeze": _unsqueeze, "Squeeze": _squeeze,
    "Concat": _concat,
    "Transpose": lambda a, ins, consts: (_Fn(lambda x: x.permute(*(a.get("perm") or
                                                                   list(range(x.dim()))[::-1])).contiguous()), [0]),
    "Shape": lambda a, ins, consts: (OnnxShape(), [0]), "Gather": _gather,
    "ReduceMean": _reduce(lambda x, ax, k: x.float().mean(ax, keepdim=k).to(x.dtype)),
    "ReduceSum": _reduce(lambda x, ax, k: x.sum(ax, keepdim=k)),
    "ReduceMax": _reduce(lambda x, ax, k: x.amax(ax, keepdim=k)),
    "Pad": _pad,
    "LRN": lambda a, ins, consts: (nn.SpatialCrossMapLRN(int(a["size"]), float(a.get("alpha", 1e-4)),
                                                         float(a.get("beta", 0.75)), float(a.get("bias", 1.0))), [0]),
    "Cast": lambda a, ins, consts: (_Fn(lambda x: x.to({1: torch.float32, 6: torch.int32, 7: torch.int64,
                                                        9: torch.bool, 11: torch.float64}[int(a["to"])])), [0]),
}


class OnnxLoader:
    def load_model(self, file_path):
        m = onnx_classes()["onnx.ModelProto"]()
        with open(file_path, "rb") as f:
            m.ParseFromString(f.read())
        return self.load_graph(m.graph)

    def load_graph(self, graph):
        consts: Dict[str, np.ndarray] = {}
        for t in graph.initializer:
            if not t.name.strip():
                raise ValueError("Tensor's name is required")
            consts[t.name] = to_array(t)
        producers: Dict[str, object] = {}
        inputs = []
        for gi in graph.input:
            if gi.name in consts:
                continue
            node = nn.Input(gi.name)
            producers[gi.name] = node
            inputs.append(node)
        for node in graph.node:
            a = _attrs(node)
            if node.op_type == "Constant":
                consts[node.output[0]] = np.asarray(a["value"])
                continue
            ins = list(node.input)
            cvals = {i: consts[n] for i, n in enumerate(ins) if n and n in consts}
            conv = _CONVERT.get(node.op_type)
            if conv is None:
                raise NotImplementedError(f"ONNX op {node.op_type} is not supported")
            module, feed = conv(a, ins, cvals)
            module.set_name(node.name or node.output[0])
            prevs = [producers[ins[i]] for i in feed if ins[i]]
            mn = ModuleNode.create(module, prevs)
            for o in node.output[:1]:
                producers[o] = mn
        outs = [producers[o.name] for o in graph.output]
        return nn.Graph(inputs, outs)


def load(model_path):
    return OnnxLoader().load_model(model_path)


def load_model_proto(model_proto):
    return OnnxLoader().load_graph(model_proto.graph)
