"""BigDL model → TensorFlow GraphDef (``DL/utils/tf/TensorflowSaver.scala``,
``BigDLToTensorflow.scala``).

Each supported layer becomes a small TF subgraph with its weights as ``Const`` nodes: ``Linear`` →
``MatMul`` + ``BiasAdd``; ``SpatialConvolution`` → ``Conv2D`` (+ ``BiasAdd``) in the layer's own data
format; pooling → ``MaxPool``/``AvgPool``; batch norm (inference) → ``FusedBatchNorm``; activations,
``Reshape``/``View``, ``Dropout`` (identity at inference), ``CAddTable`` → ``AddN``,
``JoinTable`` → ``ConcatV2``.  ``Sequential`` and ``Graph`` containers are walked recursively.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch

from ...nn import Graph, Sequential
from ...nn.layers import activation as A
from ...nn.layers import conv as C
from ...nn.layers import dropout as D
from ...nn.layers import linear as L
from ...nn.layers import normalization as N
from ...nn.layers import pooling as P
from ...nn.layers import shape as S
from ...nn.layers import table_ops as TO
from .proto import graph_classes, torch_to_tensor


class _GraphDefWriter:
    def __init__(self):
        self.classes, self.dtypes = graph_classes()
        self.gd = self.classes["tensorflow.GraphDef"]()
        self.names = set()

    def uniq(self, base):
        name, i = base, 0
        while name in self.names:
            i += 1
            name = f"{base}_{i}"
        self.names.add(name)
        return name

    def node(self, op, name, inputs=(), **attrs):
        n = self.gd.node.add()
        n.op, n.name = op, self.uniq(name)
        n.input.extend(list(inputs))
        for k, v in attrs.items():
            a = n.attr[k]
            if isinstance(v, bool):
                a.b = v
            elif isinstance(v, int):
                a.i = v
            elif isinstance(v, float):
                a.f = v
            elif isinstance(v, str):
                a.s = v.encode()
            elif isinstance(v, torch.Tensor):
                a.tensor.CopyFrom(torch_to_tensor(v))
            elif isinstance(v, tuple) and v and v[0] == "type":
                a.type = v[1]
            elif isinstance(v, list):
                if all(isinstance(x, int) for x in v):
                    a.list.i.extend(v)
                else:
                    a.list.f.extend([float(x) for x in v])
            elif isinstance(v, dict) and "shape" in v:
                for s in v["shape"]:
                    a.shape.dim.add().size = int(s)
        return n.name

    def const(self, name, t: torch.Tensor):
        t = t.detach().cpu()
        if t.dtype == torch.bfloat16:
            t = t.float()
        dt = {torch.float32: 1, torch.int32: 3, torch.int64: 9}[t.dtype]
        return self.node("Const", name, value=t, dtype=("type", dt))


def _f32(x):
    return x.detach().float().cpu()


class TensorflowSaver:
    @staticmethod
    def save_graph(model, inputs: Sequence[Tuple[str, Sequence[int]]], path: str, byte_order="little",
                   data_format="NHWC"):
        """``saveGraph(model, inputs = [(name, shape)], path)`` — writes a binary GraphDef."""
        w = _GraphDefWriter()
        ins = [w.node("Placeholder", n, dtype=("type", 1), shape={"shape": [max(s, -1) for s in shape]})
               for n, shape in inputs]
        out = _emit(w, model, ins[0] if len(ins) == 1 else ins)
        outs = out if isinstance(out, list) else [out]
        for i, o in enumerate(outs):
            w.node("Identity", "output" if len(outs) == 1 else f"output_{i}", [o], T=("type", 1))
        with open(path, "wb") as f:
            f.write(w.gd.SerializeToString())
        return w.gd

    saveGraph = save_graph


def _emit(w: _GraphDefWriter, m, x):
    """Emit ``m`` applied to TF tensor name(s) ``x``; returns the output tensor name(s)."""
    name = m.get_name() if hasattr(m, "get_name") else type(m).__name__
    if isinstance(m, Graph):
        acts = {}
        ins = x if isinstance(x, list) else [x]
        for n, v in zip(m.inputs, ins):
            # an input node is a placeholder (Input()) or a real layer with no predecessor
            # (``conv1.inputs()`` in Save.scala): the latter is applied to the placeholder
            acts[n._id] = v if isinstance(n.element, S.Identity) else _emit(w, n.element, v)
        for n in m.forward_order:
            if n._id in acts:
                continue
            prev = [acts[p._id] for p in n.prev_nodes]
            prev = [p[i - 1] if i and isinstance(p, list) else p for p, i in zip(prev, n.prev_index)]
            acts[n._id] = _emit(w, n.element, prev[0] if len(prev) == 1 else prev)
        outs = [acts[o._id] for o in m.outputs_nodes]
        return outs[0] if len(outs) == 1 else outs
    if isinstance(m, Sequential):
        for c in m.modules:
            x = _emit(w, c, x)
        return x
    if isinstance(m, L.Linear):
        wt = w.const(name + "/weight", _f32(m.weight).t().contiguous())
        y = w.node("MatMul", name + "/matmul", [x, wt], T=("type", 1), transpose_a=False, transpose_b=False)
        if getattr(m, "bias", None) is not None:
            b = w.const(name + "/bias", _f32(m.bias))
            y = w.node("BiasAdd", name, [y, b], T=("type", 1), data_format="NHWC")
        return y
    if isinstance(m, C.SpatialConvolution) and m.nGroup == 1:
        fmt = m.format
        wk = _f32(m.weight).reshape(m.nOutputPlane, m.nInputPlane, m.kernelH, m.kernelW).permute(2, 3, 1, 0)
        ft = w.const(name + "/filter", wk.contiguous())
        if m.padW == -1:
            pad = "SAME"
        elif m.padW == 0 and m.padH == 0:
            pad = "VALID"
        else:
            pads = [[0, 0], [m.padH, m.padH], [m.padW, m.padW], [0, 0]] if fmt == "NHWC" else \
                [[0, 0], [0, 0], [m.padH, m.padH], [m.padW, m.padW]]
            pt = w.const(name + "/paddings", torch.tensor(pads, dtype=torch.int32))
            x = w.node("Pad", name + "/pad", [x, pt], T=("type", 1), Tpaddings=("type", 3))
            pad = "VALID"
        strides = [1, m.strideH, m.strideW, 1] if fmt == "NHWC" else [1, 1, m.strideH, m.strideW]
        y = w.node("Conv2D", name + "/conv", [x, ft], T=("type", 1), strides=strides, padding=pad,
                   data_format=fmt, use_cudnn_on_gpu=True)
        if m.bias is not None:
            b = w.const(name + "/bias", _f32(m.bias))
            y = w.node("BiasAdd", name, [y, b], T=("type", 1), data_format=fmt)
        return y
    if isinstance(m, (P.SpatialMaxPooling, P.SpatialAveragePooling)):
        fmt = getattr(m, "format", "NCHW")
        k = [1, m.kH, m.kW, 1] if fmt == "NHWC" else [1, 1, m.kH, m.kW]
        s = [1, m.dH, m.dW, 1] if fmt == "NHWC" else [1, 1, m.dH, m.dW]
        pad = "SAME" if m.padW == -1 else "VALID"
        if m.padW > 0 or m.padH > 0:
            if isinstance(m, P.SpatialAveragePooling):
                raise NotImplementedError("explicitly padded average pooling has no TF equivalent")
            pads = [[0, 0], [m.padH, m.padH], [m.padW, m.padW], [0, 0]] if fmt == "NHWC" else \
                [[0, 0], [0, 0], [m.padH, m.padH], [m.padW, m.padW]]
            pt = w.const(name + "/paddings", torch.tensor(pads, dtype=torch.int32))
            mn = w.const(name + "/neg_inf", torch.tensor(-3.4e38))
            x = w.node("PadV2", name + "/pad", [x, pt, mn], T=("type", 1), Tpaddings=("type", 3))
        op = "MaxPool" if isinstance(m, P.SpatialMaxPooling) else "AvgPool"
        return w.node(op, name, [x], T=("type", 1), ksize=k, strides=s, padding=pad, data_format=fmt)
    if isinstance(m, N.BatchNormalization):
        fmt = "NCHW" if isinstance(m, N.SpatialBatchNormalization) else "NHWC"
        ones, zeros = torch.ones(m.nOutput), torch.zeros(m.nOutput)
        g = w.const(name + "/scale", _f32(m.weight) if m.affine else ones)
        b = w.const(name + "/offset", _f32(m.bias) if m.affine else zeros)
        mu = w.const(name + "/mean", _f32(m.runningMean))
        var = w.const(name + "/variance", _f32(m.runningVar))
        if fmt == "NHWC":
            # 2-D input: FusedBatchNorm needs 4-D; express as affine ops
            inv = torch.rsqrt(_f32(m.runningVar) + m.eps)
            sc = w.const(name + "/a", (inv * (_f32(m.weight) if m.affine else ones)))
            sh = w.const(name + "/b", (_f32(m.bias) if m.affine else zeros) -
                         _f32(m.runningMean) * inv * (_f32(m.weight) if m.affine else ones))
            y = w.node("Mul", name + "/mul", [x, sc], T=("type", 1))
            return w.node("Add", name, [y, sh], T=("type", 1))
        return w.node("FusedBatchNorm", name, [x, g, b, mu, var], T=("type", 1), epsilon=float(m.eps),
                      data_format=fmt, is_training=False)
    simple = {A.ReLU: "Relu", A.Tanh: "Tanh", A.Sigmoid: "Sigmoid", A.ReLU6: "Relu6", A.SoftMax: "Softmax",
              A.LogSoftMax: "LogSoftmax"}
    for cls, op in simple.items():
        if isinstance(m, cls):
            return w.node(op, name, [x], T=("type", 1))
    if isinstance(m, (D.Dropout, S.Identity)):
        return w.node("Identity", name, [x], T=("type", 1))
    if isinstance(m, S.Reshape):
        shape = ([-1] + m.size) if m.batchMode is not False else m.size
        sh = w.const(name + "/shape", torch.tensor(shape, dtype=torch.int32))
        return w.node("Reshape", name, [x, sh], T=("type", 1), Tshape=("type", 3))
    if isinstance(m, S.View):
        sh = w.const(name + "/shape", torch.tensor([-1] + m.sizes, dtype=torch.int32))
        return w.node("Reshape", name, [x, sh], T=("type", 1), Tshape=("type", 3))
    if isinstance(m, TO.CAddTable):
        return w.node("AddN", name, list(x), T=("type", 1), N=len(x))
    if isinstance(m, TO.JoinTable):
        ax = w.const(name + "/axis", torch.tensor(m.dimension - 1 + (1 if m.nInputDims else 0), dtype=torch.int32))
        return w.node("ConcatV2", name, list(x) + [ax], T=("type", 1), N=len(x), Tidx=("type", 3))
    raise NotImplementedError(f"TensorflowSaver: no TF mapping for {type(m).__name__}")
