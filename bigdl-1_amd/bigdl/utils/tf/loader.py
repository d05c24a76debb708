"""TensorFlow GraphDef → BigDL ``Graph`` (``DL/utils/tf/TensorflowLoader.scala``,
``TensorflowToBigDL.scala``, ``DL/utils/tf/loaders/*.scala``).

Pipeline: parse the GraphDef (binary ``.pb`` or text ``.pbtxt``) → walk back from the requested
outputs to the requested inputs (``"name"`` or ``"name:i"``) → fold every subgraph that depends on
constants only (``Const``, ``Identity`` of a const, shape arithmetic …) into values at load time →
pattern-fuse the trainable layers (``MatMul`` + const weights [+ ``BiasAdd``/``Add`` const] →
``Linear``; ``Conv2D`` + const filter [+ bias] → NHWC ``SpatialConvolution``;
``FusedBatchNorm`` with const statistics → per-channel affine) → one module per remaining op,
connected as a ``Graph``.  Graphs with control flow (``Switch``/``Merge`` conditionals and
``Enter``/``Exit``/``NextIteration``/``LoopCond`` while loops) load as a forward-only
``DynamicGraph`` run by the scheduler (``nn/dynamic_graph.py``).  Queue/reader ops are not loaded
(training-input pipelines are replaced by BigDL's own data layer, as in the reference's ``Session``).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ...nn import Graph, Input, Linear, SpatialConvolution
from ...nn.ops import Operation as _Operation
from ...nn.tf import Const as _Const
import sys
O = sys.modules[_Operation.__module__]  # bigdl.nn.ops (bigdl.nn's namespace also has bigdl.ops as "ops")
T = sys.modules[_Const.__module__]
from ...nn.tf import grad_ops as G  # noqa: E402
from ...nn.layers import activation as A
from ...utils.table import Table
from .proto import graph_classes, tensor_to_torch, torch_dtype


def _attr(node, name, default=None):
    if name not in node.attr:
        return default
    a = node.attr[name]
    kind = a.WhichOneof("value")
    if kind == "list":
        lv = a.list
        for f in ("i", "f", "s", "b", "type", "shape", "tensor"):
            vals = list(getattr(lv, f))
            if vals:
                return [v.decode() if isinstance(v, bytes) else v for v in vals]
        return []
    v = getattr(a, kind) if kind else default
    return v.decode() if isinstance(v, bytes) else v


def _num_outputs(node) -> int:
    op = node.op
    if op in ("Split", "SplitV"):
        return int(_attr(node, "num_split", 1))
    if op == "Unpack":
        return int(_attr(node, "num", 1))
    if op in ("TopKV2", "TopK", "Switch", "RefSwitch", "TensorArrayV3", "TensorArrayGradV3", "TensorArrayConcatV3"):
        return 2
    if op.startswith("FusedBatchNormGrad"):
        return 5
    if op.startswith("FusedBatchNorm"):
        return 6 if op.endswith("V3") else 5
    if op == "ParseExample":
        return len(_attr(node, "Tdense", []) or []) + 3 * int(_attr(node, "Nsparse", 0) or 0)
    if op == "ParseSingleExample":
        return len(_attr(node, "dense_keys", []) or []) + 3 * int(_attr(node, "num_sparse", 0) or 0)
    if op == "BroadcastGradientArgs":
        return 2
    return 1


def _split_ref(ref: str) -> Tuple[str, int]:
    if ":" in ref:
        n, i = ref.rsplit(":", 1)
        return n, int(i)
    return ref, 0


class _Lambda(O.Operation):
    """Generic forward-only op around a torch callable taking the positional inputs."""

    def __init__(self, fn, name=""):
        super().__init__()
        self.fn = fn
        self._op = name

    def updateOutput(self, input):
        args = input.values() if isinstance(input, Table) else [input]
        return self.fn(*args)


def _pads_of(node):
    return _attr(node, "padding", "VALID")


def _reduce(fn):
    def build(node):
        keep = bool(_attr(node, "keep_dims", False) or _attr(node, "keepdims", False))

        def f(x, axes):
            ax = tuple(int(a) % max(x.dim(), 1) for a in torch.as_tensor(axes).flatten().tolist())
            return fn(x, ax, keep) if ax else x
        return _Lambda(f, node.op)
    return build


def _concat(*args):
    return torch.cat(list(args[:-1]), dim=int(args[-1]))


# TF op → builder(node) → module taking Table(inputs in TF order)
_OPS = {
    "Identity": lambda n: _Lambda(lambda x: x, "Identity"),
    "StopGradient": lambda n: _Lambda(lambda x: x, "StopGradient"),
    "Snapshot": lambda n: _Lambda(lambda x: x, "Snapshot"),
    "Add": lambda n: _Lambda(torch.add, "Add"), "AddV2": lambda n: _Lambda(torch.add, "AddV2"),
    "AddN": lambda n: _Lambda(lambda *xs: sum(xs[1:], xs[0]), "AddN"),
    "Sub": lambda n: _Lambda(torch.sub, "Sub"), "Mul": lambda n: _Lambda(torch.mul, "Mul"),
    "RealDiv": lambda n: _Lambda(torch.div, "RealDiv"), "Div": lambda n: _Lambda(torch.div, "Div"),
    "FloorDiv": lambda n: O.FloorDiv(), "FloorMod": lambda n: O.FloorMod(), "TruncateDiv": lambda n: O.TruncateDiv(),
    "Maximum": lambda n: O.Maximum(), "Minimum": lambda n: O.Minimum(), "Pow": lambda n: O.Pow(),
    "SquaredDifference": lambda n: O.SquaredDifference(),
    "Neg": lambda n: _Lambda(torch.neg, "Neg"), "Abs": lambda n: _Lambda(torch.abs, "Abs"),
    "Square": lambda n: _Lambda(torch.square, "Square"), "Sqrt": lambda n: _Lambda(torch.sqrt, "Sqrt"),
    "Rsqrt": lambda n: _Lambda(torch.rsqrt, "Rsqrt"), "Exp": lambda n: O.Exp(), "Log": lambda n: _Lambda(torch.log, "Log"),
    "Log1p": lambda n: O.Log1p(), "Expm1": lambda n: O.Expm1(), "Reciprocal": lambda n: O.Inv(), "Inv": lambda n: O.Inv(),
    "Floor": lambda n: O.Floor(), "Ceil": lambda n: O.Ceil(), "Round": lambda n: O.Round(), "Rint": lambda n: O.Rint(),
    "Sign": lambda n: O.Sign(), "Erf": lambda n: O.Erf(), "Erfc": lambda n: O.Erfc(), "Lgamma": lambda n: O.Lgamma(),
    "Digamma": lambda n: O.Digamma(), "IsFinite": lambda n: O.IsFinite(), "IsInf": lambda n: O.IsInf(),
    "IsNan": lambda n: O.IsNan(),
    "Tanh": lambda n: A.Tanh(), "Sigmoid": lambda n: A.Sigmoid(), "Relu": lambda n: A.ReLU(),
    "Relu6": lambda n: A.ReLU6(), "Elu": lambda n: A.ELU(), "Softplus": lambda n: A.SoftPlus(),
    "Softsign": lambda n: A.SoftSign(),
    "Softmax": lambda n: _Lambda(lambda x: torch.softmax(x, -1), "Softmax"),
    "LogSoftmax": lambda n: _Lambda(lambda x: torch.log_softmax(x, -1), "LogSoftmax"),
    "Equal": lambda n: O.Equal(), "NotEqual": lambda n: O.NotEqual(), "Greater": lambda n: O.Greater(),
    "GreaterEqual": lambda n: O.GreaterEqual(), "Less": lambda n: O.Less(), "LessEqual": lambda n: O.LessEqual(),
    "LogicalAnd": lambda n: O.LogicalAnd(), "LogicalOr": lambda n: O.LogicalOr(), "LogicalNot": lambda n: O.LogicalNot(),
    "ApproximateEqual": lambda n: O.ApproximateEqual(_attr(n, "tolerance", 1e-5)),
    "MatMul": lambda n: _Lambda(lambda a, b: torch.matmul(a.t() if _attr(n, "transpose_a") else a,
                                                            b.t() if _attr(n, "transpose_b") else b), "MatMul"),
    "BatchMatMul": lambda n: O.BatchMatMul(bool(_attr(n, "adj_x")), bool(_attr(n, "adj_y"))),
    "BatchMatMulV2": lambda n: O.BatchMatMul(bool(_attr(n, "adj_x")), bool(_attr(n, "adj_y"))),
    "BiasAdd": lambda n: _Lambda((lambda x, b: x + b.view(1, -1, 1, 1)) if _attr(n, "data_format") == "NCHW"
                                 else (lambda x, b: x + b), "BiasAdd"),
    "Conv2D": lambda n: T.Conv2D(_attr(n, "strides"), _pads_of(n), _attr(n, "data_format", "NHWC"),
                                 _attr(n, "dilations", [1, 1, 1, 1]) or [1, 1, 1, 1]),
    "DepthwiseConv2dNative": lambda n: _depthwise(n),
    "MaxPool": lambda n: T.MaxPool(_attr(n, "ksize"), _attr(n, "strides"), _pads_of(n), _attr(n, "data_format", "NHWC")),
    "AvgPool": lambda n: T.AvgPool(_attr(n, "ksize"), _attr(n, "strides"), _pads_of(n), _attr(n, "data_format", "NHWC")),
    "LRN": lambda n: T.LRN(_attr(n, "depth_radius", 5), _attr(n, "bias", 1.0), _attr(n, "alpha", 1.0),
                           _attr(n, "beta", 0.5)),
    "FusedBatchNorm": lambda n: T.FusedBatchNorm(_attr(n, "epsilon", 1e-3), _attr(n, "data_format", "NHWC"),
                                                 bool(_attr(n, "is_training", False))),
    "FusedBatchNormV2": lambda n: _OPS["FusedBatchNorm"](n), "FusedBatchNormV3": lambda n: _OPS["FusedBatchNorm"](n),
    "Reshape": lambda n: _Lambda(lambda x, s: x.reshape([int(v) for v in torch.as_tensor(s).flatten().tolist()]),
                                 "Reshape"),
    "Squeeze": lambda n: _Lambda((lambda x: x.squeeze()) if not _attr(n, "squeeze_dims") else
                                 (lambda x: _squeeze(x, _attr(n, "squeeze_dims"))), "Squeeze"),
    "ExpandDims": lambda n: _Lambda(lambda x, d: x.unsqueeze(int(d)), "ExpandDims"),
    "Transpose": lambda n: _Lambda(lambda x, p: x.permute(*[int(v) for v in p.tolist()]).contiguous(), "Transpose"),
    "ConcatV2": lambda n: _Lambda(_concat, "ConcatV2"),
    "Concat": lambda n: _Lambda(lambda d, *xs: torch.cat(list(xs), int(d)), "Concat"),
    "Pack": lambda n: _Lambda(lambda *xs: torch.stack(list(xs), int(_attr(n, "axis", 0))), "Pack"),
    "Unpack": lambda n: _Lambda(lambda x: Table(*torch.unbind(x, int(_attr(n, "axis", 0)))), "Unpack"),
    "Split": lambda n: T.Split(int(_attr(n, "num_split", 1))),
    "Shape": lambda n: T.Shape(), "Size": lambda n: T.SizeOp(), "Rank": lambda n: O.Rank(),
    "Fill": lambda n: T.Fill(), "Range": lambda n: O.RangeOps(), "Tile": lambda n: O.Tile(),
    "Slice": lambda n: _Lambda(lambda x, b, s: O.Slice(b.tolist(), s.tolist()).forward(x), "Slice"),
    "StridedSlice": lambda n: T.StridedSlice(begin_mask=_attr(n, "begin_mask", 0), end_mask=_attr(n, "end_mask", 0),
                                             ellipsis_mask=_attr(n, "ellipsis_mask", 0),
                                             new_axis_mask=_attr(n, "new_axis_mask", 0),
                                             shrink_axis_mask=_attr(n, "shrink_axis_mask", 0)),
    "Pad": lambda n: O.Pad(), "PadV2": lambda n: _Lambda(lambda x, p, v: O.Pad(constant_value=float(v)).forward(
        Table(x, p)), "PadV2"),
    "MirrorPad": lambda n: O.Pad(_attr(n, "mode", "REFLECT")),
    "Cast": lambda n: O.Cast(torch_dtype(_attr(n, "DstT", 1))),
    "Sum": _reduce(lambda x, a, k: x.sum(a, keepdim=k)), "Mean": _reduce(lambda x, a, k: x.float().mean(a, keepdim=k)),
    "Max": _reduce(lambda x, a, k: x.amax(a, keepdim=k)), "Min": _reduce(lambda x, a, k: x.amin(a, keepdim=k)),
    "Prod": _reduce(lambda x, a, k: _prod(x, a, k)),
    "All": _reduce(lambda x, a, k: _reduce_bool(x, a, k, torch.all)),
    "Any": _reduce(lambda x, a, k: _reduce_bool(x, a, k, torch.any)),
    "ArgMax": lambda n: _Lambda(lambda x, d: x.argmax(int(d)), "ArgMax"),
    "ArgMin": lambda n: _Lambda(lambda x, d: x.argmin(int(d)), "ArgMin"),
    "Gather": lambda n: O.Gather(), "GatherV2": lambda n: O.Gather(),
    "OneHot": lambda n: O.OneHot(int(_attr(n, "axis", -1))),
    "TopKV2": lambda n: _Lambda(lambda x, k: Table(*torch.topk(x, int(k), -1)), "TopKV2"),
    "InTopK": lambda n: O.InTopK(int(_attr(n, "k", 1)), True),
    "Select": lambda n: O.Select(), "SelectV2": lambda n: O.Select(),
    "SegmentSum": lambda n: O.SegmentSum(),
    "L2Loss": lambda n: _Lambda(lambda x: (x.float() ** 2).sum() / 2, "L2Loss"),
    "SoftmaxCrossEntropyWithLogits": lambda n: O.CrossEntropy(),
    "ResizeBilinear": lambda n: O.ResizeBilinearOps(bool(_attr(n, "align_corners", False))),
    "RandomUniform": lambda n: O.RandomUniform(seed=_attr(n, "seed", None) or None),
    "TruncatedNormal": lambda n: O.TruncatedNormal(seed=_attr(n, "seed", None) or None),
    "Substr": lambda n: O.Substr(),
    "InvertPermutation": lambda n: T.InvertPermutation(), "ConcatOffset": lambda n: T.ConcatOffset(),
    "Switch": lambda n: T.SwitchOps(), "Merge": lambda n: T.MergeOps(),
    "RefSwitch": lambda n: T.SwitchOps(), "RefMerge": lambda n: T.MergeOps(),
    "Enter": lambda n: T.Enter(_attr(n, "frame_name", "") or ""),
    "RefEnter": lambda n: T.Enter(_attr(n, "frame_name", "") or ""),
    "Exit": lambda n: T.Exit(), "RefExit": lambda n: T.Exit(),
    "NextIteration": lambda n: T.NextIteration(), "RefNextIteration": lambda n: T.NextIteration(),
    "LoopCond": lambda n: T.LoopCondition(),
    "NoOp": lambda n: T.NoOp(), "Assert": lambda n: T.Assert(),
    "DecodeJpeg": lambda n: T.DecodeImage(int(_attr(n, "channels", 3) or 3)),
    "DecodePng": lambda n: T.DecodeImage(int(_attr(n, "channels", 3) or 3)),
    "DecodeGif": lambda n: T.DecodeImage(3), "DecodeBmp": lambda n: T.DecodeImage(3),
    "DecodeRaw": lambda n: T.DecodeRaw(torch_dtype(_attr(n, "out_type", 4)), bool(_attr(n, "little_endian", True))),
}


def _g(cls, *attrs, **kw):
    """Builder of a grad op class from node attributes: ``attrs`` = (attr name, default) pairs."""
    return lambda n: cls(*[_attr(n, a, d) if not callable(d) else d(n) for a, d in attrs], **kw)


def _fmt(n):
    return _attr(n, "data_format", "NHWC") or "NHWC"


def _dil(n):
    return _attr(n, "dilations", [1, 1, 1, 1]) or [1, 1, 1, 1]


def _parse_single(n):
    dense_t = [torch_dtype(t) for t in (_attr(n, "Tdense", []) or [])]
    shapes = []
    for sh in (_attr(n, "dense_shapes", []) or []):
        dims = [int(d.size) for d in getattr(sh, "dim", [])]
        shapes.append(dims)
    return G.ParseSingleExample(_attr(n, "dense_keys", []) or [], dense_t, shapes or [[] for _ in dense_t],
                                _attr(n, "sparse_keys", []) or [],
                                [torch_dtype(t) for t in (_attr(n, "sparse_types", []) or [])])


_OPS.update({
    "ReluGrad": lambda n: G.ReluGrad(), "Relu6Grad": lambda n: G.Relu6Grad(), "EluGrad": lambda n: G.EluGrad(),
    "SoftplusGrad": lambda n: G.SoftplusGrad(), "SoftsignGrad": lambda n: G.SoftsignGrad(),
    "TanhGrad": lambda n: G.TanhGrad(), "SigmoidGrad": lambda n: G.SigmoidGrad(),
    "SqrtGrad": lambda n: G.SqrtGrad(), "RsqrtGrad": lambda n: G.RsqrtGrad(),
    "InvGrad": lambda n: G.InvGrad(), "ReciprocalGrad": lambda n: G.ReciprocalGrad(),
    "Mod": lambda n: G.Mod(), "TruncateMod": lambda n: G.TruncateMod(),
    "BiasAddGrad": lambda n: G.BiasAddGrad(_fmt(n)),
    "BiasAddV1": lambda n: _Lambda(lambda x, b: x + b, "BiasAddV1"),
    "BroadcastGradientArgs": lambda n: G.BroadcastGradientArgs(),
    "Conv2DBackpropInput": lambda n: G.Conv2DTranspose(_attr(n, "strides"), _pads_of(n), _fmt(n), _dil(n)),
    "Conv2DBackpropFilter": lambda n: G.Conv2DBackFilter(_attr(n, "strides"), _pads_of(n), _fmt(n), _dil(n)),
    "Conv3D": lambda n: G.Conv3D(_attr(n, "strides"), _pads_of(n), _attr(n, "data_format", "NDHWC") or "NDHWC"),
    "Conv3DBackpropInput": lambda n: G.Conv3DBackpropInput(_attr(n, "strides"), _pads_of(n),
                                                          _attr(n, "data_format", "NDHWC") or "NDHWC"),
    "Conv3DBackpropInputV2": lambda n: G.Conv3DBackpropInputV2(_attr(n, "strides"), _pads_of(n),
                                                              _attr(n, "data_format", "NDHWC") or "NDHWC"),
    "Conv3DBackpropFilter": lambda n: G.Conv3DBackpropFilter(_attr(n, "strides"), _pads_of(n),
                                                            _attr(n, "data_format", "NDHWC") or "NDHWC"),
    "Conv3DBackpropFilterV2": lambda n: G.Conv3DBackpropFilterV2(_attr(n, "strides"), _pads_of(n),
                                                                _attr(n, "data_format", "NDHWC") or "NDHWC"),
    "DepthwiseConv2dNativeBackpropInput": lambda n: G.DepthwiseConv2dNativeBackpropInput(
        _attr(n, "strides"), _pads_of(n), _fmt(n)),
    "DepthwiseConv2dNativeBackpropFilter": lambda n: G.DepthwiseConv2dNativeBackpropFilter(
        _attr(n, "strides"), _pads_of(n), _fmt(n)),
    "Dilation2D": lambda n: O.Dilation2D(_attr(n, "strides"), _attr(n, "rates"), _pads_of(n)),
    "Dilation2DBackpropInput": lambda n: G.Dilation2DBackpropInput(_attr(n, "strides"), _attr(n, "rates"),
                                                                  _pads_of(n)),
    "Dilation2DBackpropFilter": lambda n: G.Dilation2DBackpropFilter(_attr(n, "strides"), _attr(n, "rates"),
                                                                    _pads_of(n)),
    "FusedBatchNormGrad": lambda n: G.FusedBatchNormGrad(_attr(n, "epsilon", 1e-4), _fmt(n),
                                                         bool(_attr(n, "is_training", True))),
    "FusedBatchNormGradV2": lambda n: _OPS["FusedBatchNormGrad"](n),
    "FusedBatchNormGradV3": lambda n: _OPS["FusedBatchNormGrad"](n),
    "MaxPoolGrad": lambda n: G.MaxPoolGrad(_attr(n, "ksize"), _attr(n, "strides"), _pads_of(n), _fmt(n)),
    "AvgPoolGrad": lambda n: G.AvgPoolGrad(_attr(n, "ksize"), _attr(n, "strides"), _pads_of(n), _fmt(n)),
    "LRNGrad": lambda n: G.LRNGrad(_attr(n, "depth_radius", 5), _attr(n, "bias", 1.0), _attr(n, "alpha", 1.0),
                                   _attr(n, "beta", 0.5)),
    "ResizeBilinearGrad": lambda n: G.ResizeBilinearGrad(bool(_attr(n, "align_corners", False))),
    "ParseSingleExample": _parse_single,
})


def _squeeze(x, dims):
    for d in sorted([d % x.dim() for d in dims], reverse=True):
        x = x.squeeze(d)
    return x


def _prod(x, axes, keep):
    for a in sorted(axes, reverse=True):
        x = x.prod(a, keepdim=keep)
    return x


def _reduce_bool(x, axes, keep, fn):
    x = x.bool()
    for a in sorted(axes, reverse=True):
        x = fn(x, dim=a, keepdim=keep)
    return x


def _depthwise(n):
    s = _attr(n, "strides")
    fmt = _attr(n, "data_format", "NHWC")
    sh, sw = (s[1], s[2]) if fmt == "NHWC" else (s[2], s[3])
    if _pads_of(n) == "SAME":
        def f(x, w):
            xc = x.permute(0, 3, 1, 2) if fmt == "NHWC" else x
            kh, kw = w.shape[0], w.shape[1]
            pt, pb = T._tf_pads(xc.shape[2], kh, sh, "SAME")
            pl, pr = T._tf_pads(xc.shape[3], kw, sw, "SAME")
            xc = torch.nn.functional.pad(xc, (pl, pr, pt, pb))
            y = O.DepthwiseConv2D(sw, sh, 0, 0, "NCHW").forward(Table(xc, w))
            return y.permute(0, 2, 3, 1).contiguous() if fmt == "NHWC" else y
        return _Lambda(f, "DepthwiseConv2dNative")
    return O.DepthwiseConv2D(sw, sh, 0, 0, fmt)


def _ta_shape(n):
    """A TensorArrayV3 ``element_shape`` when fully defined, else None (no shape check)."""
    sh = _attr(n, "element_shape", None)
    if sh is None or getattr(sh, "unknown_rank", False):
        return None
    dims = [int(d.size) for d in getattr(sh, "dim", [])]
    return dims if dims and all(d >= 0 for d in dims) else None


# TensorArray / Stack resources (nn/tf/data_flow.py; the reference's loaders in DL/utils/tf/loaders)
_DATA_FLOW = {
    "TensorArrayV3": lambda n: T.TensorArrayCreator(_ta_shape(n), bool(_attr(n, "dynamic_size", False)),
                                                    bool(_attr(n, "clear_after_read", True)),
                                                    bool(_attr(n, "identical_element_shapes", False)),
                                                    (_attr(n, "tensor_array_name", "") or "")),
    "TensorArrayGradV3": lambda n: T.TensorArrayGrad(_attr(n, "source", "") or ""),
    "TensorArrayWriteV3": lambda n: T.TensorArrayWrite(), "TensorArrayReadV3": lambda n: T.TensorArrayRead(),
    "TensorArrayGatherV3": lambda n: T.TensorArrayGather(), "TensorArrayScatterV3": lambda n: T.TensorArrayScatter(),
    "TensorArrayConcatV3": lambda n: T.TensorArrayConcat(), "TensorArraySplitV3": lambda n: T.TensorArraySplit(),
    "TensorArraySizeV3": lambda n: T.TensorArraySize(), "TensorArrayCloseV3": lambda n: T.TensorArrayClose(),
    "StackV2": lambda n: T.StackCreator(_attr(n, "stack_name", "") or ""),
    "StackPushV2": lambda n: T.StackPush(), "StackPopV2": lambda n: T.StackPop(),
}
_OPS.update(_DATA_FLOW)

# data-dependent control flow: executed by a DynamicGraph scheduler, never constant-folded
_CONTROL = {"Switch", "RefSwitch", "Merge", "RefMerge", "Enter", "RefEnter", "Exit", "RefExit", "NextIteration",
            "RefNextIteration", "LoopCond"}
_NOT_LOADABLE = {"FIFOQueueV2", "QueueDequeueV2", "QueueDequeueManyV2",
                 "QueueEnqueueV2", "QueueEnqueueManyV2", "TFRecordReaderV2", "ReaderReadV2", "RandomShuffleQueueV2"}
_STATEFUL = {"RandomUniform", "TruncatedNormal", "RandomShuffle", "Placeholder", "PlaceholderWithDefault", "VariableV2",
             *_DATA_FLOW}


class TensorflowLoader:
    """``TensorflowLoader.scala``: ``load(path, inputs, outputs, byte_order, bin_file)``."""

    @staticmethod
    def parse(path: str) -> List:
        classes, _ = graph_classes()
        gd = classes["tensorflow.GraphDef"]()
        with open(path, "rb") as f:
            data = f.read()
        if path.endswith(".pbtxt") or path.endswith(".txt"):
            from google.protobuf import text_format
            text_format.Merge(data.decode(), gd)
        else:
            gd.ParseFromString(data)
        return list(gd.node)

    @staticmethod
    def load(path: str, inputs: Sequence[str], outputs: Sequence[str], byte_order: str = "little",
             bin_file: Optional[str] = None, generated_backward: bool = False):
        """``bin_file``: variable values for the graph's ``VariableV2`` / ``VarHandleOp`` nodes — a
        TensorFlow V2 checkpoint prefix (``<prefix>.index`` + data shards, read without
        TensorFlow, :mod:`bigdl.utils.tf.checkpoint`) or an ``.npz`` / ``.safetensors`` file of
        name → array.  Variables consumed by MatMul / Conv2D / BiasAdd become the trainable
        weights of the fused Linear / SpatialConvolution layers."""
        nodes = TensorflowLoader.parse(path)
        variables = load_variables(bin_file) if bin_file else None
        return _Builder(nodes, byte_order, variables).build(list(inputs), list(outputs))

    @staticmethod
    def checkpoints(graph_file: str, bin_file: str, byte_order: str = "little"):
        """``TensorflowLoader.checkpoints`` (TensorflowLoader.scala:88): a :class:`Session` over the
        graph with its variables loaded from ``bin_file``."""
        from .session import Session
        return Session(TensorflowLoader.parse(graph_file), load_variables(bin_file), byte_order)


def load_variables(path: str) -> Dict[str, torch.Tensor]:
    from .checkpoint import is_checkpoint, read_checkpoint
    if is_checkpoint(path):
        arrs = read_checkpoint(path)
    elif path.endswith(".safetensors"):
        from safetensors.numpy import load_file
        arrs = load_file(path)
    else:
        with np.load(path, allow_pickle=False) as z:
            arrs = {k: z[k] for k in z.files}
    return {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in arrs.items()}


_VAR_OPS = ("VariableV2", "Variable", "VarHandleOp")
_VAR_READS = ("ReadVariableOp", "Identity", "StopGradient", "Snapshot")


class _Builder:
    def __init__(self, nodes, byte_order, variables: Optional[Dict[str, torch.Tensor]] = None):
        self.nodes = {n.name: n for n in nodes}
        self.byte_order = byte_order
        self.variables = variables or {}
        self.var_bindings: List = []   # (variable, module, attr, module-param → TF-layout fn)
        self.consts: Dict[str, object] = {}
        self.consumers: Dict[str, List[str]] = {}
        for n in nodes:
            for i in n.input:
                if not i.startswith("^"):
                    self.consumers.setdefault(_split_ref(i)[0], []).append(n.name)

    # ------------------------------------------------------------------ validation
    def _check_inputs(self, inputs):
        """``"name"`` feeds node ``name`` (a Placeholder is replaced; any other node keeps its op and
        gets the data in place of its inputs); ``"name:i"`` feeds the i-th input edge of ``name``."""
        if len(set(inputs)) != len(inputs):
            raise ValueError(f"duplicate input names {inputs}")
        names = [_split_ref(i)[0] for i in inputs]
        if len(set(names)) != len(names):
            raise ValueError(f"conflicting input names {inputs}")
        for spec in inputs:
            n, idx = _split_ref(spec)
            if n not in self.nodes:
                raise ValueError(f"input {n} not in the graph")
            n_in = len([i for i in self.nodes[n].input if not i.startswith("^")])
            if ":" in spec and idx >= n_in:
                raise ValueError(f"input {spec}: {n} has {n_in} input(s)")

    # ------------------------------------------------------------------ constant folding
    def _const(self, ref: str):
        """Value of tensor ``ref`` if it depends on constants only, else None."""
        n, idx = _split_ref(ref)
        key = f"{n}:{idx}"
        if key in self.consts:
            return self.consts[key]
        node = self.nodes[n]
        val = None
        if n not in self._fed_nodes and node.op in _VAR_OPS and n in self.variables:
            val = self.variables[n]
        elif (n not in self._fed_nodes and node.op in _VAR_READS and self._var_of(ref) is not None):
            val = self.variables[self._var_of(ref)]
        elif n in self._fed_nodes or node.op in _STATEFUL or node.op in _NOT_LOADABLE or node.op in _CONTROL:
            val = None
        elif node.op == "Const":
            val = tensor_to_torch(node.attr["value"].tensor, self.byte_order)
        elif node.op in _OPS:
            data_in = [i for i in node.input if not i.startswith("^")]
            vals = [self._const(i) for i in data_in]
            if data_in and all(v is not None for v in vals):
                m = _OPS[node.op](node)
                out = m.forward(vals[0] if len(vals) == 1 else Table(*vals))
                val = out[idx + 1] if isinstance(out, Table) else out
        self.consts[key] = val
        return val

    def _var_of(self, ref: str) -> Optional[str]:
        """The variable whose value tensor ``ref`` is (through reads / identities), if any."""
        n, _ = _split_ref(ref)
        seen = 0
        while n in self.nodes and seen < 64:
            node = self.nodes[n]
            if node.op in _VAR_OPS:
                return n if n in self.variables else None
            if node.op not in _VAR_READS:
                return None
            data_in = [i for i in node.input if not i.startswith("^")]
            if not data_in:
                return None
            n, _ = _split_ref(data_in[0])
            seen += 1
        return None

    def _bind(self, ref, module, attr, to_tf):
        v = self._var_of(ref)
        if v is not None:
            self.var_bindings.append((v, module, attr, to_tf))

    # ------------------------------------------------------------------ graph construction
    def build(self, inputs, outputs):
        self._check_inputs(inputs)
        self._feed_node, self._feed_edge, self._fed_nodes = {}, {}, set()
        ins = []
        for spec in inputs:
            n, idx = _split_ref(spec)
            node = Input(spec)
            ins.append(node)
            if ":" in spec:
                self._feed_edge[(n, idx)] = node
            else:
                self._feed_node[n] = node
            self._fed_nodes.add(n)
        self._made = {}
        self._has_control = False
        out_nodes = [self._node_for(o) for o in outputs]
        outs = [o if not isinstance(o, tuple) else o[0] for o in out_nodes]
        if self._has_control:
            from ...nn.dynamic_graph import DynamicGraph
            return DynamicGraph(ins, outs, None, generate_backward=False)
        return Graph(ins, outs)

    def _edge(self, name: str, pos: int):
        """Producer of the ``pos``-th data input of node ``name``."""
        if (name, pos) in self._feed_edge:
            return self._feed_edge[(name, pos)]
        data_in = [i for i in self.nodes[name].input if not i.startswith("^")]
        return self._node_for(data_in[pos])

    def _node_for(self, ref: str):
        """ModuleNode (or (node, 1-based output index)) producing tensor ``ref``."""
        from ...nn.graph import ModuleNode
        n, idx = _split_ref(ref)
        node = self.nodes[n]
        if n in self._feed_node and node.op in ("Placeholder", "PlaceholderWithDefault"):
            return self._feed_node[n]
        if node.op in ("Identity", "StopGradient", "Snapshot") and n not in self._fed_nodes:
            return self._edge(n, 0)
        if n in self._made:
            m = self._made[n]
            return (m, idx + 1) if _num_outputs(node) > 1 else m
        c = self._const(ref)
        if c is not None:
            mn = ModuleNode(T.Const(c).set_name(n))
            self._made[n] = mn
            return mn
        if node.op in ("Placeholder", "PlaceholderWithDefault"):
            raise ValueError(f"placeholder {n} is not among the given inputs")
        if node.op in _NOT_LOADABLE:
            raise NotImplementedError(f"TF op {node.op} ({n}) is not loadable; feed data through bigdl.dataset")
        fused = None if n in self._feed_node else self._fuse(node)
        if fused is not None:
            module, edges = fused
        else:
            if node.op not in _OPS:
                raise NotImplementedError(f"unsupported TF op {node.op} ({n})")
            module = _OPS[node.op](node)
            edges = [(n, i) for i in range(len([x for x in node.input if not x.startswith("^")]))]
        module.set_name(n)
        if node.op in _CONTROL:
            from ...nn.dynamic_graph import MergeControlNode, SwitchControlNode
            self._has_control = True
            cls = (SwitchControlNode if node.op in ("Switch", "RefSwitch") else
                   MergeControlNode if node.op in ("Merge", "RefMerge") else ModuleNode)
            # register before resolving inputs: a loop's Merge is reached again through its
            # NextIteration input (the graph has a cycle)
            mn = cls(module)
            self._made[n] = mn
            prevs = [self._feed_node[n]] if n in self._feed_node else [self._edge(nm, pos) for nm, pos in edges]
            mn(*prevs)
            return (mn, idx + 1) if _num_outputs(node) > 1 else mn
        if n in self._feed_node:
            prevs = [self._feed_node[n]]
        else:
            prevs = [self._edge(nm, pos) for nm, pos in edges]
        mn = ModuleNode.create(module, prevs)
        self._made[n] = mn
        return (mn, idx + 1) if _num_outputs(node) > 1 else mn

    # ------------------------------------------------------------------ pattern fusion
    def _bias_of(self, node):
        """If ``node``'s sole consumer is BiasAdd/Add(V2) with a const vector, return (consumer, bias)."""
        cons = self.consumers.get(node.name, [])
        if len(cons) != 1:
            return None, None
        c = self.nodes[cons[0]]
        if c.op not in ("BiasAdd", "Add", "AddV2"):
            return None, None
        ins = [i for i in c.input if not i.startswith("^")]
        other = [i for i in ins if _split_ref(i)[0] != node.name]
        if len(other) != 1:
            return None, None
        b = self._const(other[0])
        if b is None or not isinstance(b, torch.Tensor) or b.dim() != 1:
            return None, None
        return c, b

    def _fuse(self, node):
        ins = [i for i in node.input if not i.startswith("^")]
        if node.op == "MatMul" and not _attr(node, "transpose_a"):
            fused = self._producer_fusable(node)  # Linear weight is [out, in]
            if fused is not None:
                return fused
        if node.op in ("BiasAdd", "Add", "AddV2"):
            src = self.nodes[_split_ref(ins[0])[0]]
            if src.name in self._feed_node:
                return None
            prod = self._producer_fusable(src)
            if prod is not None and self._bias_of(src)[0] is node:
                _, b = self._bias_of(src)
                layer, data = prod
                if isinstance(layer, Linear):
                    nl = Linear(layer.weight.shape[1], layer.weight.shape[0])
                    nl.weight.data.copy_(layer.weight.data)
                    nl.bias.data.copy_(b.float())
                    self.var_bindings = [(v, nl if m is layer else m, a, f) for (v, m, a, f) in self.var_bindings]
                    layer = nl
                else:
                    layer.bias.data.copy_(b.float())
                other = [i for i in ins if _split_ref(i)[0] != src.name]
                self._bind(other[0], layer, "bias", lambda t: t)
                return layer, data
        if node.op == "Conv2D":
            prod = self._producer_fusable(node)
            if prod is not None:
                return prod
        return None

    def _producer_fusable(self, node):
        ins = [i for i in node.input if not i.startswith("^")]
        if node.op == "MatMul" and not _attr(node, "transpose_a"):
            w = self._const(ins[1])
            if w is not None and w.dim() == 2:
                tb = bool(_attr(node, "transpose_b"))
                w = w.t() if not tb else w
                lin = Linear(w.shape[1], w.shape[0], with_bias=False)
                lin.weight.data.copy_(w.float())
                self._bind(ins[1], lin, "weight", (lambda t: t) if tb else (lambda t: t.t()))
                return lin, [(node.name, 0)]
        if node.op == "Conv2D" and _attr(node, "data_format", "NHWC") == "NHWC":
            f = self._const(ins[1])
            dil = _attr(node, "dilations", [1, 1, 1, 1]) or [1, 1, 1, 1]
            if f is not None and dil == [1, 1, 1, 1]:
                kh, kw, cin, cout = f.shape
                s = _attr(node, "strides")
                pad = -1 if _pads_of(node) == "SAME" else 0
                conv = SpatialConvolution(cin, cout, kw, kh, s[2], s[1], pad, pad, data_format="NHWC")
                conv.weight.data.copy_(f.permute(3, 2, 0, 1).reshape(conv.weight.shape).float())
                conv.bias.data.zero_()
                self._bind(ins[1], conv, "weight", lambda t, shp=tuple(f.shape): t.reshape(
                    shp[3], shp[2], shp[0], shp[1]).permute(2, 3, 1, 0))
                return conv, [(node.name, 0)]
        return None
