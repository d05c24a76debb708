"""TensorFlow graph-op layers (``DL/nn/tf/*.scala``): constants and shape ops, ``BiasAdd``,
``StridedSlice``, ``SplitAndSelect``, control-flow primitives, variables/assign, ``ParseExample``,
image decoding and the NN-op forms (``Conv2D``, pooling, their gradient ops) the TF loader maps
GraphDefs onto.  All are forward-only ``Operation``s except ``BiasAdd`` and ``Variable`` which
carry trainable state, as in the reference.
"""
from __future__ import annotations

import io
from typing import List, Sequence

import numpy as np
import torch
import torch.nn.functional as F

from ...utils.table import Table
from ..abstractnn import AbstractModule, TensorModule
from ..ops import Operation, _scalar


# ------------------------------------------------------------------------------------------------ sources
class Const(Operation):
    """A constant source (``nn/tf/ArrayOps.scala`` Const)."""

    def __init__(self, value):
        super().__init__()
        self.value = value

    def updateOutput(self, input=None):
        return self.value


class Fill(Operation):
    """Table(shape, value) → filled tensor."""

    def updateOutput(self, t):
        shape = [int(v) for v in t[1].flatten().tolist()]
        v = t[2]
        return torch.full(shape, _scalar(v), dtype=v.dtype if isinstance(v, torch.Tensor) else torch.float32)


class Shape(Operation):
    def updateOutput(self, x):
        return torch.tensor(list(x.shape), dtype=torch.int32)


class SizeOp(Operation):
    def updateOutput(self, x):
        return torch.tensor(x.numel(), dtype=torch.int32)


class NoOp(Operation):
    def updateOutput(self, input=None):
        return torch.zeros(0)


class ControlDependency(Operation):
    """Marks an execution-order edge; passes its (first) input through (``ControlDependency.scala``)."""

    def updateOutput(self, input):
        return input[1] if isinstance(input, Table) else input


class Assert(Operation):
    """Table(condition, message...) → raises when the condition is false (``Assert.scala``)."""

    def updateOutput(self, t):
        cond = t[1] if isinstance(t, Table) else t
        if not bool(torch.as_tensor(cond).all()):
            msg = t[2] if isinstance(t, Table) and len(t) > 1 else "assertion failed"
            raise AssertionError(str(msg))
        return cond


class InvertPermutation(Operation):
    def updateOutput(self, x):
        out = torch.empty_like(x)
        out[x.long()] = torch.arange(x.numel(), dtype=x.dtype)
        return out


class ConcatOffset(Operation):
    """Table(axis, shape1, shape2, …) → per-input offsets along ``axis``."""

    def updateOutput(self, t):
        axis = int(_scalar(t[1]))
        off, outs = 0, []
        for i in range(2, len(t) + 1):
            o = torch.zeros_like(t[i])
            o[axis] = off
            off += int(t[i][axis])
            outs.append(o)
        return Table(*outs)


# ------------------------------------------------------------------------------------------------ array ops
class StridedSlice(Operation):
    """TF ``StridedSlice`` with begin/end/strides and the five masks (``StridedSlice.scala``).
    Input Table(x, begin, end, strides) or just x when the slice spec is given at construction."""

    def __init__(self, begin=None, end=None, strides=None, begin_mask=0, end_mask=0, ellipsis_mask=0,
                 new_axis_mask=0, shrink_axis_mask=0):
        super().__init__()
        self.begin, self.end, self.strides = begin, end, strides
        self.beginMask, self.endMask, self.ellipsisMask = begin_mask, end_mask, ellipsis_mask
        self.newAxisMask, self.shrinkAxisMask = new_axis_mask, shrink_axis_mask

    def updateOutput(self, t):
        if isinstance(t, Table):
            x = t[1]
            b, e, s = (t[i].flatten().tolist() for i in (2, 3, 4))
        else:
            x, b, e, s = t, list(self.begin), list(self.end), list(self.strides)
        idx, shrink = [], []
        d = 0
        for i in range(len(b)):
            if self.ellipsisMask >> i & 1:
                n_after = len(b) - i - 1
                while d < x.dim() - n_after:
                    idx.append(slice(None))
                    d += 1
                continue
            if self.newAxisMask >> i & 1:
                idx.append(None)
                continue
            if self.shrinkAxisMask >> i & 1:
                bi = b[i] + x.shape[d] if b[i] < 0 else b[i]
                idx.append(bi)
                d += 1
                continue
            st = s[i]
            bi = None if self.beginMask >> i & 1 else b[i]
            ei = None if self.endMask >> i & 1 else e[i]
            if st > 0:
                idx.append(slice(bi, ei, st))
            else:
                idx.append(("rev", bi, ei, st, d))
            d += 1
        out = x
        # apply positive-stride slices via indexing; negative strides via flip
        simple = [i if not isinstance(i, tuple) else slice(None) for i in idx]
        out = out[tuple(simple)]
        dim = 0
        for i in idx:
            if isinstance(i, tuple):
                _, bi, ei, st, _ = i
                n = out.shape[dim]
                bi = n - 1 if bi is None else (bi + n if bi < 0 else bi)
                ei = -1 if ei is None else (ei + n if ei < 0 else ei)
                sel = torch.arange(bi, ei, st)
                out = out.index_select(dim, sel)
            if not isinstance(i, int):
                dim += 1
        return out


class SplitAndSelect(Operation):
    """Split along 1-based ``dimension`` into ``numSplit`` parts and select ``index`` (1-based)."""

    def __init__(self, dimension, index, num_split):
        super().__init__()
        self.dimension, self.index, self.numSplit = dimension, index, num_split

    def updateOutput(self, x):
        return torch.chunk(x, self.numSplit, dim=self.dimension - 1)[self.index - 1].contiguous()


class Split(Operation):
    """TF ``Split``: Table(axis, x) → Table of ``num_split`` pieces."""

    def __init__(self, num_split):
        super().__init__()
        self.numSplit = num_split

    def updateOutput(self, t):
        axis, x = int(_scalar(t[1])), t[2]
        return Table(*[c.contiguous() for c in torch.chunk(x, self.numSplit, dim=axis)])


class BiasAdd(TensorModule):
    """TF ``BiasAdd`` on the last (NHWC) or channel (NCHW) dim with a trainable bias
    (``nn/tf/BiasAdd.scala``; the loader's Const-bias form)."""

    def __init__(self, bias: torch.Tensor = None, data_format="NHWC", size=None):
        super().__init__()
        b = bias if bias is not None else torch.zeros(size)
        self.format = data_format
        self.register_parameter("bias", torch.as_tensor(b, dtype=torch.float32).clone(), "gradBias")

    def _view(self, x):
        if self.format == "NCHW" and x.dim() == 4:
            return self.bias.view(1, -1, 1, 1)
        return self.bias

    def updateOutput(self, x):
        return x + self._view(x).to(x.dtype)

    def updateGradInput(self, x, gy):
        return gy

    def accGradParameters(self, x, gy):
        dims = [d for d in range(gy.dim()) if d != (1 if self.format == "NCHW" and gy.dim() == 4 else gy.dim() - 1)]
        self.gradBias.add_(gy.float().sum(dims).reshape(self.gradBias.shape))


# ------------------------------------------------------------------------------------------------ control flow
class SwitchOps(Operation):
    """Table(data, pred) → Table(false_out, true_out); the untaken branch is ``None`` (dead)."""

    def updateOutput(self, t):
        d, p = t[1], bool(_scalar(t[2]))
        return Table(None if p else d, d if p else None)


class MergeOps(Operation):
    """Forwards one of its inputs: the one the scheduler selected with ``setSwitch`` (1-based,
    ``ControlOps.scala`` MergeOps) or, when unset, the first live (non-None) input."""

    def __init__(self, switch: int = 0):
        super().__init__()
        self.switch = switch

    def setSwitch(self, s: int):
        self.switch = s
        return self

    def updateOutput(self, t):
        if self.switch and isinstance(t, Table):
            return t.get(self.switch)
        if self.switch == 1 and not isinstance(t, Table):
            return t
        vals = t.values() if isinstance(t, Table) else [t]
        for v in vals:
            if v is not None:
                return v
        return None


class Enter(Operation):
    def __init__(self, frame=""):
        super().__init__()
        self.frame = frame

    def updateOutput(self, x):
        return x


class Exit(Enter):
    pass


class NextIteration(Enter):
    """Carries a loop variable to the next iteration; copies it, since the producing module may
    overwrite its output buffer in that iteration."""

    def updateOutput(self, x):
        return x.clone() if isinstance(x, torch.Tensor) else x


class LoopCondition(Operation):
    def updateOutput(self, x):
        return x


# ------------------------------------------------------------------------------------------------ state
class Variable(TensorModule):
    """A trainable tensor source (``nn/tf/StateOps.scala`` Variable)."""

    def __init__(self, value: torch.Tensor, grad: torch.Tensor = None):
        super().__init__()
        self.register_parameter("weight", torch.as_tensor(value, dtype=torch.float32).clone(), "gradWeight")

    def updateOutput(self, input=None):
        return self.weight

    def updateGradInput(self, input, gy):
        return None

    def accGradParameters(self, input, gy):
        self.gradWeight.add_(gy.float())


class Assign(Operation):
    """Table(ref, value) → ref ← value (``StateOps.scala`` Assign)."""

    def __init__(self, validate_shape=True, use_locking=True):
        super().__init__()
        self.validateShape = validate_shape

    def updateOutput(self, t):
        ref, v = t[1], t[2]
        if self.validateShape and ref.shape != v.shape:
            raise ValueError(f"Assign: shape {tuple(v.shape)} != {tuple(ref.shape)}")
        if ref.shape != v.shape:
            ref.resize_(v.shape)
        ref.copy_(v)
        return ref


# ------------------------------------------------------------------------------------------------ NN ops
def _tf_pads(in_size, k, s, padding, dilation=1):
    if padding == "VALID":
        return 0, 0
    ek = (k - 1) * dilation + 1
    out = -(-in_size // s)
    total = max((out - 1) * s + ek - in_size, 0)
    return total // 2, total - total // 2


class Conv2D(Operation):
    """Table(x, filter [kh, kw, Cin, Cout]) with TF strides/padding/format (``nn/tf/NNOps.scala``)."""

    def __init__(self, strides=(1, 1, 1, 1), padding="SAME", data_format="NHWC", dilations=(1, 1, 1, 1)):
        super().__init__()
        self.strides, self.padding, self.format, self.dilations = list(strides), padding, data_format, list(dilations)

    def updateOutput(self, t):
        x, f = t[1], t[2]
        nhwc = self.format == "NHWC"
        xc = x.permute(0, 3, 1, 2) if nhwc else x
        sh, sw = (self.strides[1], self.strides[2]) if nhwc else (self.strides[2], self.strides[3])
        dh, dw = (self.dilations[1], self.dilations[2]) if nhwc else (self.dilations[2], self.dilations[3])
        kh, kw = f.shape[0], f.shape[1]
        pt, pb = _tf_pads(xc.shape[2], kh, sh, self.padding, dh)
        pl, pr = _tf_pads(xc.shape[3], kw, sw, self.padding, dw)
        xc = F.pad(xc.float(), (pl, pr, pt, pb))
        y = F.conv2d(xc, f.permute(3, 2, 0, 1).float(), None, (sh, sw), 0, (dh, dw)).to(x.dtype)
        return y.permute(0, 2, 3, 1).contiguous() if nhwc else y


class _Pool(Operation):
    def __init__(self, ksize, strides, padding="VALID", data_format="NHWC"):
        super().__init__()
        self.ksize, self.strides, self.padding, self.format = list(ksize), list(strides), padding, data_format

    def _geom(self, xc):
        nhwc = self.format == "NHWC"
        kh, kw = (self.ksize[1], self.ksize[2]) if nhwc else (self.ksize[2], self.ksize[3])
        sh, sw = (self.strides[1], self.strides[2]) if nhwc else (self.strides[2], self.strides[3])
        return kh, kw, sh, sw, _tf_pads(xc.shape[2], kh, sh, self.padding), _tf_pads(xc.shape[3], kw, sw, self.padding)

    def updateOutput(self, x):
        nhwc = self.format == "NHWC"
        xc = x.permute(0, 3, 1, 2) if nhwc else x
        y = self._pool(xc.float(), *self._geom(xc)).to(x.dtype)
        return y.permute(0, 2, 3, 1).contiguous() if nhwc else y


class MaxPool(_Pool):
    def _pool(self, xc, kh, kw, sh, sw, ph, pw):
        xc = F.pad(xc, (pw[0], pw[1], ph[0], ph[1]), value=-float("inf"))
        return F.max_pool2d(xc, (kh, kw), (sh, sw))


class AvgPool(_Pool):
    """TF AvgPool: padded cells are excluded from the mean."""

    def _pool(self, xc, kh, kw, sh, sw, ph, pw):
        ones = torch.ones_like(xc[:1, :1])
        pad = (pw[0], pw[1], ph[0], ph[1])
        s = F.avg_pool2d(F.pad(xc, pad), (kh, kw), (sh, sw), divisor_override=1)
        c = F.avg_pool2d(F.pad(ones, pad), (kh, kw), (sh, sw), divisor_override=1)
        return s / c


class LRN(Operation):
    """TF local response normalisation over the last (channel) dim."""

    def __init__(self, depth_radius=5, bias=1.0, alpha=1.0, beta=0.5):
        super().__init__()
        self.depthRadius, self.bias, self.alpha, self.beta = depth_radius, bias, alpha, beta

    def updateOutput(self, x):
        sq = (x.float() ** 2).permute(0, 3, 1, 2).unsqueeze(1)
        r = self.depthRadius
        s = F.avg_pool3d(F.pad(sq, (0, 0, 0, 0, r, r)), (2 * r + 1, 1, 1), 1, divisor_override=1)[:, 0]
        return (x.float() / (self.bias + self.alpha * s.permute(0, 2, 3, 1)) ** self.beta).to(x.dtype)


class FusedBatchNorm(Operation):
    """Inference ``FusedBatchNorm``: Table(x, scale, offset, mean, variance) → Table(y, mean, var)."""

    def __init__(self, epsilon=1e-3, data_format="NHWC", is_training=False):
        super().__init__()
        self.epsilon, self.format, self.isTraining = epsilon, data_format, is_training

    def updateOutput(self, t):
        x, sc, off, mean, var = (t[i] for i in range(1, 6))
        shape = (1, -1, 1, 1) if self.format == "NCHW" else (1, 1, 1, -1)
        xf = x.float()
        if self.isTraining or mean.numel() == 0:
            dims = (0, 2, 3) if self.format == "NCHW" else (0, 1, 2)
            mean = xf.mean(dims)
            var = xf.var(dims, unbiased=False)
        y = (xf - mean.view(shape)) * torch.rsqrt(var.view(shape) + self.epsilon) * sc.view(shape) + off.view(shape)
        return Table(y.to(x.dtype), mean, var)


# ------------------------------------------------------------------------------------------------ parsing / image
class ParseExample(Operation):
    """Parse serialised ``tf.train.Example`` records into dense tensors (``ParsingOps.scala``).
    ``keys``/``types``/``shapes`` name the dense features; input: a list of serialised bytes."""

    def __init__(self, keys: Sequence[str], types: Sequence[torch.dtype], shapes: Sequence[Sequence[int]]):
        super().__init__()
        self.keys, self.types, self.shapes = list(keys), list(types), [list(s) for s in shapes]

    def updateOutput(self, records):
        from ...utils.tf.proto import example_classes
        Example = example_classes()["tensorflow.Example"]
        cols = [[] for _ in self.keys]
        if isinstance(records, Table):
            vals = records.values()
            records = vals[0] if isinstance(vals[0], (list, tuple)) else [v for v in vals if isinstance(v, bytes)]
        for r in records:
            ex = Example.FromString(r)
            for j, k in enumerate(self.keys):
                f = ex.features.feature[k]
                kind = f.WhichOneof("kind")
                vals = list(getattr(f, kind).value) if kind else []
                if kind == "bytes_list":
                    cols[j].append(vals)
                else:
                    cols[j].append(torch.tensor(vals, dtype=self.types[j]).reshape(self.shapes[j] or [-1]))
        return Table(*[torch.stack(c) if c and isinstance(c[0], torch.Tensor) else c for c in cols])


class DecodeImage(Operation):
    """Decode encoded image bytes (JPEG/PNG/BMP/GIF) to uint8 HWC (``nn/tf/ImageOps.scala``)."""

    def __init__(self, channels=3):
        super().__init__()
        self.channels = channels

    def updateOutput(self, data):
        from PIL import Image
        if isinstance(data, torch.Tensor):
            data = bytes(data.to(torch.uint8).tolist())
        im = Image.open(io.BytesIO(data))
        im = im.convert({1: "L", 3: "RGB", 4: "RGBA"}.get(self.channels, "RGB"))
        arr = np.asarray(im, dtype=np.uint8)
        if arr.ndim == 2:
            arr = arr[:, :, None]
        return torch.from_numpy(arr.copy())


DecodeJpeg = DecodePng = DecodeBmp = DecodeGif = DecodeImage


class DecodeRaw(Operation):
    def __init__(self, out_type=torch.uint8, little_endian=True):
        super().__init__()
        self.outType, self.littleEndian = out_type, little_endian

    def updateOutput(self, data):
        np_t = {torch.uint8: np.uint8, torch.int8: np.int8, torch.int16: np.int16, torch.int32: np.int32,
                torch.int64: np.int64, torch.float32: np.float32, torch.float64: np.float64}[self.outType]
        dt = np.dtype(np_t).newbyteorder("<" if self.littleEndian else ">")
        return torch.from_numpy(np.frombuffer(data, dtype=dt).astype(np_t))


__all__ = [n for n, v in list(globals().items()) if isinstance(v, type) and issubclass(v, AbstractModule)
           and v.__module__ == __name__]

from .grad_ops import *  # noqa: E402,F401,F403  (TF backward / training-graph ops)
from . import grad_ops as _grad_ops  # noqa: E402
__all__ += _grad_ops.__all__


# data-flow resources (TensorArray / Stack) and AssignGrad: DataFlowOps.scala, StateOps.scala
from .data_flow import (TensorArray, TensorArrayCreator, TensorArrayGrad, TensorArrayWrite, TensorArrayRead,  # noqa: E402,F401
                        TensorArrayGather, TensorArrayScatter, TensorArrayConcat, TensorArraySplit, TensorArraySize,
                        TensorArrayClose, StackCreator, StackPush, StackPop, AssignGrad)


def _set_scala_package():
    """The TF op layers live in ``com.intel.analytics.bigdl.nn.tf`` (their .bigdl module type)."""
    for _v in list(globals().values()):
        if (isinstance(_v, type) and issubclass(_v, AbstractModule) and _v.__module__.startswith(__name__)
                and "SCALA_PACKAGE" not in _v.__dict__):
            _v.SCALA_PACKAGE = "com.intel.analytics.bigdl.nn.tf"


_set_scala_package()
