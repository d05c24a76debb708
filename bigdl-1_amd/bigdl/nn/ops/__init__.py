"""TensorFlow-style operation layers (``DL/nn/ops/*.scala``, 71 files).

An ``Operation`` (``DL/nn/ops/Operation.scala``) is a forward-only module: ``updateGradInput`` /
``accGradParameters`` raise.  Multi-input ops take a ``Table`` of tensors in TF input order; index
semantics follow TensorFlow (0-based axes and indices) except where the reference documents a
``startIndex`` / ``startFromZero`` switch.  Everything runs with torch ops on the tensors' device.
"""
from __future__ import annotations

import hashlib
import math
from typing import List, Sequence

import torch
import torch.nn.functional as F

from ...utils.table import Table
from ..abstractnn import AbstractModule


def _in(input, i):
    return input[i] if isinstance(input, Table) else (input if i == 1 else None)


def _strings(x):
    """Normalise a string batch (list, or the Table ``forward`` makes of a list) to a list."""
    if isinstance(x, Table):
        vals = x.values()
        if vals and isinstance(vals[0], (list, tuple)):
            return list(vals[0])
        return [v for v in vals if isinstance(v, str)]
    if isinstance(x, str):
        return [x]
    return list(x)


def _scalar(t):
    return t.item() if isinstance(t, torch.Tensor) else t


class Operation(AbstractModule):
    """Forward-only op (``Operation.scala:31``)."""

    def updateGradInput(self, input, gradOutput):
        raise NotImplementedError(f"{type(self).__name__}: operation does not support backward")

    def accGradParameters(self, input, gradOutput):
        raise NotImplementedError(f"{type(self).__name__}: operation does not support backward")

    def backward(self, input, gradOutput):
        return self.updateGradInput(input, gradOutput)


class ModuleToOperation(Operation):
    """Wrap a module as a forward-only op (``ModuleToOperation.scala``)."""

    def __init__(self, module):
        super().__init__()
        self.module = module

    def updateOutput(self, input):
        return self.module.forward(input)


class TensorOp(Operation):
    """Composable elementwise tensor transform (``TensorOp.scala``): ``TensorOp().exp().mul(2)``."""

    def __init__(self, fns=None):
        super().__init__()
        self.fns = list(fns or [])

    def _chain(self, fn):
        return TensorOp(self.fns + [fn])

    def __getattr__(self, name):
        if name.startswith("_") or name in ("fns",):
            raise AttributeError(name)
        tf = getattr(torch, name, None)
        if tf is None:
            raise AttributeError(name)

        def build(*args):
            return self._chain(lambda x: tf(x, *args))
        return build

    def updateOutput(self, input):
        y = input
        for f in self.fns:
            y = f(y)
        return y


# ------------------------------------------------------------------------------------------------ unary
def _unary(name, fn, doc=""):
    cls = type(name, (Operation,), {"updateOutput": lambda self, x: fn(x),
                                    "__doc__": doc or f"Elementwise ``{name}`` (``ops/{name}.scala``)."})
    return cls


Ceil = _unary("Ceil", torch.ceil)
Floor = _unary("Floor", torch.floor)
Exp = _unary("Exp", torch.exp)
Expm1 = _unary("Expm1", torch.expm1)
Erf = _unary("Erf", torch.erf)
Erfc = _unary("Erfc", torch.erfc)
Digamma = _unary("Digamma", torch.digamma)
Lgamma = _unary("Lgamma", torch.lgamma)
Inv = _unary("Inv", torch.reciprocal)
IsFinite = _unary("IsFinite", torch.isfinite)
IsInf = _unary("IsInf", torch.isinf)
IsNan = _unary("IsNan", torch.isnan)
Rint = _unary("Rint", torch.round)  # round-half-to-even, as TF Rint
Sign = _unary("Sign", torch.sign)
LogicalNot = _unary("LogicalNot", torch.logical_not)
Log1p = _unary("Log1p", torch.log1p)


class Round(Operation):
    """TF ``Round``: banker's rounding (``Round.scala``)."""

    def updateOutput(self, x):
        return torch.round(x)


class Cast(Operation):
    """``Cast.scala``: convert to ``dtype`` (a torch dtype or its name)."""

    def __init__(self, dtype=torch.float32):
        super().__init__()
        self.dtype = getattr(torch, dtype) if isinstance(dtype, str) else dtype

    def updateOutput(self, x):
        return x.to(self.dtype)


class Rank(Operation):
    def updateOutput(self, x):
        return torch.tensor(x.dim(), dtype=torch.int32)


class L2Loss(Operation):
    """``sum(x²) / 2`` (``L2Loss.scala``)."""

    def updateOutput(self, x):
        return (x.float() ** 2).sum().div(2).reshape(1).to(x.dtype)


# ------------------------------------------------------------------------------------------------ binary
def _binary(name, fn, doc=""):
    cls = type(name, (Operation,), {"updateOutput": lambda self, t: fn(t[1], t[2]),
                                    "__doc__": doc or f"Broadcasting ``{name}`` (``ops/{name}.scala``)."})
    return cls


Equal = _binary("Equal", torch.eq)
NotEqual = _binary("NotEqual", torch.ne)
Greater = _binary("Greater", torch.gt)
GreaterEqual = _binary("GreaterEqual", torch.ge)
Less = _binary("Less", torch.lt)
LessEqual = _binary("LessEqual", torch.le)
LogicalAnd = _binary("LogicalAnd", torch.logical_and)
LogicalOr = _binary("LogicalOr", torch.logical_or)
Maximum = _binary("Maximum", torch.maximum)
Minimum = _binary("Minimum", torch.minimum)
Pow = _binary("Pow", torch.pow)
SquaredDifference = _binary("SquaredDifference", lambda a, b: (a - b) * (a - b))
FloorDiv = _binary("FloorDiv", lambda a, b: torch.div(a, b, rounding_mode="floor"))
TruncateDiv = _binary("TruncateDiv", lambda a, b: torch.div(a, b, rounding_mode="trunc"))
FloorMod = _binary("FloorMod", torch.remainder)
Mod = _binary("Mod", torch.fmod, "C-style remainder (sign of the dividend), ``Mod.scala``.")


class ApproximateEqual(Operation):
    def __init__(self, tolerance=1e-5):
        super().__init__()
        self.tolerance = tolerance

    def updateOutput(self, t):
        return (t[1] - t[2]).abs() < self.tolerance


class Compare(Operation):
    """Generic comparison by name (``Compare.scala``)."""

    _OPS = {"eq": torch.eq, "ne": torch.ne, "gt": torch.gt, "ge": torch.ge, "lt": torch.lt, "le": torch.le}

    def __init__(self, op="eq"):
        super().__init__()
        self.op = op

    def updateOutput(self, t):
        return self._OPS[self.op](t[1], t[2])


# ------------------------------------------------------------------------------------------------ reductions
def _axes(t, ndim, start_from_zero=True):
    ax = [int(v) for v in torch.as_tensor(t).flatten().tolist()]
    if not start_from_zero:
        ax = [a - 1 for a in ax]
    return tuple(a + ndim if a < 0 else a for a in ax)


class _Reduce(Operation):
    _fn = None

    def __init__(self, keep_dims=False, start_from_zero=True):
        super().__init__()
        self.keepDims, self.startFromZero = keep_dims, start_from_zero

    def updateOutput(self, t):
        x, axes = t[1], _axes(t[2], t[1].dim(), self.startFromZero)
        if not axes:
            return x.clone()
        return type(self)._fn(x, axes, self.keepDims)


class Sum(_Reduce):
    """``Sum.scala``: Table(x, axes) → sum over axes (``startFromZero`` picks 0/1-based axes)."""
    _fn = staticmethod(lambda x, a, k: x.sum(dim=a, keepdim=k))


class Max(_Reduce):
    _fn = staticmethod(lambda x, a, k: x.amax(dim=a, keepdim=k))


class Prod(Operation):
    """``Prod.scala``: product along a 1-based ``dimension`` (negative counts from the end)."""

    def __init__(self, dimension=1, keep_dim=False):
        super().__init__()
        self.dimension, self.keepDim = dimension, keep_dim

    def updateOutput(self, x):
        d = self.dimension - 1 if self.dimension > 0 else x.dim() + self.dimension
        return x.prod(dim=d, keepdim=self.keepDim)


class All(Operation):
    def __init__(self, keep_dims=False, start_from_zero=True):
        super().__init__()
        self.keepDims, self.startFromZero = keep_dims, start_from_zero

    def updateOutput(self, t):
        x = t[1].bool()
        for a in sorted(_axes(t[2], x.dim(), self.startFromZero), reverse=True):
            x = x.all(dim=a, keepdim=self.keepDims)
        return x


class Any(All):
    def updateOutput(self, t):
        x = t[1].bool()
        for a in sorted(_axes(t[2], x.dim(), self.startFromZero), reverse=True):
            x = x.any(dim=a, keepdim=self.keepDims)
        return x


class ArgMax(Operation):
    """Table(x, axis) → 0-based argmax along TF ``axis`` (``ArgMax.scala``)."""

    def updateOutput(self, t):
        return t[1].argmax(dim=int(_scalar(t[2]))).to(torch.int32)


class TopK(Operation):
    """``TopK.scala``: values and ``startIndex``-based indices of the k largest on the last dim."""

    def __init__(self, k, sorted=True, start_index=1):
        super().__init__()
        self.k, self.sorted, self.startIndex = k, sorted, start_index

    def updateOutput(self, x):
        v, i = torch.topk(x, self.k, dim=-1, largest=True, sorted=self.sorted)
        return Table(v, (i + self.startIndex).to(torch.int32))


class InTopK(Operation):
    """Table(predictions [B, C], targets [B]) → bool [B] (``InTopK.scala``)."""

    def __init__(self, k, start_from_zero=False):
        super().__init__()
        self.k, self.startFromZero = k, start_from_zero

    def updateOutput(self, t):
        pred, tgt = t[1], t[2].long()
        if not self.startFromZero:
            tgt = tgt - 1
        top = torch.topk(pred, self.k, dim=-1).indices
        return (top == tgt.unsqueeze(-1)).any(-1)


class SegmentSum(Operation):
    """Table(data, sorted 0-based segment ids) → per-segment sums (``SegmentSum.scala``)."""

    def updateOutput(self, t):
        x, ids = t[1], t[2].long()
        n = int(ids[-1]) + 1
        out = x.new_zeros((n,) + tuple(x.shape[1:]))
        return out.index_add_(0, ids, x)


# ------------------------------------------------------------------------------------------------ shape / index
class Gather(Operation):
    """Table(params, 0-based indices[, axis]) → gathered slices (``Gather.scala``)."""

    def updateOutput(self, t):
        x, idx = t[1], t[2].long()
        axis = int(_scalar(t[3])) if isinstance(t, Table) and len(t) > 2 else 0
        axis = axis + x.dim() if axis < 0 else axis
        out = torch.index_select(x, axis, idx.flatten())
        return out.reshape(tuple(x.shape[:axis]) + tuple(idx.shape) + tuple(x.shape[axis + 1:]))


class OneHot(Operation):
    """Table(indices, depth, on_value, off_value) → one-hot along ``axis`` (``OneHot.scala``)."""

    def __init__(self, axis=-1):
        super().__init__()
        self.axis = axis

    def updateOutput(self, t):
        idx, depth = t[1].long(), int(_scalar(t[2]))
        on, off = _scalar(t[3]), _scalar(t[4])
        valid = (idx >= 0) & (idx < depth)
        oh = F.one_hot(idx.clamp(0, depth - 1), depth).bool() & valid.unsqueeze(-1)
        out = torch.where(oh, torch.tensor(on, dtype=torch.float32), torch.tensor(off, dtype=torch.float32))
        if self.axis != -1:
            out = out.movedim(-1, self.axis)
        dt = t[3].dtype if isinstance(t[3], torch.Tensor) else torch.float32
        return out.to(dt)


class Pad(Operation):
    """Table(x, paddings [ndim, 2]) → constant pad (``Pad.scala``)."""

    def __init__(self, mode="CONSTANT", constant_value=0.0):
        super().__init__()
        self.mode, self.constantValue = mode, constant_value

    def updateOutput(self, t):
        x, p = t[1], t[2].long().tolist()
        flat = []
        for before, after in reversed(p):
            flat += [before, after]
        if self.mode.upper() == "CONSTANT":
            return F.pad(x, flat, value=self.constantValue)
        mode = {"REFLECT": "reflect", "SYMMETRIC": "replicate"}[self.mode.upper()]
        return F.pad(x.unsqueeze(0).float(), flat[:-2] if len(p) == x.dim() else flat, mode=mode)[0].to(x.dtype)


class Slice(Operation):
    """``Slice.scala``: 0-based ``begin`` and ``size`` (−1 = to the end)."""

    def __init__(self, begin: Sequence[int], size: Sequence[int]):
        super().__init__()
        self.begin, self.size = list(begin), list(size)

    def updateOutput(self, x):
        y = x
        for d, (b, s) in enumerate(zip(self.begin, self.size)):
            y = y.narrow(d, b, (x.shape[d] - b) if s == -1 else s)
        return y.contiguous()


class Tile(Operation):
    """Table(x, multiples) → ``x.repeat(multiples)`` (``Tile.scala``)."""

    def updateOutput(self, t):
        reps = [int(v) for v in t[2].flatten().tolist()]
        x = torch.as_tensor(t[1])
        return x.repeat(*reps) if reps else x.clone()  # a scalar tiles to itself


class Select(Operation):
    """Table(cond, t, e) → ``where(cond, t, e)``; a scalar cond picks a whole input (``Select.scala``)."""

    def updateOutput(self, t):
        c = t[1]
        if c.numel() == 1:
            return t[2] if bool(c) else t[3]
        return torch.where(c.bool().view(c.shape + (1,) * (t[2].dim() - c.dim())), t[2], t[3])


class RangeOps(Operation):
    """Table(start, limit, delta) → ``arange`` (``RangeOps.scala``)."""

    def updateOutput(self, t):
        s, l, d = _scalar(t[1]), _scalar(t[2]), _scalar(t[3])
        dt = t[1].dtype if isinstance(t[1], torch.Tensor) else torch.float32
        return torch.arange(s, l, d, dtype=dt)


class BatchMatMul(Operation):
    """``BatchMatMul.scala``: batched matmul with optional adjoints on the last two dims."""

    def __init__(self, adj_x=False, adj_y=False):
        super().__init__()
        self.adjX, self.adjY = adj_x, adj_y

    def updateOutput(self, t):
        x, y = t[1], t[2]
        if self.adjX:
            x = x.transpose(-1, -2)
        if self.adjY:
            y = y.transpose(-1, -2)
        return torch.matmul(x, y)


class CrossEntropy(Operation):
    """Table(logits, labels one-hot/probabilities) → Table(loss per row, grad) (``CrossEntropy.scala``)."""

    def updateOutput(self, t):
        logits, labels = t[1].float(), t[2].float()
        lsm = torch.log_softmax(logits, -1)
        loss = -(labels * lsm).sum(-1)
        grad = torch.softmax(logits, -1) - labels
        return Table(loss, grad)


class DepthwiseConv2D(Operation):
    """TF depthwise conv (``DepthwiseConv2D.scala``): Table(x, filter [kh, kw, C, M]) with
    ``stride``/``pad`` and NHWC/NCHW ``format``."""

    def __init__(self, stride_w=1, stride_h=1, pad_w=0, pad_h=0, data_format="NHWC"):
        super().__init__()
        self.strideW, self.strideH, self.padW, self.padH, self.format = stride_w, stride_h, pad_w, pad_h, data_format

    def updateOutput(self, t):
        x, f = t[1], t[2]
        if self.format == "NHWC":
            x = x.permute(0, 3, 1, 2)
        kh, kw, C, M = f.shape
        w = f.permute(2, 3, 0, 1).reshape(C * M, 1, kh, kw)
        pad = (self.padH, self.padW) if self.padH >= 0 else "same"
        y = F.conv2d(x.float(), w.float(), None, (self.strideH, self.strideW), pad, groups=C).to(x.dtype)
        return y.permute(0, 2, 3, 1).contiguous() if self.format == "NHWC" else y


class Dilation2D(Operation):
    """Grayscale morphological dilation (``Dilation2D.scala``): Table(x NHWC, filter [kh, kw, C])."""

    def __init__(self, strides=(1, 1, 1, 1), rates=(1, 1, 1, 1), padding="VALID"):
        super().__init__()
        self.strides, self.rates, self.padding = list(strides), list(rates), padding.upper()

    def updateOutput(self, t):
        x, f = t[1].float(), t[2].float()
        N, H, W, C = x.shape
        kh, kw, _ = f.shape
        sh, sw = self.strides[1], self.strides[2]
        rh, rw = self.rates[1], self.rates[2]
        ekh, ekw = (kh - 1) * rh + 1, (kw - 1) * rw + 1
        if self.padding == "SAME":
            oh, ow = -(-H // sh), -(-W // sw)
            ph = max((oh - 1) * sh + ekh - H, 0)
            pw = max((ow - 1) * sw + ekw - W, 0)
            x = F.pad(x, (0, 0, pw // 2, pw - pw // 2, ph // 2, ph - ph // 2), value=-float("inf"))
        xc = x.permute(0, 3, 1, 2)
        cols = F.unfold(xc, (kh, kw), dilation=(rh, rw), stride=(sh, sw))  # N, C·kh·kw, L
        Lh = (xc.shape[2] - ekh) // sh + 1
        Lw = (xc.shape[3] - ekw) // sw + 1
        cols = cols.view(N, C, kh * kw, Lh, Lw) + f.permute(2, 0, 1).reshape(1, C, kh * kw, 1, 1)
        return cols.amax(2).permute(0, 2, 3, 1).contiguous()


class ResizeBilinearOps(Operation):
    """Table(images NHWC, size [2]) → bilinear resize (``ResizeBilinear.scala``)."""

    def __init__(self, align_corner=False):
        super().__init__()
        self.alignCorner = align_corner

    def updateOutput(self, t):
        from ...ops.reference import resize_bilinear
        x, size = t[1], [int(v) for v in t[2].flatten().tolist()]
        y = resize_bilinear(x.permute(0, 3, 1, 2).float(), size[0], size[1], self.alignCorner)
        return y.permute(0, 2, 3, 1).contiguous().to(x.dtype if x.is_floating_point() else torch.float32)


ResizeBilinear = ResizeBilinearOps


class RandomUniform(Operation):
    """``RandomUniform.scala``: shape tensor → U[minVal, maxVal)."""

    is_random = True  # never memoised as a const node by the dynamic-graph scheduler

    def __init__(self, min_val=0.0, max_val=1.0, seed=None):
        super().__init__()
        self.minVal, self.maxVal, self.seed = min_val, max_val, seed

    def updateOutput(self, shape):
        g = torch.Generator().manual_seed(self.seed) if self.seed is not None else None
        s = [int(v) for v in shape.flatten().tolist()]
        return torch.rand(s, generator=g) * (self.maxVal - self.minVal) + self.minVal


class TruncatedNormal(Operation):
    """``TruncatedNormal.scala``: normal(mean, stddev) re-drawn outside 2σ."""

    is_random = True

    def __init__(self, mean=0.0, stddev=1.0, seed=None):
        super().__init__()
        self.mean, self.stddev, self.seed = mean, stddev, seed

    def updateOutput(self, shape):
        s = [int(v) for v in shape.flatten().tolist()]
        out = torch.empty(s)
        torch.nn.init.trunc_normal_(out, self.mean, self.stddev, self.mean - 2 * self.stddev,
                                    self.mean + 2 * self.stddev)
        return out


# ------------------------------------------------------------------------------------------------ feature columns
class BucketizedCol(Operation):
    """``BucketizedCol.scala``: bucket ids of numeric values given sorted ``boundaries``."""

    def __init__(self, boundaries: Sequence[float]):
        super().__init__()
        self.boundaries = torch.tensor(sorted(boundaries), dtype=torch.float64)

    def updateOutput(self, x):
        return torch.bucketize(x.double(), self.boundaries, right=True).to(torch.int32)


def _hash_bucket(s: str, n: int) -> int:
    """Scala ``MurmurHash3.stringHash(s) % n`` made non-negative (``HashFunc.stringHashBucket32``)."""
    from ...utils.hash_func import stringHashBucket32
    return stringHashBucket32(s, n)


class CategoricalColHashBucket(Operation):
    """Strings (comma-joined multi-values) → hash bucket ids, as a sparse (indices, values, shape)
    Table or a dense [B, maxLen] tensor padded with −1 (``CategoricalColHashBucket.scala``)."""

    def __init__(self, hash_bucket_size, str_delimiter=",", is_sparse=True):
        super().__init__()
        self.hashBucketSize, self.strDelimiter, self.isSparse = hash_bucket_size, str_delimiter, is_sparse

    def _ids(self, strings):
        return [[_hash_bucket(v, self.hashBucketSize) for v in s.split(self.strDelimiter) if v != ""]
                for s in strings]

    def updateOutput(self, strings: List[str]):
        return _sparse_or_dense(self._ids(_strings(strings)), self.isSparse)


class CategoricalColVocaList(Operation):
    """Strings → vocabulary ids; out-of-vocabulary → ``numOovBuckets`` hash buckets or −1/default
    (``CategoricalColVocaList.scala``)."""

    def __init__(self, voca_list, str_delimiter=",", is_set_default=False, num_oov_buckets=0):
        super().__init__()
        self.vocaList = list(voca_list)
        self.index = {v: i for i, v in enumerate(self.vocaList)}
        self.strDelimiter, self.isSetDefault, self.numOovBuckets = str_delimiter, is_set_default, num_oov_buckets

    def updateOutput(self, strings: List[str]):
        n = len(self.vocaList)
        rows = []
        for s in _strings(strings):
            r = []
            for v in s.split(self.strDelimiter):
                if v in self.index:
                    r.append(self.index[v])
                elif self.numOovBuckets > 0:
                    r.append(n + _hash_bucket(v, self.numOovBuckets))
                elif self.isSetDefault:
                    r.append(n)
            rows.append(r)
        return _sparse_or_dense(rows, True)


def _sparse_or_dense(rows, sparse):
    if sparse:
        idx = [[i, j] for i, r in enumerate(rows) for j in range(len(r))]
        vals = [v for r in rows for v in r]
        width = max((len(r) for r in rows), default=0)
        return Table(torch.tensor(idx, dtype=torch.long).reshape(-1, 2), torch.tensor(vals, dtype=torch.int32),
                     torch.tensor([len(rows), width]))
    width = max((len(r) for r in rows), default=0)
    out = torch.full((len(rows), width), -1, dtype=torch.int32)
    for i, r in enumerate(rows):
        out[i, :len(r)] = torch.tensor(r, dtype=torch.int32)
    return out


class CrossCol(Operation):
    """Cross of several string columns hashed into ``hashBucketSize`` (``CrossCol.scala``)."""

    def __init__(self, hash_bucket_size, str_delimiter=","):
        super().__init__()
        self.hashBucketSize, self.strDelimiter = hash_bucket_size, str_delimiter

    def updateOutput(self, cols):
        cols = [cols[i + 1] for i in range(len(cols))] if isinstance(cols, Table) else list(cols)
        from ...utils.hash_func import string_hash
        rows = []
        for vals in zip(*cols):
            parts = [str(v).split(self.strDelimiter) for v in vals]
            rows.append([self._bucket(c, string_hash) for c in self._recombine(parts)])
        return _sparse_or_dense(rows, True)

    @staticmethod
    def _recombine(parts):
        """The reference's stack-based cartesian product order (``CrossCol.reCombine``): every level
        but the last is visited in reverse, the last in order."""
        out = []

        def rec(prefix, lvl):
            if lvl == len(parts) - 1:
                out.extend(prefix + [x] for x in parts[lvl])
                return
            for x in reversed(parts[lvl]):
                rec(prefix + [x], lvl + 1)
        rec([], 0)
        return out

    def _bucket(self, combo, string_hash):
        h = string_hash(combo[0])
        for s in combo[1:]:
            h = string_hash(s, h & 0xFFFFFFFF)
        r = int(h - self.hashBucketSize * int(h / self.hashBucketSize))
        return r + self.hashBucketSize if r < 0 else r


class IndicatorCol(Operation):
    """Sparse ids → multi-hot [B, feaLen] (``IndicatorCol.scala``)."""

    def __init__(self, fea_len, is_count=True):
        super().__init__()
        self.feaLen, self.isCount = fea_len, is_count

    def updateOutput(self, sp):
        idx, vals, shape = sp[1], sp[2].long(), sp[3]
        out = torch.zeros(int(shape[0]), self.feaLen)
        out.index_put_((idx[:, 0], vals), torch.ones(vals.numel()), accumulate=self.isCount)
        return out.clamp_max(1) if not self.isCount else out


class Kv2Tensor(Operation):
    """"k:v,k:v" strings → dense [B, feaLen] or sparse (``Kv2Tensor.scala``)."""

    def __init__(self, kv_delimiter=",", item_delimiter=":", trans_type=0, fea_len=0):
        super().__init__()
        self.kvDelimiter, self.itemDelimiter, self.transType, self.feaLen = kv_delimiter, item_delimiter, \
            trans_type, fea_len

    def updateOutput(self, t):
        strings = _strings(t)
        fea_len = self.feaLen
        if isinstance(t, Table) and len(t) > 1 and isinstance(t[2], torch.Tensor):
            fea_len = int(_scalar(t[2]))
        out = torch.zeros(len(strings), fea_len)
        for i, s in enumerate(strings):
            for kv in s.split(self.kvDelimiter):
                if kv:
                    k, v = kv.split(self.itemDelimiter)
                    out[i, int(k)] = float(v)
        if self.transType == 1:
            nz = out.nonzero()
            return Table(nz, out[nz[:, 0], nz[:, 1]], torch.tensor(list(out.shape)))
        return out


class MkString(Operation):
    """Sparse row → delimited string (``MkString.scala``)."""

    def __init__(self, str_delimiter=","):
        super().__init__()
        self.strDelimiter = str_delimiter

    def updateOutput(self, sp):
        idx, vals, shape = sp[1], sp[2], sp[3]
        rows = [[] for _ in range(int(shape[0]))]
        for (r, _), v in zip(idx.tolist(), vals.tolist()):
            rows[r].append(str(v))
        return [self.strDelimiter.join(r) for r in rows]


class Substr(Operation):
    """Table(strings, pos, len) → substrings (``Substr.scala``)."""

    def updateOutput(self, t):
        strings, pos, ln = t[1], int(_scalar(t[2])), int(_scalar(t[3]))
        if isinstance(strings, str):
            return strings[pos:pos + ln]
        return [s[pos:pos + ln] for s in strings]


__all__ = [n for n, v in list(globals().items()) if isinstance(v, type) and issubclass(v, Operation)]
