"""Torch7-style Tensor facade over a torch device tensor.

Reference: ``trait Tensor[T]`` (``DL/tensor/Tensor.scala:37-807``), ``DenseTensor.scala`` (``select``
407, ``narrow`` 442), ``TensorMath.scala:38-829``, factory ``object Tensor`` (``:853-1400``).
Semantics kept: dimensions and element indices are 1-based, ``storageOffset`` is 1-based,
in-place methods return ``self``, reductions with a dim return ``(values, 1-based indices)``.
The storage is a torch tensor (HBM when on the GPU), so a facade wraps — never copies — data
flowing in and out of modules (``.data``).
"""
from __future__ import annotations

from typing import Sequence

import numpy as np
import torch

from ..utils.random import RNG
from ..ops import vml as _vml


def _dim0(d: int, nd: int) -> int:
    if d < 0:
        return nd + d
    if d < 1 or d > nd:
        raise IndexError(f"dimension {d} out of range [1, {nd}]")
    return d - 1


_VML_UNARY = {torch.abs: "abs", torch.exp: "exp", torch.log: "log", torch.log1p: "log1p", torch.sqrt: "sqrt",
              torch.tanh: "tanh", torch.sigmoid: "sigmoid", torch.neg: "neg", torch.reciprocal: "inv"}


def _unwrap(x):
    return x.data if isinstance(x, Tensor) else x


class Tensor:
    __slots__ = ("data",)

    def __init__(self, *args, dtype=torch.float32, device=None):
        if len(args) == 1 and isinstance(args[0], torch.Tensor):
            self.data = args[0]
        elif len(args) == 1 and isinstance(args[0], np.ndarray):
            self.data = torch.from_numpy(np.ascontiguousarray(args[0]))
        elif len(args) == 1 and isinstance(args[0], Tensor):
            self.data = args[0].data
        elif len(args) == 1 and isinstance(args[0], (list, tuple)) and args[0] and isinstance(args[0][0], (list, tuple, float)):
            self.data = torch.tensor(args[0], dtype=dtype, device=device)
        elif len(args) == 1 and isinstance(args[0], (list, tuple)):
            self.data = torch.zeros(*args[0], dtype=dtype, device=device)
        elif args:
            self.data = torch.zeros(*[int(a) for a in args], dtype=dtype, device=device)
        else:
            self.data = torch.empty(0, dtype=dtype, device=device)

    # ---- factories (object Tensor) -------------------------------------------------------
    @staticmethod
    def apply(*sizes, dtype=torch.float32):
        return Tensor(*sizes, dtype=dtype)

    @staticmethod
    def scalar(v, dtype=torch.float32):
        return Tensor(torch.tensor(v, dtype=dtype))

    @staticmethod
    def ones(*sizes):
        return Tensor(torch.ones(*sizes))

    @staticmethod
    def zeros(*sizes):
        return Tensor(torch.zeros(*sizes))

    @staticmethod
    def range(xmin, xmax, step=1):
        return Tensor(torch.arange(xmin, xmax + (1e-9 if step > 0 else -1e-9), step, dtype=torch.float32))

    @staticmethod
    def randperm(n):
        return Tensor(torch.from_numpy(RNG.permutation(n) + 1).float())

    @staticmethod
    def gaussian1D(size=3, sigma=0.25, amplitude=1, normalize=False, mean=0.5, tensor=None):
        center = mean * size + 0.5
        i = torch.arange(1, size + 1, dtype=torch.float32)
        g = amplitude * torch.exp(-((i - center) / (sigma * size)) ** 2 / 2)
        if normalize:
            g = g / g.sum()
        return Tensor(g)

    @staticmethod
    def sparse(indices, values, shape):
        return Tensor(torch.sparse_coo_tensor(torch.as_tensor(indices) - 1, torch.as_tensor(values), tuple(shape)))

    @staticmethod
    def dense(sparse: "Tensor"):
        return Tensor(sparse.data.to_dense())

    @staticmethod
    def unique(t: "Tensor"):
        u, inv = torch.unique(t.data, return_inverse=True)
        return Tensor(u), Tensor((inv + 1).float())

    # ---- shape / storage ------------------------------------------------------------------------
    def nDimension(self) -> int:
        return self.data.dim()

    dim = nDimension

    def size(self, dim: int | None = None):
        if dim is None:
            return list(self.data.shape)
        return self.data.shape[_dim0(dim, self.data.dim())]

    def stride(self, dim: int | None = None):
        if dim is None:
            return list(self.data.stride())
        return self.data.stride(_dim0(dim, self.data.dim()))

    def nElement(self) -> int:
        return self.data.numel()

    def storageOffset(self) -> int:
        return self.data.storage_offset() + 1

    def isContiguous(self) -> bool:
        return self.data.is_contiguous()

    def contiguous(self):
        return Tensor(self.data.contiguous())

    def isEmpty(self) -> bool:
        return self.data.numel() == 0

    def isScalar(self) -> bool:
        return self.data.dim() == 0

    def isSameSizeAs(self, other) -> bool:
        return self.data.shape == _unwrap(other).shape

    def getType(self) -> str:
        return {torch.float32: "FloatType", torch.float64: "DoubleType", torch.int32: "IntType",
                torch.int64: "LongType", torch.bool: "BooleanType", torch.bfloat16: "BFloat16Type",
                torch.float16: "HalfType", torch.int8: "CharType", torch.int16: "ShortType"}.get(self.data.dtype, str(self.data.dtype))

    # ---- element access (1-based) -----------------------------------------------------------
    def valueAt(self, *idx):
        return self.data[tuple(i - 1 for i in idx)].item()

    def setValue(self, *args):
        *idx, v = args
        self.data[tuple(i - 1 for i in idx)] = v
        return self

    def __getitem__(self, i):
        if isinstance(i, int):
            r = self.data[i - 1]
            return Tensor(r) if r.dim() > 0 else r.item()
        return Tensor(self.data[i])

    def __setitem__(self, i, v):
        if isinstance(i, int):
            self.data[i - 1] = _unwrap(v)
        else:
            self.data[i] = _unwrap(v)

    def apply1(self, fn):
        arr = self.data.detach().cpu().numpy()
        vec = np.vectorize(fn, otypes=[arr.dtype])
        self.data.copy_(torch.from_numpy(vec(arr)))
        return self

    def map(self, other, fn):
        a = self.data.detach().cpu().numpy()
        b = _unwrap(other).detach().cpu().numpy()
        self.data.copy_(torch.from_numpy(np.vectorize(fn, otypes=[a.dtype])(a, b)))
        return self

    # ---- views --------------------------------------------------------------------------------
    def select(self, dim: int, index: int):
        d = _dim0(dim, self.data.dim())
        i = index - 1 if index > 0 else self.data.shape[d] + index
        return Tensor(self.data.select(d, i))

    def narrow(self, dim: int, index: int, size: int):
        return Tensor(self.data.narrow(_dim0(dim, self.data.dim()), index - 1, size))

    def transpose(self, d1: int, d2: int):
        nd = self.data.dim()
        return Tensor(self.data.transpose(_dim0(d1, nd), _dim0(d2, nd)))

    def t(self):
        return Tensor(self.data.t())

    def view(self, *sizes):
        if len(sizes) == 1 and isinstance(sizes[0], (list, tuple)):
            sizes = sizes[0]
        return Tensor(self.data.view(*sizes))

    def reshape(self, *sizes):
        if len(sizes) == 1 and isinstance(sizes[0], (list, tuple)):
            sizes = sizes[0]
        return Tensor(self.data.reshape(*sizes))

    def unfold(self, dim: int, size: int, step: int):
        return Tensor(self.data.unfold(_dim0(dim, self.data.dim()), size, step))

    def expand(self, *sizes):
        if len(sizes) == 1 and isinstance(sizes[0], (list, tuple)):
            sizes = sizes[0]
        return Tensor(self.data.expand(*sizes))

    def expandAs(self, other):
        return Tensor(self.data.expand_as(_unwrap(other)))

    def squeeze(self, dim: int | None = None):
        if dim is None:
            return Tensor(self.data.squeeze())
        return Tensor(self.data.squeeze(_dim0(dim, self.data.dim())))

    def unsqueeze(self, dim: int):
        return Tensor(self.data.unsqueeze(dim - 1))

    addSingletonDimension = unsqueeze

    def repeatTensor(self, *sizes):
        return Tensor(self.data.repeat(*sizes))

    def split(self, size: int, dim: int = 1):
        return [Tensor(t) for t in torch.split(self.data, size, _dim0(dim, self.data.dim()))]

    def clone(self):
        return Tensor(self.data.clone())

    # ---- in-place fill / copy ------------------------------------------------------------------
    def fill(self, v):
        self.data.fill_(v)
        return self

    def zero(self):
        self.data.zero_()
        return self

    def copy(self, other):
        self.data.copy_(_unwrap(other).reshape(self.data.shape) if _unwrap(other).shape != self.data.shape else _unwrap(other))
        return self

    def resize(self, *sizes):
        if len(sizes) == 1 and isinstance(sizes[0], (list, tuple)):
            sizes = sizes[0]
        if isinstance(sizes[0], Tensor):
            sizes = sizes[0].size()
        self.data = self.data.resize_(*sizes) if self.data.is_contiguous() else torch.empty(*sizes, dtype=self.data.dtype)
        return self

    def resizeAs(self, other):
        return self.resize(list(_unwrap(other).shape))

    def set(self, other=None):
        self.data = torch.empty(0, dtype=self.data.dtype) if other is None else _unwrap(other)
        return self

    def rand(self, lo=0.0, hi=1.0):
        self.data.copy_(RNG.uniform_tensor(tuple(self.data.shape), lo, hi))
        return self

    def randn(self, mean=0.0, std=1.0):
        self.data.copy_(RNG.normal_tensor(tuple(self.data.shape), mean, std))
        return self

    def bernoulli(self, p):
        self.data.copy_((RNG.uniform_tensor(tuple(self.data.shape)) < p).float())
        return self

    # ---- arithmetic (TensorMath) ---------------------------------------------------------------------
    def _vml2(self, other, op, p=1.0) -> bool:
        """in-place ``self ← self (op) other`` through the VML kernels (same-shape device tensors)."""
        o = _unwrap(other)
        return (isinstance(o, torch.Tensor) and self.data.is_cuda and o.shape == self.data.shape
                and _vml.binary(self.data, o, op, p, out=self.data) is not None)

    def add(self, *args):
        """add(value) | add(y) | add(value, y) | add(x, value, y) (Torch overloads)."""
        if len(args) == 1:
            a = _unwrap(args[0])
            if not self._vml2(a, "add"):
                self.data.add_(a)
        elif len(args) == 2:
            if not self._vml2(args[1], "add", float(args[0])):
                self.data.add_(_unwrap(args[1]), alpha=args[0])
        else:
            x, v, y = args
            self.data.copy_(_unwrap(x) + v * _unwrap(y))
        return self

    def sub(self, *args):
        if len(args) == 1:
            if not self._vml2(args[0], "sub"):
                self.data.sub_(_unwrap(args[0]))
        elif not self._vml2(args[1], "sub", float(args[0])):
            self.data.sub_(_unwrap(args[1]), alpha=args[0])
        return self

    def mul(self, *args):
        if len(args) == 1:
            self.data.mul_(_unwrap(args[0]))
        else:
            self.data.copy_(_unwrap(args[0]) * args[1])
        return self

    def div(self, v):
        self.data.div_(_unwrap(v))
        return self

    def cmul(self, *args):
        if len(args) == 1:
            if not self._vml2(args[0], "mul"):
                self.data.mul_(_unwrap(args[0]))
        else:
            self.data.copy_(_unwrap(args[0]) * _unwrap(args[1]))
        return self

    def cdiv(self, *args):
        if len(args) == 1:
            if not self._vml2(args[0], "div"):
                self.data.div_(_unwrap(args[0]))
        else:
            self.data.copy_(_unwrap(args[0]) / _unwrap(args[1]))
        return self

    def addcmul(self, value, t1, t2=None):
        if t2 is None:
            t1, t2, value = value, t1, 1.0
        self.data.addcmul_(_unwrap(t1), _unwrap(t2), value=value)
        return self

    def addcdiv(self, value, t1, t2):
        self.data.addcdiv_(_unwrap(t1), _unwrap(t2), value=value)
        return self

    def addmm(self, *args):
        """addmm([beta, M,] [alpha,] mat1, mat2) → self = beta·M + alpha·mat1·mat2."""
        beta, M, alpha = 1.0, self.data, 1.0
        a = list(args)
        if len(a) == 2:
            m1, m2 = a
        elif len(a) == 3:
            alpha, m1, m2 = a
        elif len(a) == 4:
            M, alpha, m1, m2 = a
            M = _unwrap(M)
        else:
            beta, M, alpha, m1, m2 = a
            M = _unwrap(M)
        r = torch.addmm(M, _unwrap(m1), _unwrap(m2), beta=beta, alpha=alpha)
        self.data = r if self.data.shape != r.shape else self.data.copy_(r)
        return self

    def addmv(self, *args):
        beta, M, alpha = 1.0, self.data, 1.0
        a = list(args)
        if len(a) == 2:
            m, v = a
        elif len(a) == 3:
            alpha, m, v = a
        else:
            beta, M, alpha, m, v = a
            M = _unwrap(M)
        r = torch.addmv(M, _unwrap(m), _unwrap(v), beta=beta, alpha=alpha)
        self.data = r if self.data.shape != r.shape else self.data.copy_(r)
        return self

    def addr(self, *args):
        a = list(args)
        alpha = 1.0
        if len(a) == 2:
            v1, v2 = a
        else:
            alpha, v1, v2 = a[-3], a[-2], a[-1]
        self.data.add_(torch.outer(_unwrap(v1), _unwrap(v2)), alpha=alpha)
        return self

    def baddbmm(self, beta, M, alpha, b1, b2):
        self.data = torch.baddbmm(_unwrap(M), _unwrap(b1), _unwrap(b2), beta=beta, alpha=alpha)
        return self

    def mm(self, a, b):
        self.data = torch.mm(_unwrap(a), _unwrap(b))
        return self

    def mv(self, a, b):
        self.data = torch.mv(_unwrap(a), _unwrap(b))
        return self

    def bmm(self, a, b):
        self.data = torch.bmm(_unwrap(a), _unwrap(b))
        return self

    def dot(self, other) -> float:
        return float((self.data * _unwrap(other)).sum())

    # elementwise unary (return new tensors like Torch's functional forms, or in place with no args)
    def _unary(self, fn, inplace=True):
        op = _VML_UNARY.get(fn)
        if op is not None and self.data.is_cuda and _vml.unary(self.data, op, out=self.data) is not None:
            return self
        r = fn(self.data)
        self.data.copy_(r)
        return self

    def abs(self):
        return self._unary(torch.abs)

    def exp(self):
        return self._unary(torch.exp)

    def log(self):
        return self._unary(torch.log)

    def log1p(self):
        return self._unary(torch.log1p)

    def sqrt(self):
        return self._unary(torch.sqrt)

    def tanh(self):
        return self._unary(torch.tanh)

    def sigmoid(self):
        return self._unary(torch.sigmoid)

    def floor(self):
        return self._unary(torch.floor)

    def ceil(self):
        return self._unary(torch.ceil)

    def negative(self):
        return self._unary(torch.neg)

    def inv(self):
        return self._unary(torch.reciprocal)

    def erf(self):
        return self._unary(torch.erf)

    def erfc(self):
        return self._unary(torch.erfc)

    def logGamma(self):
        return self._unary(torch.lgamma)

    def digamma(self):
        return self._unary(torch.digamma)

    def pow(self, n):
        if not (isinstance(n, (int, float)) and self.data.is_cuda
                and _vml.unary(self.data, "pow", float(n), out=self.data) is not None):
            self.data.pow_(n)
        return self

    def square(self):
        return self.pow(2)

    def clamp(self, lo, hi):
        self.data.clamp_(lo, hi)
        return self

    # ---- reductions ---------------------------------------------------------------------------------
    def _vml_reduce(self, op, dim):
        d = self.data
        if not d.is_cuda:
            return None
        r = _vml.reduce(d, op, None if dim is None else _dim0(dim, d.dim()), keepdim=True)
        if r is None:
            return None
        return float(r) if dim is None else Tensor(r.to(d.dtype))

    def sum(self, dim: int | None = None):
        r = self._vml_reduce("sum", dim)
        if r is not None:
            return r
        if dim is None:
            return float(self.data.sum())
        return Tensor(self.data.sum(_dim0(dim, self.data.dim()), keepdim=True))

    def mean(self, dim: int | None = None):
        r = self._vml_reduce("mean", dim)
        if r is not None:
            return r
        if dim is None:
            return float(self.data.float().mean())
        return Tensor(self.data.mean(_dim0(dim, self.data.dim()), keepdim=True))

    def prod(self, dim: int | None = None):
        if dim is None:
            return float(self.data.prod())
        return Tensor(self.data.prod(_dim0(dim, self.data.dim()), keepdim=True))

    def max(self, dim: int | None = None):
        if dim is None:
            r = self._vml_reduce("max", None)
            return r if r is not None else float(self.data.max())
        v, i = self.data.max(_dim0(dim, self.data.dim()), keepdim=True)
        return Tensor(v), Tensor((i + 1).float())

    def min(self, dim: int | None = None):
        if dim is None:
            r = self._vml_reduce("min", None)
            return r if r is not None else float(self.data.min())
        v, i = self.data.min(_dim0(dim, self.data.dim()), keepdim=True)
        return Tensor(v), Tensor((i + 1).float())

    def sumSquare(self) -> float:
        return float((self.data.float() ** 2).sum())

    def norm(self, p=2.0, dim: int | None = None):
        if dim is None:
            return float(torch.norm(self.data.float(), p))
        return Tensor(torch.norm(self.data.float(), p, dim=_dim0(dim, self.data.dim()), keepdim=True))

    def dist(self, other, p=2.0) -> float:
        return float(torch.dist(self.data.float(), _unwrap(other).float(), p))

    def topk(self, k, dim=-1, increase=True):
        d = dim if dim < 0 else dim - 1
        v, i = torch.topk(self.data, k, dim=d, largest=not increase)
        return Tensor(v), Tensor((i + 1).float())

    # ---- comparisons / masks -----------------------------------------------------------------------
    def gt(self, a, b):
        self.data = (_unwrap(a) > _unwrap(b)).to(self.data.dtype)
        return self

    def lt(self, a, b):
        self.data = (_unwrap(a) < _unwrap(b)).to(self.data.dtype)
        return self

    def le(self, a, b):
        self.data = (_unwrap(a) <= _unwrap(b)).to(self.data.dtype)
        return self

    def eq(self, a, b):
        self.data = (_unwrap(a) == _unwrap(b)).to(self.data.dtype)
        return self

    def maskedFill(self, mask, v):
        self.data.masked_fill_(_unwrap(mask).bool(), v)
        return self

    def maskedCopy(self, mask, src):
        self.data.masked_scatter_(_unwrap(mask).bool(), _unwrap(src))
        return self

    def maskedSelect(self, mask):
        return Tensor(self.data[_unwrap(mask).bool()])

    def index(self, dim, index):
        return Tensor(self.data.index_select(_dim0(dim, self.data.dim()), _unwrap(index).long() - 1))

    def indexAdd(self, dim, index, src):
        self.data.index_add_(_dim0(dim, self.data.dim()), _unwrap(index).long() - 1, _unwrap(src))
        return self

    def gather(self, dim, index):
        return Tensor(self.data.gather(_dim0(dim, self.data.dim()), _unwrap(index).long() - 1))

    def scatter(self, dim, index, src):
        self.data.scatter_(_dim0(dim, self.data.dim()), _unwrap(index).long() - 1, _unwrap(src))
        return self

    def almostEqual(self, other, delta: float) -> bool:
        o = _unwrap(other)
        return self.data.shape == o.shape and bool((self.data.float() - o.float()).abs().max() <= delta) if self.data.numel() else True

    # ---- comparison / element-wise extras (TensorMath.scala:222-824, DenseTensor.scala:2028-2271) ----
    def ge(self, a, b):
        """self = (a >= b) as 0/1 (``TensorMath.ge``, :740)."""
        self.data = (_unwrap(a) >= _unwrap(b)).to(self.data.dtype)
        return self

    def notEqualValue(self, value) -> bool:
        """True when any element differs from ``value``."""
        return bool((self.data != value).any())

    def _cpair(self, fn, a, b):
        if b is None:  # x.cmax(y) / x.cmax(value): in place
            o = _unwrap(a)
            self.data.copy_(fn(self.data, o if isinstance(o, torch.Tensor) else torch.tensor(o, dtype=self.data.dtype)))
            return self
        x, y = _unwrap(a), _unwrap(b)  # z.cmax(x, y): z = max(x, y)
        r = fn(x, y if isinstance(y, torch.Tensor) else torch.tensor(y, dtype=x.dtype))
        if self.data.shape != r.shape:
            self.data = torch.empty_like(r)
        self.data.copy_(r)
        return self

    def cmax(self, a, b=None):
        """Element-wise maximum with a tensor or a value (``TensorMath.cmax``, :305/:771/:789)."""
        return self._cpair(torch.maximum, a, b)

    def cmin(self, a, b=None):
        return self._cpair(torch.minimum, a, b)

    def sign(self):
        """In place: +1 / −1 / 0 (``DenseTensor.sign``, :2028)."""
        self.data.copy_(torch.sign(self.data))
        return self

    def _conv2(self, kernel, vf, flip):
        import torch.nn.functional as F
        vf = vf.upper() if isinstance(vf, str) else vf
        if vf not in ("V", "F"):
            raise ValueError(f"type must be 'V' (valid) or 'F' (full), got {vf!r}")
        x, k = self.data, _unwrap(kernel).to(self.data.dtype)
        if x.dim() != 2 or k.dim() != 2:
            raise ValueError("conv2 / xcorr2 take 2-D tensors")
        if flip:
            k = torch.flip(k, (0, 1))
        pad = (k.shape[0] - 1, k.shape[1] - 1) if vf == "F" else (0, 0)
        r = F.conv2d(x[None, None], k[None, None], padding=pad)[0, 0]
        return Tensor(r)

    def conv2(self, kernel, vf="V"):
        """2-D convolution (kernel flipped): valid ('V') or full ('F') (``TensorMath.conv2``, :222)."""
        return self._conv2(kernel, vf, True)

    def xcorr2(self, kernel, vf="V"):
        """2-D cross-correlation, valid or full (``TensorMath.xcorr2``, :232)."""
        return self._conv2(kernel, vf, False)

    def diff(self, other, count: int = 1, reverse: bool = False) -> bool:
        """Print up to ``count`` differing elements; True if the tensors differ (``DenseTensor.diff``,
        :1647); ``reverse`` scans from the last element."""
        o = _unwrap(other)
        if self.data.dim() != o.dim():
            print("Dimension number is different")
            return True
        for d in range(self.data.dim()):
            if self.data.shape[d] != o.shape[d]:
                print(f"Dimension {d + 1} is different, left is {self.data.shape[d]}, right is {o.shape[d]}")
                return True
        a, b = self.data.reshape(-1), o.reshape(-1)
        idx = torch.nonzero(a != b).reshape(-1)
        if reverse:
            idx = idx.flip(0)
        for i in idx[:count].tolist():
            print(f"Find difference at {i + 1}: left {a[i].item()}, right {b[i].item()}")
        return idx.numel() > 0

    def reduce(self, dim: int, result, reducer):
        """Fold dimension ``dim`` (1-based) with the binary ``reducer`` into ``result`` (size 1 along
        ``dim``; ``TensorMath.reduce``, :824 / ``DenseTensor.scala:2260``)."""
        import functools
        d = _dim0(dim, self.data.dim())
        a = self.data.detach().cpu().numpy()
        out = np.apply_along_axis(lambda v: functools.reduce(reducer, v.tolist()), d, a)
        r = torch.from_numpy(np.expand_dims(np.asarray(out, dtype=a.dtype), d))
        res = _unwrap(result)
        if tuple(res.shape) != tuple(r.shape):
            res.resize_(r.shape)
        res.copy_(r)
        return result

    def applyFun(self, t, func):
        """self[i] = func(t[i]), any source dtype (``Tensor.applyFun``, :520)."""
        src = _unwrap(t).detach().cpu().numpy()
        out = np.vectorize(func, otypes=[np.float64])(src) if src.size else src.astype(np.float64)
        if tuple(self.data.shape) != tuple(src.shape):
            self.data = torch.empty(src.shape, dtype=self.data.dtype, device=self.data.device)
        self.data.copy_(torch.from_numpy(out).to(self.data.dtype))
        return self

    def zipWith(self, t1, t2, func):
        """self[i] = func(t1[i], t2[i]) (``Tensor.zipWith``, :547)."""
        a = _unwrap(t1).detach().cpu().numpy()
        b = _unwrap(t2).detach().cpu().numpy()
        out = np.vectorize(func, otypes=[np.float64])(a, b) if a.size else a.astype(np.float64)
        if tuple(self.data.shape) != tuple(a.shape):
            self.data = torch.empty(a.shape, dtype=self.data.dtype, device=self.data.device)
        self.data.copy_(torch.from_numpy(out).to(self.data.dtype))
        return self

    def cast(self, cast_tensor):
        """Copy this tensor's values, converted, into ``cast_tensor`` (whatever its dtype) and return
        it (``Tensor.cast``, :387)."""
        dst = cast_tensor if isinstance(cast_tensor, Tensor) else Tensor(cast_tensor)
        if tuple(dst.data.shape) != tuple(self.data.shape):
            dst.data = torch.empty(self.data.shape, dtype=dst.data.dtype, device=dst.data.device)
        dst.data.copy_(self.data.to(dst.data.dtype))
        return dst

    def forceFill(self, v):
        """Fill with ``v`` converted to this tensor's dtype (``Tensor.forceFill``, :113)."""
        self.data.fill_(torch.tensor(v).to(self.data.dtype).item())
        return self

    def uniform(self, *args) -> float:
        """One uniform draw from the framework RNG: [0, 1); one arg a → between 1 and a; two args
        → [a, b] (``TensorMath.uniform``, :500)."""
        if not args:
            return RNG.uniform(0.0, 1.0)
        if len(args) == 1:
            lo, hi = sorted((1.0, float(args[0])))
        else:
            lo, hi = float(args[0]), float(args[1])
        return lo if lo == hi else RNG.uniform(lo, hi)

    # ---- storage / shape helpers (Tensor.scala:200-725) -------------------------------------------
    def storage(self):
        """The flat storage under this tensor, shared (``Tensor.storage``, :441)."""
        from .storage import Storage
        return Storage.of(self.data)

    def value(self):
        """The value of a one-element tensor (``Tensor.value``, :200)."""
        if self.data.numel() != 1:
            raise ValueError(f"value() needs a scalar tensor, got shape {tuple(self.data.shape)}")
        return self.data.reshape(()).item()

    def toArray(self):
        """Elements in row-major order as a flat Python list."""
        return self.data.detach().reshape(-1).cpu().tolist()

    def dim(self) -> int:
        return self.data.dim()

    def getTensorType(self) -> str:
        return "DenseType"

    def getTensorNumeric(self) -> str:
        return {torch.float32: "float", torch.float64: "double", torch.int32: "int", torch.int64: "long",
                torch.int16: "short", torch.bool: "boolean", torch.bfloat16: "bfloat16",
                torch.float16: "half"}.get(self.data.dtype, str(self.data.dtype))

    def shallowClone(self):
        """A new tensor over the same storage and geometry (``Tensor.shallowClone``, :358)."""
        return Tensor(self.data.view(self.data.shape) if self.data.numel() else self.data)

    def emptyInstance(self):
        return Tensor(torch.empty(0, dtype=self.data.dtype, device=self.data.device))

    def squeezeNewTensor(self):
        return Tensor(self.data.squeeze())

    def addSingletonDimension(self, t=None, dim: int = 1):
        """self ← a view of ``t`` (default self) with a size-1 dimension inserted at ``dim`` (1-based)."""
        src = self.data if t is None else _unwrap(t)
        if dim < 1 or dim > src.dim() + 1:
            raise IndexError(f"dimension {dim} out of range [1, {src.dim() + 1}]")
        self.data = src.unsqueeze(dim - 1)
        return self

    def addMultiDimension(self, t=None, dims=(1,)):
        """Insert size-1 dimensions at each of ``dims`` (positions in the source's numbering, shifted
        as earlier inserts land; ``DenseTensor.addMultiDimension``, :2095)."""
        src = self.data if t is None else _unwrap(t)
        ds = list(dims)
        for i in range(len(ds)):
            for j in range(i + 1, len(ds)):
                if ds[j] > ds[i]:
                    ds[j] += 1
        out = src
        for d in ds:
            out = out.unsqueeze(d - 1)
        self.data = out
        return self

    def numNonZeroByRow(self):
        """Non-zero count of every slice along the first dimension."""
        return (self.data.reshape(self.data.shape[0], -1) != 0).sum(1).tolist()

    def update(self, index, value):
        """``Tensor.update`` (:243-319): index = 1-based int (a value or a sub-tensor copy), a list
        of 1-based indices (one element), or a predicate (every element it accepts ← value)."""
        if callable(index):
            arr = self.data.detach().cpu().numpy()
            mask = torch.from_numpy(np.vectorize(index, otypes=[bool])(arr)).to(self.data.device)
            self.data.masked_fill_(mask, value)
        elif isinstance(index, (list, tuple)):
            self.data[tuple(i - 1 for i in index)] = value
        else:
            v = _unwrap(value)
            if isinstance(v, torch.Tensor):
                self.data[index - 1].copy_(v)
            else:
                self.data[index - 1] = v

    def save(self, path: str, over_write: bool = False):
        """Write the tensor to ``path`` (numpy .npy; loaded back by :meth:`load` without unpickling)."""
        import os
        if os.path.exists(path) and not over_write:
            raise FileExistsError(path)
        with open(path, "wb") as fh:
            np.save(fh, self.toNumpy(), allow_pickle=False)
        return self

    @staticmethod
    def load(path: str):
        with open(path, "rb") as fh:
            return Tensor(torch.from_numpy(np.load(fh, allow_pickle=False)))

    # ---- conversion ------------------------------------------------------------------------------------
    def toNumpy(self):
        return self.data.detach().cpu().numpy()

    to_ndarray = toNumpy

    def toTorch(self) -> torch.Tensor:
        return self.data

    def cuda(self):
        return Tensor(self.data.cuda())

    def cpu(self):
        return Tensor(self.data.cpu())

    def float(self):
        return Tensor(self.data.float())

    # ---- python protocol ------------------------------------------------------------------------------
    def __eq__(self, other):
        o = _unwrap(other)
        return isinstance(o, torch.Tensor) and o.shape == self.data.shape and bool(torch.equal(self.data.cpu(), o.cpu()))

    def __hash__(self):
        return id(self)

    def __repr__(self):
        return f"Tensor({self.data!r})"

    def __add__(self, o):
        return Tensor(self.data + _unwrap(o))

    def __sub__(self, o):
        return Tensor(self.data - _unwrap(o))

    def __mul__(self, o):
        return Tensor(self.data * _unwrap(o))

    def __truediv__(self, o):
        return Tensor(self.data / _unwrap(o))

    def __neg__(self):
        return Tensor(-self.data)

    def __len__(self):
        return self.data.shape[0]

    @property
    def shape(self):
        return tuple(self.data.shape)
