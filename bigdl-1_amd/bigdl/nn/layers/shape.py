"""Shape/view layers (``DL/nn/{Reshape,View,InferReshape,Squeeze,Unsqueeze,Transpose,Contiguous,
Narrow,Select,Index,Padding,SpatialZeroPadding,Cropping2D,Cropping3D,Replicate,Tile,Reverse,Pack,
ExpandSize,Masking,MaskedSelect,Identity,Echo}.scala``).  All dimension arguments are 1-based as
in the reference; ``nInputDims`` marks the non-batch rank so a leading batch dim is skipped.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from ..abstractnn import TensorModule, AutogradModule
from ...utils.table import Table

INTMIN = -2147483648
INTMAX = 2147483647


def _bdim(dim, x, n_input_dims):
    """1-based dim → 0-based, shifted by a batch dim when the input has more dims than nInputDims."""
    d = dim - 1 if dim > 0 else x.dim() + dim
    if n_input_dims is not None and n_input_dims > 0 and x.dim() > n_input_dims and dim > 0:
        d += x.dim() - n_input_dims
    return d


class Identity(TensorModule):
    def updateOutput(self, input):
        return input

    def updateGradInput(self, input, gradOutput):
        return gradOutput


class Echo(Identity):
    """Pass-through that reports activations (``Echo.scala``): ``feval(module, input)`` on forward
    and ``bfeval(module, gradOutput)`` on backward; the default prints the shapes."""

    def __init__(self, feval=None, bfeval=None, bigdl_type="float"):
        super().__init__()
        self.feval, self.bfeval = feval, bfeval

    def updateOutput(self, input):
        if self.feval is not None:
            self.feval(self, input)
        else:
            print(f"{self.get_name()} : Activation size is {tuple(input.shape) if hasattr(input, 'shape') else input}")
        return input

    def updateGradInput(self, input, gradOutput):
        if self.bfeval is not None:
            self.bfeval(self, gradOutput)
        else:
            print(f"{self.get_name()} : Gradient size is {tuple(gradOutput.shape) if hasattr(gradOutput, 'shape') else gradOutput}")
        return gradOutput


class Contiguous(TensorModule):
    def updateOutput(self, input):
        return input.contiguous()

    def updateGradInput(self, input, gradOutput):
        return gradOutput.contiguous()


class Reshape(TensorModule):
    def __init__(self, size, batch_mode=None, bigdl_type="float"):
        super().__init__()
        self.size = [int(s) for s in size]
        self.batchMode = batch_mode
        self.nElement = int(np.prod(self.size))

    def updateOutput(self, input):
        if (self.batchMode is False) or (self.batchMode is None and input.numel() == self.nElement):
            return _keep_qtags(input.reshape(self.size), input)
        return _keep_qtags(input.reshape([input.shape[0]] + self.size), input)

    def updateGradInput(self, input, gradOutput):
        return gradOutput.reshape(input.shape)


def _keep_qtags(y, x):
    """A reshaped int8 activation of a quantised chain keeps its scale tags (the 0x80 padding tail
    only when the reshape is a view of the same memory)."""
    if x.dtype == torch.int8 and getattr(x, "_qscale", None) is not None:
        y._qscale = x._qscale
        y._qzero = getattr(x, "_qzero", 0)
        y._qtail = bool(getattr(x, "_qtail", False)) and y.data_ptr() == x.data_ptr()
    return y


class View(TensorModule):
    def __init__(self, sizes, num_input_dims=0, bigdl_type="float"):
        super().__init__()
        self.sizes = [int(s) for s in (sizes if isinstance(sizes, (list, tuple)) else [sizes])]
        self.numInputDims = num_input_dims

    def setNumInputDims(self, n):
        self.numInputDims = n
        return self

    def updateOutput(self, input):
        n = int(np.prod([s for s in self.sizes if s != -1]))
        if self.numInputDims > 0 and input.dim() > self.numInputDims:
            return _keep_qtags(input.reshape([input.shape[0]] + self.sizes), input)
        if -1 not in self.sizes and input.numel() != n:
            return _keep_qtags(input.reshape([input.shape[0]] + self.sizes), input)
        return _keep_qtags(input.reshape(self.sizes), input)

    def updateGradInput(self, input, gradOutput):
        return gradOutput.reshape(input.shape)


class InferReshape(TensorModule):
    """Reshape with -1 (infer) and 0 (copy input dim) entries (``InferReshape.scala``)."""

    def __init__(self, size, batch_mode=False, bigdl_type="float"):
        super().__init__()
        self.size = [int(s) for s in size]
        self.batchMode = batch_mode

    def updateOutput(self, input):
        src = list(input.shape[1:]) if self.batchMode else list(input.shape)
        out = [src[i] if s == 0 else s for i, s in enumerate(self.size)]
        if self.batchMode:
            out = [input.shape[0]] + out
        return _keep_qtags(input.reshape(out), input)

    def updateGradInput(self, input, gradOutput):
        return gradOutput.reshape(input.shape)


class Squeeze(TensorModule):
    """``batch_mode`` (Squeeze.scala's ``batchMode``): with no ``dim``, squeeze every size-1 dimension
    except the first (a batch of one keeps its batch dimension)."""

    def __init__(self, dim=INTMIN, num_input_dims=INTMIN, bigdl_type="float", batch_mode=False):
        super().__init__()
        self.dims = None if dim == INTMIN or dim is None else ([dim] if isinstance(dim, int) else list(dim))
        self.numInputDims = None if num_input_dims == INTMIN else num_input_dims
        self.batchMode = bool(batch_mode)

    def updateOutput(self, input):
        if self.dims is None:
            if self.batchMode and input.dim() > 0:
                return input.reshape([input.shape[0]] + [s for s in input.shape[1:] if s != 1])
            return input.squeeze()
        y = input
        for d in sorted((_bdim(d, input, self.numInputDims) for d in self.dims), reverse=True):
            y = y.squeeze(d)
        return y

    def updateGradInput(self, input, gradOutput):
        return gradOutput.reshape(input.shape)


class Unsqueeze(TensorModule):
    def __init__(self, pos, num_input_dims=INTMIN, bigdl_type="float"):
        super().__init__()
        self.pos = pos
        self.numInputDims = None if num_input_dims == INTMIN else num_input_dims

    def updateOutput(self, input):
        d = self.pos - 1
        if self.numInputDims is not None and input.dim() > self.numInputDims:
            d += input.dim() - self.numInputDims
        return input.unsqueeze(d)

    def updateGradInput(self, input, gradOutput):
        return gradOutput.reshape(input.shape)


class Transpose(TensorModule):
    def __init__(self, permutations, bigdl_type="float"):
        super().__init__()
        perms = list(permutations)
        if perms and not isinstance(perms[0], (tuple, list)):
            # flat [a1, b1, a2, b2, ...] (a deserialized permutation table)
            perms = [(perms[i], perms[i + 1]) for i in range(0, len(perms), 2)]
        self.permutations = [tuple(int(v) for v in p) for p in perms]

    def updateOutput(self, input):
        y = input
        for a, b in self.permutations:
            y = y.transpose(a - 1, b - 1)
        return y.contiguous()

    def updateGradInput(self, input, gradOutput):
        g = gradOutput
        for a, b in reversed(self.permutations):
            g = g.transpose(a - 1, b - 1)
        return g.contiguous()


class Narrow(TensorModule):
    def __init__(self, dimension, offset, length=1, bigdl_type="float"):
        super().__init__()
        self.dimension, self.offset, self.length = dimension, offset, length

    def _geom(self, x):
        d = self.dimension - 1 if self.dimension > 0 else x.dim() + self.dimension
        size = x.shape[d]
        off = self.offset - 1 if self.offset > 0 else size + self.offset
        ln = self.length if self.length > 0 else size - off + self.length + 1
        return d, off, ln

    def updateOutput(self, input):
        d, off, ln = self._geom(input)
        return input.narrow(d, off, ln)

    def updateGradInput(self, input, gradOutput):
        d, off, ln = self._geom(input)
        gi = torch.zeros_like(input, dtype=gradOutput.dtype)
        gi.narrow(d, off, ln).copy_(gradOutput)
        return gi


class Select(TensorModule):
    def __init__(self, dim, index, bigdl_type="float"):
        super().__init__()
        self.dim, self.index = dim, index

    def _geom(self, x):
        d = self.dim - 1 if self.dim > 0 else x.dim() + self.dim
        i = self.index - 1 if self.index > 0 else x.shape[d] + self.index
        return d, i

    def updateOutput(self, input):
        d, i = self._geom(input)
        return input.select(d, i)

    def updateGradInput(self, input, gradOutput):
        d, i = self._geom(input)
        gi = torch.zeros_like(input, dtype=gradOutput.dtype)
        gi.select(d, i).copy_(gradOutput)
        return gi


class Index(AutogradModule):
    """Table(tensor, index(1-based)) → tensor.index_select(dimension)."""

    def __init__(self, dimension, bigdl_type="float"):
        super().__init__()
        self.dimension = dimension

    def _forward(self, x):
        return x[1].index_select(self.dimension - 1, x[2].long().reshape(-1) - 1)


class Padding(AutogradModule):
    """Pad ``|pad|`` entries of ``value`` after (pad>0) or before (pad<0) along ``dim``."""

    def __init__(self, dim, pad, n_input_dim, value=0.0, n_index=1, bigdl_type="float"):
        super().__init__()
        self.dim, self.pad, self.nInputDim, self.value, self.nIndex = dim, pad, n_input_dim, value, n_index

    def _forward(self, x):
        d = _bdim(self.dim, x, self.nInputDim)
        shp = list(x.shape)
        shp[d] = abs(self.pad)
        fill = torch.full(shp, self.value, dtype=x.dtype, device=x.device)
        return torch.cat([x, fill], d) if self.pad > 0 else torch.cat([fill, x], d)


class SpatialZeroPadding(AutogradModule):
    def __init__(self, pad_left, pad_right, pad_top, pad_bottom, bigdl_type="float"):
        super().__init__()
        self.pads = (pad_left, pad_right, pad_top, pad_bottom)

    def _forward(self, x):
        return F.pad(x, self.pads)


class Cropping2D(AutogradModule):
    def __init__(self, heightCrop, widthCrop, data_format="NCHW", bigdl_type="float"):
        super().__init__()
        self.h, self.w, self.format = list(heightCrop), list(widthCrop), data_format

    def _forward(self, x):
        if self.format == "NCHW":
            H, W = x.shape[2], x.shape[3]
            return x[:, :, self.h[0]:H - self.h[1], self.w[0]:W - self.w[1]]
        H, W = x.shape[1], x.shape[2]
        return x[:, self.h[0]:H - self.h[1], self.w[0]:W - self.w[1], :]


class Cropping3D(AutogradModule):
    def __init__(self, dim1Crop, dim2Crop, dim3Crop, data_format="channel_first", bigdl_type="float"):
        super().__init__()
        self.c = [list(dim1Crop), list(dim2Crop), list(dim3Crop)]
        self.format = data_format

    def _forward(self, x):
        off = 2 if self.format == "channel_first" else 1
        sl = [slice(None)] * x.dim()
        for i, (a, b) in enumerate(self.c):
            n = x.shape[off + i]
            sl[off + i] = slice(a, n - b)
        return x[tuple(sl)]


class Replicate(AutogradModule):
    """Insert a new dim ``dim`` of size nFeatures by replication (``Replicate.scala``)."""

    def __init__(self, n_features, dim=1, n_dim=INTMAX, bigdl_type="float"):
        super().__init__()
        self.nFeatures, self.dim, self.nDim = n_features, dim, n_dim

    def _forward(self, x):
        d = self.dim - 1
        if self.nDim != INTMAX and x.dim() > self.nDim:
            d += x.dim() - self.nDim
        return x.unsqueeze(d).expand(*x.shape[:d], self.nFeatures, *x.shape[d:]).contiguous()


class Tile(AutogradModule):
    def __init__(self, dim=1, copies=2, bigdl_type="float"):
        super().__init__()
        self.dim, self.copies = dim, copies

    def _forward(self, x):
        reps = [1] * x.dim()
        reps[self.dim - 1] = self.copies
        return x.repeat(*reps)


class Reverse(AutogradModule):
    def __init__(self, dimension=1, is_inplace=False, bigdl_type="float"):
        super().__init__()
        self.dimension = dimension

    def _forward(self, x):
        return torch.flip(x, [self.dimension - 1])


class Pack(AutogradModule):
    """Stack a Table of tensors along a new 1-based dim."""

    def __init__(self, dimension, bigdl_type="float"):
        super().__init__()
        self.dimension = dimension

    def _forward(self, x):
        ts = list(x) if isinstance(x, Table) else [x]
        return torch.stack(ts, self.dimension - 1)


class ExpandSize(AutogradModule):
    def __init__(self, sizes, bigdl_type="float"):
        super().__init__()
        self.sizes = list(sizes)

    def _forward(self, x):
        return x.expand(*[x.shape[i] if s == -1 else s for i, s in enumerate(self.sizes)]).contiguous()


class Masking(AutogradModule):
    """Zero every time step whose features all equal ``mask_value`` (``Masking.scala``)."""

    def __init__(self, mask_value=0.0, bigdl_type="float"):
        super().__init__()
        self.maskValue = mask_value

    def _forward(self, x):
        keep = (x != self.maskValue).any(dim=-1, keepdim=True)
        return x * keep.to(x.dtype)


class MaskedSelect(TensorModule):
    def updateOutput(self, input):
        return input[1][input[2].bool()]

    def updateGradInput(self, input, gradOutput):
        g = torch.zeros_like(input[1], dtype=gradOutput.dtype)
        g[input[2].bool()] = gradOutput
        return Table(g, torch.zeros_like(input[2]))


class FaultInject(Identity):
    """Test-only fault injection (the reference's ``ExceptionTest``, ``TS/utils/TestUtils.scala:126-155``):
    a pass-through that raises on its ``fail_at``-th forward (1-based) — or on every forward from
    then on when ``once`` is False — to exercise the optimizer retry loop and the launcher's
    restart path.  The counter is class-wide per ``key`` so it survives module reloads from a
    checkpoint within one process."""

    _counts = {}

    def __init__(self, fail_at: int = 1, once: bool = True, key: str = "default", bigdl_type="float"):
        super().__init__()
        self.fail_at, self.once, self.key = fail_at, once, key

    def updateOutput(self, input):
        n = FaultInject._counts.get(self.key, 0) + 1
        FaultInject._counts[self.key] = n
        if n == self.fail_at or (not self.once and n >= self.fail_at):
            raise RuntimeError(f"FaultInject[{self.key}]: injected failure at forward {n}")
        return input

    @staticmethod
    def reset(key: str = None):
        if key is None:
            FaultInject._counts.clear()
        else:
            FaultInject._counts.pop(key, None)
