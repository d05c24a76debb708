"""Table layers (``DL/nn/{CAddTable,CSubTable,CMulTable,CDivTable,CMaxTable,CMinTable,CAveTable,
JoinTable,SplitTable,SelectTable,NarrowTable,FlattenTable,MixtureTable,BifurcateSplitTable,
TableOperation}.scala``).  ``CAddTable`` is on the ResNet hot path (residual add) and
``JoinTable`` on Inception's (channel concat, K19)."""
from __future__ import annotations

import torch

from ..abstractnn import TensorModule, AutogradModule
from ...utils.table import Table


class CAddTable(TensorModule):
    def __init__(self, inplace=False, bigdl_type="float"):
        super().__init__()
        self.inplace = inplace

    #: set by bigdl.nn.fusion when the preceding ConcatTable already produced the sum
    _passthrough = False

    def updateOutput(self, input):
        if self._passthrough:
            return input[1]
        ts = list(input)
        out = ts[0]  # ``inplace`` is honoured as a hint only (see Threshold)
        for t in ts[1:]:
            out = out + t
        return out

    def updateGradInput(self, input, gradOutput):
        if self._passthrough:
            return Table(gradOutput, gradOutput)
        gi = Table()
        for i, t in enumerate(list(input)):
            if t.shape == gradOutput.shape:
                gi[i + 1] = gradOutput
            else:  # broadcast input: reduce
                g = gradOutput
                while g.dim() > t.dim():
                    g = g.sum(0)
                for d in range(t.dim()):
                    if t.shape[d] == 1 and g.shape[d] != 1:
                        g = g.sum(d, keepdim=True)
                gi[i + 1] = g
        return gi


class CSubTable(TensorModule):
    def updateOutput(self, input):
        return input[1] - input[2]

    def updateGradInput(self, input, gradOutput):
        return Table(gradOutput, -gradOutput)


class CMulTable(TensorModule):
    def updateOutput(self, input):
        out = input[1]
        for t in list(input)[1:]:
            out = out * t
        return out

    def updateGradInput(self, input, gradOutput):
        ts = list(input)
        gi = Table()
        for i in range(len(ts)):
            g = gradOutput
            for j, t in enumerate(ts):
                if j != i:
                    g = g * t
            gi[i + 1] = g
        return gi


class CDivTable(TensorModule):
    def updateOutput(self, input):
        return input[1] / input[2]

    def updateGradInput(self, input, gradOutput):
        a, b = input[1], input[2]
        return Table(gradOutput / b, -gradOutput * a / (b * b))


class CMaxTable(AutogradModule):
    def _forward(self, x):
        ts = list(x)
        out = ts[0]
        for t in ts[1:]:
            out = torch.maximum(out, t)
        return out


class CMinTable(AutogradModule):
    def _forward(self, x):
        ts = list(x)
        out = ts[0]
        for t in ts[1:]:
            out = torch.minimum(out, t)
        return out


class CAveTable(AutogradModule):
    def __init__(self, inplace=False, bigdl_type="float"):
        super().__init__()

    def _forward(self, x):
        ts = list(x)
        return sum(ts) / len(ts)


def _tiles_channels(big, ts) -> bool:
    """``ts`` are, in order, the consecutive channel slices of 4-D ``big``."""
    c0 = 0
    es = big.element_size()
    for t in ts:
        if (t.dim() != 4 or t.shape[0] != big.shape[0] or t.shape[2:] != big.shape[2:]
                or t.data_ptr() != big.data_ptr() + c0 * es or t.stride() != big.stride()):
            return False
        c0 += t.shape[1]
    return c0 == big.shape[1]


class JoinTable(TensorModule):
    """Concatenate table entries along ``dimension`` (1-based, batch-shifted by nInputDims)."""

    def __init__(self, dimension, n_input_dims=0, bigdl_type="float"):
        super().__init__()
        self.dimension, self.nInputDims = dimension, n_input_dims

    def _d(self, x):
        d = self.dimension - 1 if self.dimension > 0 else x.dim() + self.dimension
        if self.nInputDims > 0 and x.dim() > self.nInputDims and self.dimension > 0:
            d += x.dim() - self.nInputDims
        return d

    #: preallocated output whose channel slices the producing convs wrote directly (zero-copy
    #: concat, planned by :func:`bigdl.nn.containers.plan_concat`); consumed once
    _planned = None

    #: set by the int8 quantizer (nn/quantized/quantizer.py _link_graph): the inputs arrive as int8 codes
    #: of one common scale
    _i8_join = False

    def _i8_cat_buffer(self, N_, C_, H, W, dev, u8):
        """This forward's concat output, shared by the producing int8 convs (each writes its channel
        slice: quantizer._link_graph ``_cat_join``); the 0x80 tail of an unsigned code written once."""
        from ...ops import native_ops as NO
        b = self.__dict__.get("_i8buf")
        if b is None or tuple(b.shape) != (N_, C_, H, W) or b.device != dev or bool(b._qtail) != bool(u8):
            b = NO._i8_act(N_, C_, H, W, dev, u8)
            if u8:
                n = b.numel()
                b._base.view(-1)[n:n + 16].fill_(-128)
            b._qtail = bool(u8)
            self.__dict__["_i8buf"] = b
        return b

    def _int8_cat(self, ts, d):
        """Concat of int8 activations sharing one scale / code (a quantised Inception block): the
        codes are concatenated as they are and the result keeps the tag (+ the 0x80 tail an unsigned
        code carries for padded consumer taps)."""
        from ...ops import native_ops as NO
        t0 = ts[0]
        sc, z = getattr(t0, "_qscale", None), getattr(t0, "_qzero", 0)
        if (sc is None or d != 1 or t0.dim() != 4 or not t0.is_cuda
                or any(t.dtype != torch.int8 or getattr(t, "_qscale", None) != sc or getattr(t, "_qzero", 0) != z
                       or t.shape[0] != t0.shape[0] or t.shape[2:] != t0.shape[2:] for t in ts)):
            return None
        u8 = bool(z)
        N_, H, W = t0.shape[0], t0.shape[2], t0.shape[3]
        y = NO._i8_act(N_, sum(t.shape[1] for t in ts), H, W, t0.device, u8)
        c0 = 0
        for t in ts:
            y[:, c0:c0 + t.shape[1]].copy_(t)
            c0 += t.shape[1]
        if u8:
            n = y.numel()
            y._base.view(-1)[n:n + 16].fill_(-128)
        return NO._tag(y, sc, u8)

    def updateOutput(self, input):
        ts = list(input)
        d = self._d(ts[0])
        self._sizes = [t.shape[d] for t in ts]
        if ts[0].dtype == torch.int8:
            buf = self.__dict__.pop("_i8buf", None)
            if buf is not None and d == 1:
                off, ok = 0, True
                for t in ts:  # every input is the producer's slice of the shared output, in order
                    ok = ok and (t.dtype == torch.int8 and t.data_ptr() == buf.data_ptr() + off
                                 and t.shape[0] == buf.shape[0] and t.shape[2:] == buf.shape[2:]
                                 and getattr(t, "_qscale", None) == getattr(ts[0], "_qscale", None))
                    off += t.shape[1]
                if ok and off == buf.shape[1]:
                    from ...ops import native_ops as NO
                    y = NO._tag(buf, ts[0]._qscale, bool(getattr(ts[0], "_qzero", 0)))
                    y._qtail = bool(getattr(ts[0], "_qzero", 0))
                    return y
            y = self._int8_cat(ts, d)
            if y is not None:
                return y
            from ..quantized.layers import dequant
            ts = [dequant(t) if getattr(t, "_qscale", None) is not None else t for t in ts]
        big, self._planned = self._planned, None
        if big is not None and d == 1 and _tiles_channels(big, ts):
            return big
        if ts[0].is_cuda and ts[0].dim() == 4 and d == 1:
            return torch.cat(ts, d).contiguous(memory_format=torch.channels_last)
        return torch.cat(ts, d)

    def updateGradInput(self, input, gradOutput):
        ts = list(input)
        d = self._d(ts[0])
        parts = torch.split(gradOutput, self._sizes, dim=d)
        gi = Table()
        for i, p in enumerate(parts):
            if p.is_cuda and p.dim() == 4:
                gi[i + 1] = p.contiguous(memory_format=torch.channels_last)
            else:
                gi[i + 1] = p.contiguous()
        return gi


class SplitTable(TensorModule):
    def __init__(self, dimension, n_input_dims=-1, bigdl_type="float"):
        super().__init__()
        self.dimension, self.nInputDims = dimension, n_input_dims

    def _d(self, x):
        d = self.dimension - 1 if self.dimension > 0 else x.dim() + self.dimension
        if self.nInputDims > 0 and x.dim() > self.nInputDims and self.dimension > 0:
            d += x.dim() - self.nInputDims
        return d

    def updateOutput(self, input):
        d = self._d(input)
        return Table(*[t for t in torch.unbind(input, d)])

    def updateGradInput(self, input, gradOutput):
        d = self._d(input)
        return torch.stack(list(gradOutput), d)


class BifurcateSplitTable(TensorModule):
    def __init__(self, dimension, bigdl_type="float"):
        super().__init__()
        self.dimension = dimension

    def updateOutput(self, input):
        d = self.dimension - 1
        n = input.shape[d] // 2
        return Table(input.narrow(d, 0, n), input.narrow(d, n, input.shape[d] - n))

    def updateGradInput(self, input, gradOutput):
        return torch.cat([gradOutput[1], gradOutput[2]], self.dimension - 1)


class SelectTable(TensorModule):
    def __init__(self, index, bigdl_type="float"):
        super().__init__()
        self.index = index

    def _i(self, input):
        return self.index if self.index > 0 else input.length() + self.index + 1

    def updateOutput(self, input):
        return input[self._i(input)]

    def updateGradInput(self, input, gradOutput):
        gi = Table()
        idx = self._i(input)
        for k in range(1, input.length() + 1):
            if k == idx:
                gi[k] = gradOutput
            else:
                v = input[k]
                gi[k] = torch.zeros_like(v) if isinstance(v, torch.Tensor) else _zeros_like_table(v)
        return gi


def _zeros_like_table(t):
    out = Table()
    for k, v in t.items():
        out[k] = torch.zeros_like(v) if isinstance(v, torch.Tensor) else _zeros_like_table(v)
    return out


class NarrowTable(TensorModule):
    def __init__(self, offset, length=1, bigdl_type="float"):
        super().__init__()
        self.offset, self.length = offset, length

    def _range(self, input):
        n = input.length()
        ln = self.length if self.length > 0 else n - self.offset + 2 + self.length
        return self.offset, ln

    def updateOutput(self, input):
        off, ln = self._range(input)
        return Table(*[input[off + i] for i in range(ln)])

    def updateGradInput(self, input, gradOutput):
        off, ln = self._range(input)
        gi = Table()
        for k in range(1, input.length() + 1):
            if off <= k < off + ln:
                gi[k] = gradOutput[k - off + 1]
            else:
                gi[k] = torch.zeros_like(input[k])
        return gi


class FlattenTable(TensorModule):
    def updateOutput(self, input):
        return input.flatten()

    def updateGradInput(self, input, gradOutput):
        flat = list(gradOutput)
        pos = [0]

        def rebuild(t):
            out = Table()
            for k in range(1, t.length() + 1):
                v = t[k]
                if isinstance(v, Table):
                    out[k] = rebuild(v)
                else:
                    out[k] = flat[pos[0]]
                    pos[0] += 1
            return out
        return rebuild(input)


class MixtureTable(AutogradModule):
    """Mixture of experts: Table(gater (N,E), experts Table or tensor) (``MixtureTable.scala``)."""

    def __init__(self, dim=INT_MAX if False else 2147483647, bigdl_type="float"):
        super().__init__()
        self.dim = dim

    def _forward(self, x):
        gater, experts = x[1], x[2]
        if isinstance(experts, Table):
            ex = torch.stack(list(experts), 1)
        else:
            ex = experts
        g = gater
        while g.dim() < ex.dim():
            g = g.unsqueeze(-1)
        return (g * ex).sum(1)


class TableOperation(AutogradModule):
    """Apply a 2-input table op, broadcasting the smaller operand (``TableOperation.scala``)."""

    def __init__(self, operation_layer, bigdl_type="float"):
        super().__init__()
        self.operation = operation_layer

    def _forward(self, x):
        a, b = x[1], x[2]
        if a.numel() < b.numel():
            a = a.expand_as(b)
        elif b.numel() < a.numel():
            b = b.expand_as(a)
        op = self.operation
        name = type(op).__name__
        if name == "CAddTable":
            return a + b
        if name == "CMulTable":
            return a * b
        if name == "CSubTable":
            return a - b
        if name == "CDivTable":
            return a / b
        if name == "CMaxTable":
            return torch.maximum(a, b)
        if name == "CMinTable":
            return torch.minimum(a, b)
        return op.forward(Table(a, b))
