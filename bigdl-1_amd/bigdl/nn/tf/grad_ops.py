"""TensorFlow backward ("*Grad") and training-graph operations for imported TF graphs.

Reference: ``DL/nn/tf/NNOps.scala`` (Conv2DTranspose :84, Conv2DBackFilter :170, Conv3D :248,
Conv3DBackpropFilter(V2) :317/:394, Conv3DBackpropInput(V2) :431/:521, Relu6Grad … SigmoidGrad
:600-700, MaxPoolGrad :771, LRNGrad :830, FusedBatchNormGrad :994, AvgPoolGrad :1041, BiasAddGrad
:1089, ReluGrad :1149), ``DL/nn/tf/MathOps.scala`` (SqrtGrad, RsqrtGrad), ``ArrayOps.scala``
(BroadcastGradientArgs :197), ``ParsingOps.scala`` (ParseSingleExample :93), ``DL/nn/ops/Mod.scala``
and the loaders ``DL/utils/tf/loaders/*Grad*.scala``, ``Dilation2D*.scala``, ``TruncateMod.scala``.

These are cold-path host/torch operations (a TF training graph's own backward, imported as
forward-only ``Operation`` nodes).  Every backprop op is DEFINED as the exact gradient of the
corresponding forward op of this package (``Conv2D``, ``MaxPool``, ``AvgPool``, ``LRN``,
``ops.Dilation2D``, ``ResizeBilinearOps``) through ``torch.autograd.grad`` on that forward — so the
TF padding / data-format conventions of the forward and its gradient can never disagree — and the
elementwise *Grad ops are TensorFlow's closed forms.
"""
from __future__ import annotations

from typing import List, Sequence

import torch
import torch.nn.functional as F

from ...utils.table import Table
from ..ops import Operation


def _vals(t):
    return t.values() if isinstance(t, Table) else [t]


def _ints(t) -> List[int]:
    return [int(v) for v in torch.as_tensor(t).flatten().tolist()]


def _vjp(fwd, primal: torch.Tensor, dy: torch.Tensor) -> torch.Tensor:
    """d(fwd(primal))/d(primal) applied to ``dy`` (fp32, autograd on the forward definition)."""
    with torch.enable_grad():
        p = primal.detach().float().requires_grad_(True)
        y = fwd(p)
        (g,) = torch.autograd.grad(y, p, dy.float())
    return g


# ------------------------------------------------------------------------------------------------ elementwise
class _Binary(Operation):
    def updateOutput(self, t):
        a, b = _vals(t)[:2]
        return self._f(a, b)


class ReluGrad(_Binary):
    """(gradients, features) → gradients · [features > 0]."""

    def _f(self, g, x):
        return g * (x > 0).to(g.dtype)


class Relu6Grad(_Binary):
    """(gradients, features) → gradients · [0 < features < 6]."""

    def _f(self, g, x):
        return g * ((x > 0) & (x < 6)).to(g.dtype)


class EluGrad(_Binary):
    """(gradients, outputs) → gradients · (outputs > 0 ? 1 : outputs + 1)."""

    def _f(self, g, y):
        return torch.where(y > 0, g, g * (y + 1))


class SoftplusGrad(_Binary):
    """(gradients, features) → gradients · sigmoid(features)."""

    def _f(self, g, x):
        return g * torch.sigmoid(x)


class SoftsignGrad(_Binary):
    """(gradients, features) → gradients / (1 + |features|)²."""

    def _f(self, g, x):
        return g / (1 + x.abs()) ** 2


class TanhGrad(_Binary):
    """(y, dy) → dy · (1 − y²)."""

    def _f(self, y, dy):
        return dy * (1 - y * y)


class SigmoidGrad(_Binary):
    """(y, dy) → dy · y · (1 − y)."""

    def _f(self, y, dy):
        return dy * y * (1 - y)


class SqrtGrad(_Binary):
    """(y, dy) → dy · 0.5 / y."""

    def _f(self, y, dy):
        return dy * 0.5 / y


class RsqrtGrad(_Binary):
    """(y, dy) → dy · (−0.5) · y³."""

    def _f(self, y, dy):
        return dy * -0.5 * y * y * y


class InvGrad(_Binary):
    """(y, dy) → −dy · y² (also TF's ReciprocalGrad)."""

    def _f(self, y, dy):
        return -dy * y * y


ReciprocalGrad = InvGrad


class Mod(_Binary):
    """TF ``Mod`` / ``TruncateMod``: remainder of the truncating division (C ``fmod`` semantics;
    ``DL/nn/ops/Mod.scala``)."""

    def _f(self, a, b):
        return torch.fmod(a, b)


TruncateMod = Mod


class BiasAddGrad(Operation):
    """out_backprop → Σ over every dim but the channel one (last for NHWC, dim 1 for NCHW)."""

    def __init__(self, data_format="NHWC"):
        super().__init__()
        self.format = data_format

    def updateOutput(self, g):
        g = _vals(g)[0]
        if self.format == "NCHW" and g.dim() >= 3:
            dims = [d for d in range(g.dim()) if d != 1]
        else:
            dims = list(range(g.dim() - 1))
        return g.sum(dims) if dims else g


class BroadcastGradientArgs(Operation):
    """(s0, s1) → (r0, r1): the axes each input's gradient must be summed over after a broadcast
    binary op (``ArrayOps.scala:197``)."""

    def updateOutput(self, t):
        s0, s1 = (_ints(v) for v in _vals(t)[:2])
        n = max(len(s0), len(s1))
        a = [1] * (n - len(s0)) + s0
        b = [1] * (n - len(s1)) + s1
        r0, r1 = [], []
        for i, (x, y) in enumerate(zip(a, b)):
            if x == 1 and y != 1:
                r0.append(i)
            elif y == 1 and x != 1:
                r1.append(i)
            elif x == 1 and y == 1:
                r0.append(i)
                r1.append(i)
            elif x != y:
                raise ValueError(f"BroadcastGradientArgs: incompatible shapes {s0} and {s1}")
        return Table(torch.tensor(r0, dtype=torch.int32), torch.tensor(r1, dtype=torch.int32))


# ------------------------------------------------------------------------------------------------ conv 2-D / 3-D
def _conv2d_fwd(strides, padding, data_format, dilations):
    from . import Conv2D
    op = Conv2D(strides, padding, data_format, dilations)
    return lambda x, f: op.updateOutput(Table(x, f))


class Conv2DTranspose(Operation):
    """TF ``Conv2DBackpropInput``: Table(input_sizes, filter [kh, kw, Cin, Cout], out_backprop)
    → gradient w.r.t. the conv input (``NNOps.scala:84``)."""

    def __init__(self, strides=(1, 1, 1, 1), padding="SAME", data_format="NHWC", dilations=(1, 1, 1, 1)):
        super().__init__()
        self.strides, self.padding, self.format = list(strides), padding, data_format
        self.dilations = list(dilations or (1, 1, 1, 1))

    def updateOutput(self, t):
        sizes, f, dy = _vals(t)[:3]
        fwd = _conv2d_fwd(self.strides, self.padding, self.format, self.dilations)
        x0 = torch.zeros(_ints(sizes), dtype=torch.float32)
        ff = f.float()
        return _vjp(lambda x: fwd(x, ff), x0, dy).to(dy.dtype)


Conv2DBackpropInput = Conv2DTranspose


class Conv2DBackFilter(Operation):
    """TF ``Conv2DBackpropFilter``: Table(input, filter_sizes, out_backprop) → filter gradient
    [kh, kw, Cin, Cout] (``NNOps.scala:170``)."""

    def __init__(self, strides=(1, 1, 1, 1), padding="SAME", data_format="NHWC", dilations=(1, 1, 1, 1)):
        super().__init__()
        self.strides, self.padding, self.format = list(strides), padding, data_format
        self.dilations = list(dilations or (1, 1, 1, 1))

    def updateOutput(self, t):
        x, sizes, dy = _vals(t)[:3]
        fwd = _conv2d_fwd(self.strides, self.padding, self.format, self.dilations)
        f0 = torch.zeros(_ints(sizes), dtype=torch.float32)
        xf = x.float()
        return _vjp(lambda f: fwd(xf, f), f0, dy).to(dy.dtype)


Conv2DBackpropFilter = Conv2DBackFilter


def _pads3(size, k, s, padding):
    if padding == "VALID":
        return 0, 0
    out = -(-size // s)
    total = max((out - 1) * s + k - size, 0)
    return total // 2, total - total // 2


class Conv3D(Operation):
    """TF ``Conv3D``: Table(input N D H W C, filter [kd, kh, kw, Cin, Cout]) with TF strides /
    padding (``NNOps.scala:248``; NDHWC only, like the reference)."""

    def __init__(self, strides=(1, 1, 1, 1, 1), padding="SAME", data_format="NDHWC"):
        super().__init__()
        self.strides, self.padding, self.format = list(strides), padding, data_format

    def conv(self, x, f):
        ncdhw = self.format == "NCDHW"
        xc = x if ncdhw else x.permute(0, 4, 1, 2, 3)
        kd, kh, kw = f.shape[0], f.shape[1], f.shape[2]
        sd, sh, sw = (self.strides[2:5] if ncdhw else self.strides[1:4])
        pd = _pads3(xc.shape[2], kd, sd, self.padding)
        ph = _pads3(xc.shape[3], kh, sh, self.padding)
        pw = _pads3(xc.shape[4], kw, sw, self.padding)
        xc = F.pad(xc.float(), (pw[0], pw[1], ph[0], ph[1], pd[0], pd[1]))
        y = F.conv3d(xc, f.float().permute(4, 3, 0, 1, 2), None, (sd, sh, sw))
        return y if ncdhw else y.permute(0, 2, 3, 4, 1).contiguous()

    def updateOutput(self, t):
        x, f = _vals(t)[:2]
        return self.conv(x, f).to(x.dtype if x.is_floating_point() else torch.float32)


class Conv3DBackpropInput(Conv3D):
    """V1: Table(input, filter, out_backprop) — the input tensor gives the shape."""

    def updateOutput(self, t):
        x, f, dy = _vals(t)[:3]
        ff = f.float()
        return _vjp(lambda v: self.conv(v, ff), torch.zeros(x.shape), dy).to(dy.dtype)


class Conv3DBackpropInputV2(Conv3D):
    """V2: Table(input_sizes, filter, out_backprop)."""

    def updateOutput(self, t):
        sizes, f, dy = _vals(t)[:3]
        ff = f.float()
        return _vjp(lambda v: self.conv(v, ff), torch.zeros(_ints(sizes)), dy).to(dy.dtype)


class Conv3DBackpropFilter(Conv3D):
    """V1: Table(input, filter, out_backprop) — the filter tensor gives the shape."""

    def updateOutput(self, t):
        x, f, dy = _vals(t)[:3]
        xf = x.float()
        return _vjp(lambda w: self.conv(xf, w), torch.zeros(f.shape), dy).to(dy.dtype)


class Conv3DBackpropFilterV2(Conv3D):
    """V2: Table(input, filter_sizes, out_backprop)."""

    def updateOutput(self, t):
        x, sizes, dy = _vals(t)[:3]
        xf = x.float()
        return _vjp(lambda w: self.conv(xf, w), torch.zeros(_ints(sizes)), dy).to(dy.dtype)


class DepthwiseConv2dNativeBackpropInput(Operation):
    """Table(input_sizes, filter [kh, kw, C, M], out_backprop) → input gradient."""

    def __init__(self, strides=(1, 1, 1, 1), padding="SAME", data_format="NHWC"):
        super().__init__()
        self.strides, self.padding, self.format = list(strides), padding, data_format

    def conv(self, x, f):
        from . import _tf_pads
        nhwc = self.format == "NHWC"
        xc = x.permute(0, 3, 1, 2) if nhwc else x
        sh, sw = (self.strides[1], self.strides[2]) if nhwc else (self.strides[2], self.strides[3])
        kh, kw, C, M = f.shape
        pt, pb = _tf_pads(xc.shape[2], kh, sh, self.padding)
        pl, pr = _tf_pads(xc.shape[3], kw, sw, self.padding)
        xc = F.pad(xc.float(), (pl, pr, pt, pb))
        w = f.float().permute(2, 3, 0, 1).reshape(C * M, 1, kh, kw)
        y = F.conv2d(xc, w, None, (sh, sw), groups=C)
        return y.permute(0, 2, 3, 1).contiguous() if nhwc else y

    def updateOutput(self, t):
        sizes, f, dy = _vals(t)[:3]
        ff = f.float()
        return _vjp(lambda v: self.conv(v, ff), torch.zeros(_ints(sizes)), dy).to(dy.dtype)


class DepthwiseConv2dNativeBackpropFilter(DepthwiseConv2dNativeBackpropInput):
    """Table(input, filter_sizes, out_backprop) → filter gradient [kh, kw, C, M]."""

    def updateOutput(self, t):
        x, sizes, dy = _vals(t)[:3]
        xf = x.float()
        return _vjp(lambda w: self.conv(xf, w), torch.zeros(_ints(sizes)), dy).to(dy.dtype)


# ------------------------------------------------------------------------------------------------ pooling / LRN
class MaxPoolGrad(Operation):
    """Table(orig_input, orig_output, grad) → gradient routed to each window's max
    (``NNOps.scala:771``)."""

    def __init__(self, ksize, strides, padding="VALID", data_format="NHWC"):
        super().__init__()
        from . import MaxPool
        self.pool = MaxPool(ksize, strides, padding, data_format)

    def updateOutput(self, t):
        x, _y, g = _vals(t)[:3]
        return _vjp(self.pool.updateOutput, x, g).to(g.dtype)


class AvgPoolGrad(Operation):
    """Table(orig_input_shape, grad) → input gradient of TF AvgPool (padded cells excluded from the
    mean, ``NNOps.scala:1041`` ``countIncludePad = false``)."""

    def __init__(self, ksize, strides, padding="VALID", data_format="NHWC"):
        super().__init__()
        from . import AvgPool
        self.pool = AvgPool(ksize, strides, padding, data_format)

    def updateOutput(self, t):
        shape, g = _vals(t)[:2]
        return _vjp(self.pool.updateOutput, torch.zeros(_ints(shape)), g).to(g.dtype)


class LRNGrad(Operation):
    """Table(input_grads, input_image, output_image) → gradient of TF LRN w.r.t. its input
    (``NNOps.scala:830``)."""

    def __init__(self, depth_radius=5, bias=1.0, alpha=1.0, beta=0.5):
        super().__init__()
        from . import LRN
        self.lrn = LRN(depth_radius, bias, alpha, beta)

    def updateOutput(self, t):
        g, x, _y = _vals(t)[:3]
        return _vjp(self.lrn.updateOutput, x, g).to(g.dtype)


class FusedBatchNormGrad(Operation):
    """Table(y_backprop, x, scale, reserve_1 = batch mean, reserve_2 = batch variance) →
    Table(dx, dscale, doffset, empty, empty) of training batch normalisation
    (``NNOps.scala:994``; also FusedBatchNormGradV2)."""

    def __init__(self, epsilon=1e-4, data_format="NHWC", is_training=True):
        super().__init__()
        self.epsilon, self.format, self.isTraining = epsilon, data_format, is_training

    def updateOutput(self, t):
        dy, x, scale, mean, var = (v.float() for v in _vals(t)[:5])
        nchw = self.format == "NCHW"
        dims = (0, 2, 3) if nchw else (0, 1, 2)
        shape = (1, -1, 1, 1) if nchw else (1, 1, 1, -1)
        invstd = torch.rsqrt(var + self.epsilon)
        xhat = (x - mean.view(shape)) * invstd.view(shape)
        dbeta = dy.sum(dims)
        dgamma = (dy * xhat).sum(dims)
        if self.isTraining:
            m = x.numel() // x.shape[1 if nchw else -1]
            dx = scale.view(shape) * invstd.view(shape) * (dy - dbeta.view(shape) / m - xhat * dgamma.view(shape) / m)
        else:
            dx = dy * (scale * invstd).view(shape)
        e = torch.zeros(0)
        return Table(dx, dgamma, dbeta, e, e)


FusedBatchNormGradV2 = FusedBatchNormGrad


# ------------------------------------------------------------------------------------------------ dilation / resize
class Dilation2DBackpropInput(Operation):
    """Table(input, filter, out_backprop) → input gradient of grayscale dilation (the gradient goes
    to each window's arg-max)."""

    def __init__(self, strides=(1, 1, 1, 1), rates=(1, 1, 1, 1), padding="VALID"):
        super().__init__()
        from ..ops import Dilation2D
        self.dil = Dilation2D(strides, rates, padding)

    def updateOutput(self, t):
        x, f, g = _vals(t)[:3]
        ff = f.float()
        return _vjp(lambda v: self.dil.updateOutput(Table(v, ff)), x, g).to(g.dtype)


class Dilation2DBackpropFilter(Dilation2DBackpropInput):
    """Table(input, filter, out_backprop) → filter gradient."""

    def updateOutput(self, t):
        x, f, g = _vals(t)[:3]
        xf = x.float()
        return _vjp(lambda w: self.dil.updateOutput(Table(xf, w)), f, g).to(g.dtype)


class ResizeBilinearGrad(Operation):
    """Table(grads, original_image) → gradient w.r.t. the original image."""

    def __init__(self, align_corners=False):
        super().__init__()
        self.alignCorners = align_corners

    def updateOutput(self, t):
        g, img = _vals(t)[:2]
        size = [g.shape[1], g.shape[2]]

        from ...ops.reference import resize_bilinear

        def fwd(x):
            return resize_bilinear(x.permute(0, 3, 1, 2), size[0], size[1], self.alignCorners).permute(0, 2, 3, 1)
        return _vjp(fwd, img, g).to(g.dtype if g.is_floating_point() else torch.float32)


# ------------------------------------------------------------------------------------------------ parsing
class ParseSingleExample(Operation):
    """Parse ONE serialised ``tf.train.Example`` (``ParsingOps.scala:93``): input Table(serialized,
    dense_default_1, …); output Table(sparse_indices…, sparse_values…, sparse_shapes…, dense…) in
    TF's order.  ``dense_keys`` / ``dense_types`` / ``dense_shapes`` name the dense features,
    ``sparse_keys`` / ``sparse_types`` the sparse ones (as 1-D index / value / shape triples)."""

    def __init__(self, dense_keys: Sequence[str], dense_types: Sequence[torch.dtype],
                 dense_shapes: Sequence[Sequence[int]], sparse_keys: Sequence[str] = (),
                 sparse_types: Sequence[torch.dtype] = ()):
        super().__init__()
        self.denseKeys, self.denseTypes = list(dense_keys), list(dense_types)
        self.denseShapes = [list(s) for s in dense_shapes]
        self.sparseKeys, self.sparseTypes = list(sparse_keys), list(sparse_types)

    @staticmethod
    def _feature(ex, key):
        f = ex.features.feature[key] if key in ex.features.feature else None
        if f is None:
            return None, None
        kind = f.WhichOneof("kind")
        return kind, (list(getattr(f, kind).value) if kind else [])

    def updateOutput(self, t):
        from ...utils.tf.proto import example_classes
        vals = _vals(t)
        rec = vals[0]
        if isinstance(rec, torch.Tensor):
            rec = bytes(rec.to(torch.uint8).tolist())
        elif isinstance(rec, (list, tuple)):
            rec = rec[0]
        defaults = vals[1:]
        ex = example_classes()["tensorflow.Example"].FromString(rec)
        idx, val, shp = [], [], []
        for k, dt in zip(self.sparseKeys, self.sparseTypes):
            kind, v = self._feature(ex, k)
            v = v or []
            idx.append(torch.arange(len(v), dtype=torch.int64).view(-1, 1))
            val.append(v if kind == "bytes_list" else torch.tensor(v, dtype=dt))
            shp.append(torch.tensor([len(v)], dtype=torch.int64))
        dense = []
        for j, (k, dt, sh) in enumerate(zip(self.denseKeys, self.denseTypes, self.denseShapes)):
            kind, v = self._feature(ex, k)
            if kind is None:
                if j >= len(defaults) or defaults[j] is None or (isinstance(defaults[j], torch.Tensor)
                                                                 and defaults[j].numel() == 0):
                    raise ValueError(f"ParseSingleExample: feature '{k}' is required but missing")
                dense.append(defaults[j])
            elif kind == "bytes_list":
                dense.append(v)
            else:
                dense.append(torch.tensor(v, dtype=dt).reshape(sh or [-1]))
        return Table(*(idx + val + shp + dense))


__all__ = [n for n, v in list(globals().items()) if isinstance(v, type) and issubclass(v, Operation)
           and v.__module__ == __name__]
