"""Reference implementations of every hot op, on plain torch.

These are (a) the CPU execution path (config 1 — LeNet LocalOptimizer — runs without a GPU) and
(b) the fp32 ORACLES that the native HIP kernels in ``bigdl/ops/csrc`` are tested against.
Semantics follow the reference layers cited per function.
"""
from __future__ import annotations

import ctypes
import math
from typing import Optional, Tuple

import torch
import torch.nn.functional as F
from ..utils import acc_float

aten = torch.ops.aten


# ------------------------------------------------------------------------- casts / elementwise
def zero_fill(t: torch.Tensor):
    return t.zero_()


def cast_copy(dst: torch.Tensor, src: torch.Tensor):
    dst.copy_(src.reshape(dst.shape) if src.shape != dst.shape else src)
    return dst


def relu_forward(x: torch.Tensor, threshold: float = 0.0, value: float = 0.0, inplace=False):
    """``Threshold.updateOutput`` (``DL/nn/Threshold.scala:46``): y = x > th ? x : value."""
    if threshold == 0.0 and value == 0.0:
        return torch.relu_(x) if inplace else torch.relu(x)
    y = torch.where(x > threshold, x, torch.full_like(x, value))
    if inplace:
        x.copy_(y)
        return x
    return y


def relu_backward(gy: torch.Tensor, y_or_x: torch.Tensor, threshold: float = 0.0):
    return gy * (y_or_x > threshold).to(gy.dtype)


# ------------------------------------------------------------------------- convolution
def conv2d_forward(x, w4, b, stride, pad, dilation=(1, 1), groups=1, relu=False, out=None, res=None, pad_slot=None):
    """``SpatialConvolution.updateOutput`` (``DL/nn/SpatialConvolution.scala:253-362``).

    ``w4`` is (O, I/g, kH, kW); ``pad`` is (padH, padW) after SAME resolution.  ``relu`` applies a
    fused ReLU; ``out`` (optional) receives the result (a slice of a concat output).
    """
    y = F.conv2d(x, w4.to(x.dtype), None if b is None else b.to(x.dtype), stride, pad, dilation, groups)
    if res is not None:
        y = y + res.to(y.dtype)
    if relu:
        y = torch.relu(y)
    if out is not None:
        out.copy_(y)
        return out
    return y


def conv2d_backward(gy, x, w4, stride, pad, dilation=(1, 1), groups=1, need_input=True, gw_acc=None,
                    gb_acc=None, scale=1.0, residual=None, bn_fuse=None, pad_slot=None, lazy_strided=False):
    """``SpatialConvolution.updateGradInput`` + ``accGradParameters`` (``:364-505``).

    Returns gradInput (or None); ACCUMULATES ``scale·dW`` into ``gw_acc`` (O, I/g, kH, kW view,
    fp32) and ``scale·db`` into ``gb_acc``.  ``residual`` (optional, x-shaped) is added to gradInput."""
    gy = gy.to(x.dtype)
    need_w = gw_acc is not None and scale != 0
    need_b = gb_acc is not None and scale != 0
    gi, gw, gb = aten.convolution_backward(gy, x, w4.to(x.dtype), [w4.shape[0]] if need_b else None,
                                           list(stride), list(pad), list(dilation), False, [0, 0], groups,
                                           [need_input, need_w, need_b])
    if need_w:
        gw_acc.add_(acc_float(gw), alpha=scale)
    if need_b:
        gb_acc.add_(acc_float(gb), alpha=scale)
    if residual is not None and gi is not None:
        gi = gi + as_dense(residual).to(gi.dtype)
    return gi


class StridedGrad:
    """Input gradient of a 1×1, stride-s, unpadded convolution: nonzero only at pixels (s·i, s·j),
    kept as the dense tensor ``t`` [N][C][ceil(H/s)][ceil(W/s)] of exactly those pixels.  A conv whose
    dgrad sums it as a residual reads it in its epilogue (``res_sh``/``res_sw``) — the zero-filled
    full-resolution copy is built only by :meth:`dense` when something else needs it."""
    __slots__ = ("t", "stride", "shape")

    def __init__(self, t, stride, shape):
        self.t, self.stride, self.shape = t, tuple(stride), tuple(shape)

    def dense(self):
        fmt = torch.channels_last if self.t.is_contiguous(memory_format=torch.channels_last) else \
            torch.contiguous_format
        out = torch.empty(self.shape, dtype=self.t.dtype, device=self.t.device, memory_format=fmt).zero_()
        out[:, :, ::self.stride[0], ::self.stride[1]] = self.t
        return out


class BNOut:
    """Deferred output of a training BatchNorm: y = [relu](x·coef[c] + coef[C + c]), with ``x`` the
    BN input and ``coef`` fp32 [scale; shift].  The fused ResNet block tail takes a shortcut BN's
    output this way (no ReLU) and applies it inside its own pass (ops/csrc/batchnorm.hip rcoef); in
    fp32 compute a mid-block BN + ReLU hands its output to the next conv this way (``relu``), which
    applies it in its operand prologues (bigdl.fp32.bnPrologue) — either way the activation is never
    written; :meth:`dense` builds it for any other consumer."""
    __slots__ = ("x", "coef", "shape", "relu")

    def __init__(self, x, coef, relu=False):
        self.x, self.coef, self.shape, self.relu = x, coef, tuple(x.shape), relu

    @property
    def dtype(self):
        return self.x.dtype

    @property
    def is_cuda(self):
        return self.x.is_cuda

    @property
    def device(self):
        return self.x.device

    def dim(self):
        return self.x.dim()

    def dense(self):
        C = self.shape[1]
        sc = self.coef[:C].view(1, C, *([1] * (self.x.dim() - 2)))
        sh = self.coef[C:2 * C].view(1, C, *([1] * (self.x.dim() - 2)))
        y = torch.addcmul(sh, self.x.float(), sc)  # one rounding, like the kernels' fma
        if self.relu:
            y = torch.relu(y)
        return y.to(self.x.dtype).contiguous(memory_format=torch.channels_last) if self.x.dim() == 4 \
            else y.to(self.x.dtype)


class BNGrad:
    """Deferred input gradient of a training BatchNorm: gx = A·g + B·x + Cc per channel, with ``g``
    the (ReLU-masked) gradient at the BN output, ``x`` the BN input and ``coef`` = fp32 [A; B; Cc]
    ([3][C]).  A 1×1 stride-1 conv consuming it applies the affine map while loading its backward-
    data and weight-gradient operands (conv_igemm.hip / conv_wgrad.hip AT prologues), so the
    gradient tensor is never written; :meth:`dense` builds it for any other consumer."""
    __slots__ = ("g", "x", "coef", "shape")

    def __init__(self, g, x, coef):
        self.g, self.x, self.coef, self.shape = g, x, coef, tuple(x.shape)

    @property
    def dtype(self):
        return self.g.dtype

    @property
    def is_cuda(self):
        return self.g.is_cuda

    def dense(self):
        from . import native as N
        if self.g.is_cuda and N.has("batchnorm_backward"):
            M, C = self.g.numel() // self.shape[1], self.shape[1]
            gx = torch.empty_like(self.g)
            N.check(N.lib().bigdl_bn_bwd_apply_coef(N.ptr(self.g), N.ptr(self.x), N.ptr(gx), ctypes.c_longlong(M),
                                                    ctypes.c_int(C), N.ptr(self.coef),
                                                    ctypes.c_void_p(N.stream_ptr())), "bn_bwd_apply_coef")
            return gx
        C = self.shape[1]
        sh = [1, C] + [1] * (len(self.shape) - 2)
        a, b, c = (self.coef[i * C:(i + 1) * C].view(sh) for i in range(3))
        return (a * self.g.float() + b * self.x.float() + c).to(self.g.dtype)


def as_dense(g):
    return g.dense() if isinstance(g, (StridedGrad, BNGrad)) else g


def conv_transpose2d_forward(x, w4, b, stride, pad, adj, dilation=(1, 1), groups=1):
    return F.conv_transpose2d(x, w4.to(x.dtype), None if b is None else b.to(x.dtype), stride, pad, adj, groups,
                              dilation)


# ------------------------------------------------------------------------- bilinear resize
def _resize_axis(n_in, n_out, align, device):
    """(lower, upper, lerp) per output index, the reference's sampling (ResizeBilinear.scala:266-284,
    406-412): src = dst·scale, scale = in/out or (in−1)/(out−1) with alignCorners — no half-pixel."""
    scale = (n_in - 1) / (n_out - 1) if (align and n_out > 1) else n_in / n_out
    src = torch.arange(n_out, dtype=torch.float32, device=device) * torch.tensor(scale, dtype=torch.float32)
    lo = src.to(torch.int64).clamp_max(n_in - 1)
    hi = (lo + 1).clamp_max(n_in - 1)
    return lo, hi, src - lo.to(torch.float32)


def resize_bilinear(x, oh, ow, align=False):
    """Differentiable bilinear resize of an NCHW tensor with the reference's sampling (fp32 math)."""
    y0, y1, ly = _resize_axis(x.shape[2], oh, align, x.device)
    x0, x1, lx = _resize_axis(x.shape[3], ow, align, x.device)
    xf = x if x.dtype == torch.float64 else x.float()
    top, bot = xf.index_select(2, y0), xf.index_select(2, y1)
    lx_, ly_ = lx.to(xf.dtype).view(1, 1, 1, -1), ly.to(xf.dtype).view(1, 1, -1, 1)
    t = top.index_select(3, x0) + (top.index_select(3, x1) - top.index_select(3, x0)) * lx_
    b = bot.index_select(3, x0) + (bot.index_select(3, x1) - bot.index_select(3, x0)) * lx_
    return (t + (b - t) * ly_).to(x.dtype)


# ------------------------------------------------------------------------- batch norm
def batchnorm_forward_train(x, gamma, beta, running_mean, running_var, momentum, eps, relu=False, residual=None,
                            in_bias=None, coef_out=None, bits_out=None):
    """Training BN (``SpatialBatchNormalization.updateOutputNCHWTrainFloat``, ``:1211``).

    Normalises with the biased variance, updates ``runningVar`` with the UNBIASED variance and
    momentum 0.1 by default (``DL/nn/BatchNormalization.scala:53-54, 85-88``).
    Returns (y, save_mean, save_invstd).  Optional fused residual add and ReLU (K9).
    """
    C = x.shape[1]
    dims = [d for d in range(x.dim()) if d != 1]
    xf = acc_float(x)
    n = x.numel() // C
    mean = xf.mean(dim=dims)
    var = xf.var(dim=dims, unbiased=False)
    invstd = torch.rsqrt(var + eps)
    if running_mean is not None:
        with torch.no_grad():
            unbiased = var * (n / max(n - 1, 1))
            true_mean = mean if in_bias is None else mean + acc_float(in_bias)
            running_mean.mul_(1 - momentum).add_(true_mean, alpha=momentum)
            running_var.mul_(1 - momentum).add_(unbiased, alpha=momentum)
    shape = [1, C] + [1] * (x.dim() - 2)
    g = acc_float(gamma).view(shape) if gamma is not None else 1.0
    bb = acc_float(beta).view(shape) if beta is not None else 0.0
    if coef_out is not None:
        sc = invstd * (acc_float(gamma) if gamma is not None else 1.0)
        coef_out[:C].copy_(sc)
        coef_out[C:2 * C].copy_((acc_float(beta) if beta is not None else 0.0) - mean * sc)
    y = (xf - mean.view(shape)) * invstd.view(shape) * g + bb
    if residual is not None:
        y = y + acc_float(residual)
    if relu:
        y = torch.relu(y)
    y = y.to(x.dtype)
    if bits_out is not None and relu and x.dim() == 4 and C % 8 == 0:
        # ReLU mask bits in NHWC chunk order: byte (pixel·C + c) / 8, bit c % 8
        pos = (y.permute(0, 2, 3, 1).reshape(-1, 8) > 0).to(torch.int32)
        w = (2 ** torch.arange(8, device=y.device, dtype=torch.int32)).view(1, 8)
        bits_out.copy_((pos * w).sum(1).to(torch.uint8))
    return y, mean, invstd


def batchnorm_forward_infer(x, gamma, beta, running_mean, running_var, eps, relu=False, in_bias=None):
    """Inference BN; ``in_bias`` is a per-channel producer bias folded into this BN (x excludes it)."""
    C = x.shape[1]
    shape = [1, C] + [1] * (x.dim() - 2)
    invstd = torch.rsqrt(acc_float(running_var) + eps)
    scale = invstd * (acc_float(gamma) if gamma is not None else 1.0)
    rm = acc_float(running_mean) - (acc_float(in_bias) if in_bias is not None else 0.0)
    shift = (acc_float(beta) if beta is not None else 0.0) - rm * scale
    y = acc_float(x) * scale.view(shape) + shift.view(shape)
    if relu:
        y = torch.relu(y)
    return y.to(x.dtype)


def batchnorm_backward(gy, x, gamma, save_mean, save_invstd, y=None, relu=False, need_input=True, gg_acc=None,
                       gb_acc=None, scale=1.0, cbias_acc=None, cbias_scale=1.0, want_gres=False):
    """Returns (gradInput, gradGamma, gradBeta) — ``updateGradInputNCHWTrainFloat`` (:1048) and
    ``accGradientNCHWFloat`` (:1970).  With ``relu`` the ReLU mask is taken from ``y`` (the BN+ReLU
    output) and fused in (K7/K8)."""
    C = x.shape[1]
    dims = [d for d in range(x.dim()) if d != 1]
    shape = [1, C] + [1] * (x.dim() - 2)
    g = acc_float(gy)
    if relu:
        g = g * (y > 0).float()
    xhat = (acc_float(x) - save_mean.view(shape)) * save_invstd.view(shape)
    dbeta = g.sum(dim=dims)
    dgamma = (g * xhat).sum(dim=dims)
    gi = None
    if need_input or cbias_acc is not None:
        n = x.numel() // C
        gam = acc_float(gamma).view(shape) if gamma is not None else 1.0
        gif = (gam * save_invstd.view(shape) / n) * (n * g - dbeta.view(shape) - xhat * dgamma.view(shape))
        if cbias_acc is not None and cbias_scale != 0:
            cbias_acc.add_(gif.sum(dim=dims), alpha=cbias_scale)
        gi = gif.to(x.dtype) if need_input else None
    if gg_acc is not None and scale != 0:
        gg_acc.add_(dgamma, alpha=scale)
    if gb_acc is not None and scale != 0:
        gb_acc.add_(dbeta, alpha=scale)
    return gi, (g.to(gy.dtype) if want_gres else None)


# ---- SyncBN sums contract (native_ops.bn_local_sums & co.; the host path of P6 runs on these on
# CPU tensors, so the gloo multi-rank tests exercise exactly the collective sequence of the GPU path)
def _bn_dims(x):
    return [d for d in range(x.dim()) if d != 1], [1, x.shape[1]] + [1] * (x.dim() - 2)


def bn_local_sums(x, shift, partial=None, G=0, rezero=False):
    """[Σ(x−K), Σ(x−K)², rows] fp32 [2C + 1] with K = ``shift``."""
    C = x.shape[1]
    dims, shape = _bn_dims(x)
    if partial is not None:
        p = partial.view(2, G, C).sum(1)
        out = torch.cat([p.reshape(-1), p.new_tensor([float(x.numel() // C)])])
        if rezero:
            partial.zero_()
        return out
    # fp64 accumulation (the fp32 buffer the collective sums is the rounding of exact-ish sums: the
    # finalize's E[(x−K)²] − E[x−K]² then does not inherit fp32 summation error on large batches)
    xf = acc_float(x).double() - acc_float(shift).double().view(shape)
    out = torch.cat([xf.sum(dims), (xf * xf).sum(dims), xf.new_tensor([float(x.numel() // C)])])
    return out.to(acc_float(x).dtype if acc_float(x).dtype != torch.float64 else torch.float64)


def bn_forward_from_sums(x, sums, count, shift, gamma, beta, running_mean, running_var, momentum, eps, relu=False,
                         residual=None, in_bias=None, coef_out=None, bits_out=None, apply=True):
    """Training BN from GLOBAL shifted sums over ``count`` rows (0: ``sums[2C]``); ``apply=False``:
    finalize only (y = None, ``coef_out`` filled); ``residual`` may be a deferred :class:`BNOut`."""
    C = x.shape[1]
    dims, shape = _bn_dims(x)
    n = sums[2 * C].double() if count == 0 else torch.tensor(float(count), dtype=torch.float64, device=x.device)
    dm = sums[:C].double() / n
    var = (sums[C:2 * C].double() / n - dm * dm).clamp_min(0)
    fd = acc_float(x).dtype
    mean = (acc_float(shift).double() + dm).to(fd)
    var = var.to(fd)
    invstd = torch.rsqrt(var + eps)
    if running_mean is not None:
        with torch.no_grad():
            unb = (var.double() * n / (n - 1).clamp_min(1)).to(fd)
            tm = mean if in_bias is None else mean + acc_float(in_bias)
            running_mean.mul_(1 - momentum).add_(tm, alpha=momentum)
            running_var.mul_(1 - momentum).add_(unb, alpha=momentum)
    sc = invstd * (acc_float(gamma) if gamma is not None else 1.0)
    sh = (acc_float(beta) if beta is not None else 0.0) - mean * sc
    if coef_out is not None:
        coef_out[:C].copy_(sc)
        coef_out[C:2 * C].copy_(sh)
    if not apply:
        return None, mean, invstd
    y = acc_float(x) * sc.view(shape) + sh.view(shape)
    if isinstance(residual, BNOut):
        residual = residual.dense()
    if residual is not None:
        y = y + acc_float(residual)
    if relu:
        y = torch.relu(y)
    return y.to(x.dtype), mean, invstd


def bn_bwd_local_sums(gy, x, save_mean, y=None, relu=False):
    """[Σg', Σg'·(x − μ)] twice, then this rank's rows: fp32 [4C + 1]."""
    C = x.shape[1]
    dims, shape = _bn_dims(x)
    g = acc_float(gy)
    if relu:
        g = g * (y > 0).float()
    xc = acc_float(x) - save_mean.view(shape)
    loc = torch.cat([g.sum(dims), (g * xc).sum(dims)])
    return torch.cat([loc, loc, loc.new_tensor([float(x.numel() // C)])])


def bn_bwd_partials_sums(partial, G, C_, dev, rows=None, rezero=False):
    p = partial.view(2, G, C_).sum(1).reshape(-1)
    out = torch.cat([p, p, p.new_tensor([float(rows)])])
    if rezero:
        partial.zero_()
    return out


def bn_backward_from_sums(gy, x, gamma, save_mean, save_invstd, local_sums, global_sums, count, y=None, relu=False,
                          need_input=True, gg_acc=None, gb_acc=None, scale=1.0, cbias_acc=None, cbias_scale=1.0):
    """SyncBN backward from LOCAL (dγ/dβ of this rank) and GLOBAL (gradInput) sums."""
    C = x.shape[1]
    dims, shape = _bn_dims(x)
    n = global_sums[2 * C] if count == 0 else torch.tensor(float(count), device=x.device)
    is_ = save_invstd
    if gg_acc is not None and scale != 0:
        gg_acc.add_(local_sums[C:2 * C] * is_, alpha=scale)
    if gb_acc is not None and scale != 0:
        gb_acc.add_(local_sums[:C], alpha=scale)
    gm = acc_float(gamma) if gamma is not None else torch.ones_like(is_)
    db, dgc = global_sums[:C], global_sums[C:2 * C]
    A = gm * is_
    B = -gm * is_ * is_ * (dgc * is_) / n
    Cc = -gm * is_ * db / n - B * save_mean
    if cbias_acc is not None and cbias_scale != 0:
        m_loc = float(x.numel() // C)
        cbias_acc.add_(A * local_sums[:C] + m_loc * (B * save_mean + Cc), alpha=cbias_scale)
    if not need_input:
        return None
    g = acc_float(gy)
    if relu:
        g = g * (y > 0).float()
    gx = A.view(shape) * g + B.view(shape) * acc_float(x) + Cc.view(shape)
    return gx.to(x.dtype)


# ------------------------------------------------------------------------- pooling
def maxpool2d_forward(x, k, s, p, ceil_mode, need_indices=True):
    if not need_indices:
        return F.max_pool2d(x, k, s, p, 1, ceil_mode), None
    y, idx = F.max_pool2d(x, k, s, p, 1, ceil_mode, return_indices=True)
    return y, idx


def maxpool2d_backward(gy, x, idx, k, s, p, ceil_mode):
    if hasattr(idx, "t") and not isinstance(idx, torch.Tensor):  # native int8 argmax → recompute
        _, idx = maxpool2d_forward(x, k, s, p, ceil_mode)
    return aten.max_pool2d_with_indices_backward(gy, x, list(k), list(s), list(p), [1, 1], ceil_mode, idx)


def avgpool2d_forward(x, k, s, p, ceil_mode, count_include_pad, divisor=None):
    return F.avg_pool2d(x, k, s, p, ceil_mode, count_include_pad, divisor)


def avgpool2d_backward(gy, x, k, s, p, ceil_mode, count_include_pad, divisor=None):
    if (x.dim() == 4 and tuple(k) == tuple(x.shape[-2:]) and tuple(p) == (0, 0) and tuple(gy.shape[-2:]) == (1, 1)):
        # global average pool (ResNet / Inception heads): gx is gy / (H·W) broadcast — one copy
        # kernel instead of the generic windowed backward
        fmt = torch.channels_last if x.is_contiguous(memory_format=torch.channels_last) and not x.is_contiguous() \
            else torch.contiguous_format
        g = torch.div(gy, float(divisor or x.shape[-2] * x.shape[-1]))
        return g.expand(x.shape).contiguous(memory_format=fmt)
    return aten.avg_pool2d_backward(gy, x, list(k), list(s), list(p), ceil_mode, count_include_pad, divisor)


# ------------------------------------------------------------------------- linear
def linear_forward(x, w, b):
    """``Linear.updateOutput`` (``DL/nn/Linear.scala:108-109``): y = x Wᵀ + b."""
    y = x @ w.to(x.dtype).t()
    if b is not None:
        y = y + b.to(y.dtype)
    return y


def linear_backward(gy, x, w, need_input=True, gw_acc=None, gb_acc=None, scale=1.0):
    """``Linear.scala:128-158``: gradInput = gy·W; gradWeight += scale·gyᵀx; gradBias += scale·Σgy."""
    gi = gy @ w.to(gy.dtype) if need_input else None
    if gw_acc is not None and scale != 0:
        gw_acc.add_(acc_float(gy).t() @ acc_float(x), alpha=scale)
    if gb_acc is not None and scale != 0:
        gb_acc.add_(acc_float(gy).sum(0), alpha=scale)
    return gi


# ------------------------------------------------------------------------- softmax / criteria
def log_softmax_forward(x):
    """Row-wise log-softmax over the last dim (``DL/nn/LogSoftMax.scala:49-130``)."""
    return torch.log_softmax(acc_float(x), dim=-1).to(x.dtype)


def log_softmax_backward(gy, y):
    gyf = acc_float(gy)
    return (gyf - torch.exp(acc_float(y)) * gyf.sum(-1, keepdim=True)).to(y.dtype)


def softmax_forward(x):
    return torch.softmax(acc_float(x), dim=-1).to(x.dtype)


def softmax_backward(gy, y):
    gyf, yf = acc_float(gy), acc_float(y)
    return (yf * (gyf - (gyf * yf).sum(-1, keepdim=True))).to(y.dtype)


def class_nll_forward(logp, target_1b, weights=None, size_average=True, padding_value=-1):
    """``ClassNLLCriterion.updateOutput`` (``DL/nn/ClassNLLCriterion.scala:89-170``): 1-based
    targets, targets equal to ``paddingValue`` contribute nothing."""
    if logp.dim() == 1:
        logp = logp.unsqueeze(0)
        target_1b = target_1b.reshape(1)
    t = target_1b.long().reshape(-1)
    valid = t != padding_value
    idx = torch.where(valid, t - 1, torch.zeros_like(t))
    picked = acc_float(logp).gather(1, idx.unsqueeze(1)).squeeze(1)
    w = acc_float(weights)[idx] if weights is not None else torch.ones_like(picked)
    w = w * acc_float(valid)
    total = -(picked * w).sum()
    if size_average:
        denom = w.sum()
        total = total / torch.clamp(denom, min=1e-12) if weights is not None else total / torch.clamp(acc_float(valid).sum(), min=1)
    return total


def class_nll_backward(logp, target_1b, weights=None, size_average=True, padding_value=-1):
    squeeze = logp.dim() == 1
    lp = logp.unsqueeze(0) if squeeze else logp
    t = target_1b.long().reshape(-1)
    valid = t != padding_value
    idx = torch.where(valid, t - 1, torch.zeros_like(t))
    w = acc_float(weights)[idx] if weights is not None else torch.ones(t.shape[0], device=lp.device)
    w = w * acc_float(valid)
    if size_average:
        denom = w.sum() if weights is not None else acc_float(valid).sum()
        w = w / torch.clamp(denom, min=1e-12 if weights is not None else 1)
    g = torch.zeros(lp.shape, dtype=torch.float32, device=lp.device)
    g.scatter_(1, idx.unsqueeze(1), (-w).unsqueeze(1))
    g = g.to(logp.dtype)
    return g.squeeze(0) if squeeze else g


def cross_entropy_fused(x, target_1b, weights=None, size_average=True, padding_value=-1):
    """Fused LogSoftMax + ClassNLL (K12+K13): returns (loss, grad_x)."""
    logp = torch.log_softmax(acc_float(x), dim=-1)
    loss = class_nll_forward(logp, target_1b, weights, size_average, padding_value)
    gl = class_nll_backward(logp, target_1b, weights, size_average, padding_value).float()
    gx = gl - torch.exp(logp) * gl.sum(-1, keepdim=True)
    return loss, gx.to(x.dtype)


# ------------------------------------------------------------------------- optimizer
def sgd_step(w, g, buf, lr, momentum, dampening, weight_decay, nesterov, first_step, grad_scale=1.0,
             shadow=None, lrs=None, wds=None, first_dev=None):
    """Fused SGD (``DL/optim/SGD.scala:61-124``): g += wd·x; v = μv + (1-d)g; nesterov; x -= lr·v.

    ``grad_scale`` folds the 1/N gradient averaging in; ``lrs``/``wds`` are per-element
    learning-rate / weight-decay multipliers (``learningRates``/``weightDecays``)."""
    g = g.float()  # a bf16-wire gradient shard is consumed directly
    gg = g * grad_scale if grad_scale != 1.0 else g.clone()
    if weight_decay != 0:
        gg.add_(w * (wds if wds is not None else 1.0), alpha=weight_decay)
    if momentum != 0:
        if first_step:
            buf.copy_(gg)
        elif first_dev is not None:
            # the device-side first-step flag (graph mode) is applied on the device: no host read,
            # so this fallback stays legal inside a HIP-graph capture
            first = first_dev.reshape(-1)[:1] != 0
            buf.copy_(torch.where(first, gg, buf * momentum + (1 - dampening) * gg))
        else:
            buf.mul_(momentum).add_(gg, alpha=1 - dampening)
        if nesterov:
            gg = gg.add(buf, alpha=momentum)
        else:
            gg = buf
    if lrs is not None:
        w.add_(gg * lrs, alpha=-lr)
    else:
        w.add_(gg, alpha=-lr)
    if shadow is not None:
        shadow.copy_(w)
    return w


def adam_step(w, g, m, v, lr, beta1, beta2, eps, step, weight_decay=0.0, grad_scale=1.0, shadow=None):
    """``DL/optim/Adam.scala``: bias-corrected Adam."""
    gg = g * grad_scale
    if weight_decay != 0:
        gg = gg + weight_decay * w
    m.mul_(beta1).add_(gg, alpha=1 - beta1)
    v.mul_(beta2).addcmul_(gg, gg, value=1 - beta2)
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    step_size = lr * math.sqrt(bc2) / bc1
    w.addcdiv_(m, v.sqrt().add_(eps), value=-step_size)
    if shadow is not None:
        shadow.copy_(w)
    return w


# ------------------------------------------------------------------------- recurrent
def lstm_cell_forward(xg, hg, c_prev, h_out=None, c_out=None, act_out=None, tc_out=None):
    """Pointwise LSTM cell (``DL/nn/LSTM.scala:124-187``), gate order (i, g, f, o) along the
    last dim in blocks of H: i=σ, g=tanh, f=σ, o=σ; c' = i·g + f·c; h' = o·tanh(c').
    ``xg`` is the input projection for this step (i2g, bias included), ``hg`` the recurrent
    projection h·Uᵀ (or None); the gate sum is formed here in fp32.  Returns (h, c, act, tc):
    h in xg's dtype (written into ``h_out`` when given), c/act/tc fp32 (saved for backward)."""
    H = c_prev.shape[-1]
    gf = acc_float(xg) if hg is None else acc_float(xg) + acc_float(hg)
    i = torch.sigmoid(gf[..., 0:H])
    g = torch.tanh(gf[..., H:2 * H])
    f = torch.sigmoid(gf[..., 2 * H:3 * H])
    o = torch.sigmoid(gf[..., 3 * H:4 * H])
    c = i * g + f * acc_float(c_prev)
    tc = torch.tanh(c)
    h = (o * tc).to(xg.dtype)
    act = torch.cat([i, g, f, o], dim=-1)
    res = []
    for v, dst in ((h, h_out), (c, c_out), (act, act_out), (tc, tc_out)):
        if dst is not None:
            dst.copy_(v)
            v = dst
        res.append(v)
    return tuple(res)


def lstm_cell_backward(gh, gh2, gc_next, act, tc, c_prev, dg_out=None):
    """Backward of :func:`lstm_cell_forward`.  ``gh`` (+ ``gh2``, the recurrent gradient, when
    not None) is dL/dh', ``gc_next`` dL/dc' from the next step (or None).  Returns
    (d gates [compute dtype of gh], dc_prev fp32)."""
    H = c_prev.shape[-1]
    i, g, f, o = act[..., 0:H], act[..., H:2 * H], act[..., 2 * H:3 * H], act[..., 3 * H:]
    ghf = acc_float(gh) if gh2 is None else acc_float(gh) + acc_float(gh2)
    dc = ghf * o * (1 - tc * tc) + (acc_float(gc_next) if gc_next is not None else 0.0)
    do = ghf * tc
    di = dc * g
    dg = dc * i
    df = dc * acc_float(c_prev)
    dc_prev = dc * f
    dgates = torch.cat([di * i * (1 - i), dg * (1 - g * g), df * f * (1 - f), do * o * (1 - o)], dim=-1)
    dgates = dgates.to(gh.dtype)
    if dg_out is not None:
        dg_out.copy_(dgates)
        dgates = dg_out
    return dgates, dc_prev


# ------------------------------------------------------------------------- embedding / dropout / lrn
def embedding_forward(weight, idx_1b, padding_value=0, mask_zero=False):
    """``weight[id - 1]``; ids outside [1, nIndex] raise (``LookupTable.scala:96-98``) except the
    padding id under ``mask_zero`` (its rows are zeroed by the layer)."""
    idx = idx_1b.long() - 1
    bad = (idx < 0) | (idx >= weight.shape[0]) | (idx_1b != idx_1b.long().to(idx_1b.dtype))
    if mask_zero:
        bad &= idx_1b != padding_value
    if bool(bad.any()):
        raise IndexError(f"LookupTable: an input id is outside [1, {weight.shape[0]}] "
                         "(elements of input should be >= 1 and <= nIndex)")
    return weight[idx.clamp(min=0, max=weight.shape[0] - 1)]


def embedding_backward(grad_weight, idx_1b, gy, scale=1.0, padding_value=0):
    idx = (idx_1b.long() - 1).reshape(-1)
    g = gy.reshape(idx.numel(), -1).float() * scale
    if padding_value != 0:
        keep = (idx_1b.reshape(-1).long() != padding_value)
        idx = idx[keep]
        g = g[keep]
    grad_weight.index_add_(0, idx, g.to(grad_weight.dtype))


def dropout_forward(x, p, generator=None):
    """``DL/nn/Dropout.scala:64-150``: drop with probability p, scale kept values by 1/(1-p)."""
    if p <= 0:
        return x.clone(), None
    mask = (torch.rand(x.shape, device=x.device, generator=generator) >= p)
    scale = 1.0 / (1.0 - p)
    return x * mask.to(x.dtype) * scale, mask


def dropout_backward(gy, mask, p):
    if mask is None:
        return gy.clone()
    return gy * mask.to(gy.dtype) * (1.0 / (1.0 - p))


def lrn_forward(x, size, alpha, beta, k):
    """``SpatialCrossMapLRN`` (``DL/nn/SpatialCrossMapLRN.scala:96-200``):
    y = x / (k + α/size · Σ_{window} x²)^β."""
    return F.local_response_norm(x, size, alpha, beta, k)


def lrn_backward(gy, x, size, alpha, beta, k):
    """Gradient of :func:`lrn_forward` w.r.t. ``x`` (``SpatialCrossMapLRN.updateGradInput``)."""
    xr = x.detach().requires_grad_(True)
    with torch.enable_grad():
        y = F.local_response_norm(xr, size, alpha, beta, k)
    return torch.autograd.grad(y, xr, gy.to(y.dtype))[0]


# ------------------------------------------------------------------------- int8 (K26)
def quant_rows(x2d: torch.Tensor, kp: Optional[int] = None):
    """Per-row symmetric int8 (``Quantization.quantize``: round-half-up(v / max|row| · 127)).
    Returns (q [M][Kp] int8 zero-padded, scale [M] fp32 = max|row| / 127)."""
    M, K = x2d.shape
    kp = kp or (K + 63) // 64 * 64
    xf = acc_float(x2d)
    amax = xf.abs().amax(dim=1) if K else torch.zeros(M, device=x2d.device)
    inv = torch.where(amax > 0, 127.0 / amax, torch.zeros_like(amax))
    q = torch.floor(xf * inv[:, None] + 0.5).clamp(-127, 127).to(torch.int8)
    out = torch.zeros((M, kp), dtype=torch.int8, device=x2d.device)
    out[:, :K] = q
    return out, amax / 127.0


def gemm_i8(qa, sa, qb, sb, bias=None, out_dtype=torch.float32, relu=False):
    """C = (qa · qbᵀ) · sa[:, None] · sb[None, :] + bias, exact int32 accumulation."""
    acc = (qa.to(torch.int32) @ qb.to(torch.int32).t()) if qa.device.type == "cpu" else \
        (qa.double() @ qb.double().t())
    y = acc.double() * sa.double()[:, None] * sb.double()[None, :]
    if bias is not None:
        y = y + bias.double()[None, :]
    if relu:
        y = torch.relu(y)
    return y.to(out_dtype)


# ------------------------------------------------------------------------- image (K25)
def image_crop_flip_norm(src, oy, ox, flip, out_h, out_w, mean, std, to_rgb, out_dtype=torch.float32):
    """Batched crop + horizontal mirror + per-channel (x − mean)/std (+ BGR→RGB) of HWC images
    ``src [B, H, W, C]`` (uint8 or float) → NCHW-logical channels-last tensor of ``out_dtype``.
    ``mean``/``std`` are given in OUTPUT channel order."""
    B, H, W, C = src.shape
    outs = []
    for i in range(B):
        y, x = int(oy[i]), int(ox[i])
        t = acc_float(src[i, y:y + out_h, x:x + out_w])
        if int(flip[i]):
            t = t.flip(1)
        if to_rgb and C == 3:
            t = t.flip(2)
        outs.append(t)
    t = torch.stack(outs)
    m = torch.tensor(list(mean)[:C], dtype=torch.float32, device=src.device)
    s = torch.tensor(list(std)[:C], dtype=torch.float32, device=src.device)
    t = (t - m) / s
    return t.permute(0, 3, 1, 2).to(out_dtype)


# ------------------------------------------------------------------------- attention (K30)
_M32 = 0xFFFFFFFF


def _mul32(x, c):
    """(x · c) mod 2³² for an int64 tensor x ∈ [0, 2³²) (split so no int64 product overflows)."""
    lo, hi = x & 0xFFFF, x >> 16
    return (lo * c + (((hi * c) & 0xFFFF) << 16)) & _M32


def _amix(x):
    x = x ^ (x >> 16)
    x = _mul32(x, 0x7feb352d)
    x = x ^ (x >> 15)
    x = _mul32(x, 0x846ca68b)
    return x ^ (x >> 16)


def _seed32(seed):
    """A host seed, or the device seed snapshot a captured forward used (its low 32 bits)."""
    if isinstance(seed, torch.Tensor):
        return int(seed.reshape(-1)[0].item()) & _M32
    return int(seed) & _M32


def attention_dropout_mask(seed, B, Hh, Lq, Lk, keep, device="cpu"):
    """The attention kernels' dropout keep mask (bool [B, Hh, Lq, Lk]) — the same counter hash as
    ``attention.hip`` (akeep): bit = mix(mix(seed + (b·Hh + h)·c₁) ^ mix(q·c₂ + k)) < keep·2³²."""
    import numpy as np
    thr = min(int(float(np.float32(keep)) * 4294967296.0), _M32)
    bh = torch.arange(B * Hh, dtype=torch.int64, device=device)
    s = _amix((_seed32(seed) + _mul32(bh, 0x85EBCA77)) & _M32).view(B, Hh, 1, 1)
    q = torch.arange(Lq, dtype=torch.int64, device=device).view(Lq, 1)
    k = torch.arange(Lk, dtype=torch.int64, device=device).view(1, Lk)
    inner = _amix((_mul32(q, 0x9E3779B1) + k) & _M32).view(1, 1, Lq, Lk)
    return _amix(s ^ inner) < thr


def _heads(t, B, L, Hh, D):
    return acc_float(t[:, :Hh * D]).reshape(B, L, Hh, D).transpose(1, 2)


def _attn_probs(q, k, B, Hh, Lq, Lk, D, scale, bias, causal):
    s = (_heads(q, B, Lq, Hh, D) @ _heads(k, B, Lk, Hh, D).transpose(-1, -2)) * scale
    if bias is not None:
        s = s + acc_float(bias)
    if causal:
        s = s.masked_fill(torch.ones(Lq, Lk, dtype=torch.bool, device=s.device).triu(1), float("-inf"))
    return s


def attention_decode(q, kc, vc, L, Hh, D, scale, bias=None, bias_rev=True):
    """Cached decoding attention over the first ``L`` cache positions (Attention.scala:118-140):
    softmax(scale·q·kᵀ + bias)·v per head; ``bias_rev``: bias indexed newest key first."""
    rows, Lq, H = q.shape
    qh = q.float().reshape(rows, Lq, Hh, D).transpose(1, 2)
    kh = kc[:, :L].float().reshape(rows, L, Hh, D).transpose(1, 2)
    vh = vc[:, :L].float().reshape(rows, L, Hh, D).transpose(1, 2)
    s = (qh @ kh.transpose(-1, -2)) * scale
    if bias is not None:
        b = bias.float()
        s = s + (b.flip(-1) if bias_rev else b)
    o = torch.softmax(s, -1) @ vh
    return o.transpose(1, 2).reshape(rows, Lq, H).to(q.dtype)


def attention_forward(q, k, v, B, Hh, Lq, Lk, D, scale, bias=None, causal=False, keep=1.0, seed=0):
    """Multi-head attention on projection rows (``Attention.scala:30-111``): q [B·Lq][≥Hh·D],
    k / v [B·Lk][≥Hh·D] with head h at columns h·D; O = (softmax(scale·QKᵀ + bias [causal]) ∘ M /
    keep)·V with the kernels' dropout mask M when keep < 1.  Returns (o [B·Lq][Hh·D] in q's
    dtype, lse₂ fp32 [B][Hh][Lq] = log2 Σ exp of the logits)."""
    s = _attn_probs(q, k, B, Hh, Lq, Lk, D, scale, bias, causal)
    lse2 = torch.logsumexp(s, -1) / math.log(2.0)
    p = torch.softmax(s, -1)
    if keep < 1.0:
        p = p * attention_dropout_mask(seed, B, Hh, Lq, Lk, keep, s.device).to(p.dtype) / keep
    o = p @ _heads(v, B, Lk, Hh, D)
    return o.transpose(1, 2).reshape(B * Lq, Hh * D).to(q.dtype), lse2


def attention_backward(dout, q, k, v, o, lse, B, Hh, Lq, Lk, D, scale, bias=None, causal=False, keep=1.0, seed=0,
                       dq=None, dk=None, dv=None):
    """(dq, dk, dv), each [B·L][Hh·D] in q's dtype, of :func:`attention_forward` (recomputed in fp32
    through autograd; ``o`` / ``lse`` are accepted for signature parity with the kernel).  Given
    ``dq``/``dk``/``dv`` (e.g. column slices of one fused buffer) receive the results."""
    qf = _heads(q, B, Lq, Hh, D).detach().requires_grad_(True)
    kf = _heads(k, B, Lk, Hh, D).detach().requires_grad_(True)
    vf = _heads(v, B, Lk, Hh, D).detach().requires_grad_(True)
    with torch.enable_grad():
        s = (qf @ kf.transpose(-1, -2)) * scale
        if bias is not None:
            s = s + acc_float(bias)
        if causal:
            s = s.masked_fill(torch.ones(Lq, Lk, dtype=torch.bool, device=s.device).triu(1), float("-inf"))
        p = torch.softmax(s, -1)
        if keep < 1.0:
            p = p * attention_dropout_mask(seed, B, Hh, Lq, Lk, keep, s.device).to(p.dtype) / keep
        out = p @ vf
    g = _heads(dout, B, Lq, Hh, D)
    dq_out, dk_out, dv_out = dq, dk, dv
    dq, dk, dv = torch.autograd.grad(out, (qf, kf, vf), g)
    res = []
    for t, L, dst in ((dq, Lq, dq_out), (dk, Lk, dk_out), (dv, Lk, dv_out)):
        r = t.transpose(1, 2).reshape(B * L, Hh * D).to(q.dtype)
        if dst is not None:
            dst.copy_(r)
            r = dst
        res.append(r)
    return tuple(res)
