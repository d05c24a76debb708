"""Python wrappers for the native HIP kernels.

Every wrapper checks dtype / layout / alignment / sizes on the host before launching and returns
``NotImplemented`` for configurations the kernel does not cover (the dispatcher then uses the
reference op).  No wrapper launches a kernel whose shape assumptions were not verified here.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import torch

from . import native as N
from .native import register, ptr, stream_ptr, check

_bf16 = torch.bfloat16
_f32 = torch.float32


def _al16(t: Optional[torch.Tensor]) -> bool:
    return t is None or t.data_ptr() % 16 == 0


def _dense(t: torch.Tensor) -> bool:
    """Memory is one dense block in NHWC (channels_last) or row-major order."""
    if t.dim() == 4:
        return t.is_contiguous(memory_format=torch.channels_last)
    return t.is_contiguous()


def _rows_c(t: torch.Tensor):
    """(M rows, C channels) of a channels-last 4-D or contiguous 2-D activation, else None."""
    if t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last):
        n, c, h, w = t.shape
        return n * h * w, c
    if t.dim() == 2 and t.is_contiguous():
        return t.shape[0], t.shape[1]
    return None


def _lib():
    return N.lib()


def _s():
    return C.c_void_p(stream_ptr())


def _f(x):
    return C.c_float(float(x))


def _ll(x):
    return C.c_longlong(int(x))


# ------------------------------------------------------------------------------------------------ casts
@register("cast_copy")
def cast_copy(dst, src):
    if not (dst.is_cuda and src.is_cuda and dst.numel() == src.numel()):
        return NotImplemented
    if not (dst.is_contiguous() and src.is_contiguous() and _al16(dst) and _al16(src)):
        return NotImplemented
    if dst.dtype == _bf16 and src.dtype == _f32:
        mode = 0
    elif dst.dtype == _f32 and src.dtype == _bf16:
        mode = 1
    else:
        return NotImplemented
    check(_lib().bigdl_cast(ptr(src), ptr(dst), _ll(src.numel()), C.c_int(mode), _s()), "cast")
    return dst


# ------------------------------------------------------------------------------------------------ relu
@register("relu_forward")
def relu_forward(x, threshold=0.0, value=0.0, inplace=False):
    if x.dtype != _bf16 or not _dense(x) or x.numel() % 8 or not _al16(x):
        return NotImplemented
    y = x if inplace else torch.empty_like(x)
    check(_lib().bigdl_threshold_fwd_bf16(ptr(x), ptr(y), _ll(x.numel()), _f(threshold), _f(value), _s()),
          "threshold_fwd")
    return y


@register("relu_backward")
def relu_backward(gy, ref, threshold=0.0):
    if gy.dtype != _bf16 or ref.dtype != _bf16 or gy.shape != ref.shape:
        return NotImplemented
    if not (_dense(gy) and _dense(ref)) or gy.stride() != ref.stride() or gy.numel() % 8:
        return NotImplemented
    if not (_al16(gy) and _al16(ref)):
        return NotImplemented
    gx = torch.empty_like(gy)
    check(_lib().bigdl_threshold_bwd_bf16(ptr(gy), ptr(ref), ptr(gx), _ll(gy.numel()), _f(threshold), _s()),
          "threshold_bwd")
    return gx


# ------------------------------------------------------------------------------------------------ batchnorm
def _bn_ok(x, C_):
    return x.dtype == _bf16 and C_ % 8 == 0 and _al16(x) and C_ <= 8192


def _f32vec(t, C_):
    return t is None or (t.dtype == _f32 and t.is_contiguous() and t.numel() == C_ and t.is_cuda)


@register("batchnorm_forward_train")
def batchnorm_forward_train(x, gamma, beta, running_mean, running_var, momentum, eps, relu=False, residual=None,
                            in_bias=None):
    rc = _rows_c(x)
    if rc is None:
        return NotImplemented
    M, C_ = rc
    if not _bn_ok(x, C_) or not all(_f32vec(t, C_) for t in (gamma, beta, running_mean, running_var, in_bias)):
        return NotImplemented
    if residual is not None and (residual.shape != x.shape or residual.stride() != x.stride() or
                                 residual.dtype != _bf16 or not _al16(residual)):
        return NotImplemented
    lib = _lib()
    G = lib.bigdl_bn_num_partials(_ll(M), C.c_int(C_))
    ws = torch.empty(2 * G * C_, dtype=_f32, device=x.device)
    coef = torch.empty(2 * C_, dtype=_f32, device=x.device)
    mean = torch.empty(C_, dtype=_f32, device=x.device)
    invstd = torch.empty(C_, dtype=_f32, device=x.device)
    y = torch.empty_like(x)
    check(lib.bigdl_bn_fwd_train(ptr(x), ptr(residual), ptr(y), _ll(M), C.c_int(C_), ptr(gamma), ptr(beta),
                                 ptr(in_bias), ptr(running_mean), ptr(running_var), _f(momentum), _f(eps), ptr(mean),
                                 ptr(invstd), ptr(ws), ptr(coef), C.c_int(1 if relu else 0), _s()), "bn_fwd_train")
    return y, mean, invstd


@register("batchnorm_forward_infer")
def batchnorm_forward_infer(x, gamma, beta, running_mean, running_var, eps, relu=False, in_bias=None):
    rc = _rows_c(x)
    if rc is None:
        return NotImplemented
    M, C_ = rc
    if not _bn_ok(x, C_) or not all(_f32vec(t, C_) for t in (gamma, beta, running_mean, running_var, in_bias)):
        return NotImplemented
    coef = torch.empty(2 * C_, dtype=_f32, device=x.device)
    y = torch.empty_like(x)
    check(_lib().bigdl_bn_fwd_infer(ptr(x), ptr(y), _ll(M), C.c_int(C_), ptr(gamma), ptr(beta), ptr(running_mean),
                                    ptr(running_var), ptr(in_bias), _f(eps), ptr(coef), C.c_int(1 if relu else 0),
                                    _s()), "bn_fwd_infer")
    return y


@register("batchnorm_backward")
def batchnorm_backward(gy, x, gamma, save_mean, save_invstd, y=None, relu=False, need_input=True, gg_acc=None,
                       gb_acc=None, scale=1.0, cbias_acc=None, cbias_scale=1.0, want_gres=False):
    """Returns (gradInput or None, g' or None).  g' is the masked upstream gradient for a fused
    residual branch (``want_gres``); ``cbias_acc`` receives the gradient of a folded producer bias."""
    rc = _rows_c(x)
    if rc is None:
        return NotImplemented
    M, C_ = rc
    if not _bn_ok(x, C_) or gy.dtype != _bf16 or gy.shape != x.shape or gy.stride() != x.stride() or not _al16(gy):
        return NotImplemented
    if relu and (y is None or y.dtype != _bf16 or y.stride() != x.stride() or not _al16(y)):
        return NotImplemented
    if not all(_f32vec(t, C_) for t in (gamma, save_mean, save_invstd, gg_acc, gb_acc, cbias_acc)):
        return NotImplemented
    lib = _lib()
    G = lib.bigdl_bn_num_partials(_ll(M), C.c_int(C_))
    ws = torch.empty(2 * G * C_, dtype=_f32, device=x.device)
    coef = torch.empty(3 * C_, dtype=_f32, device=x.device)
    gx = torch.empty_like(x) if need_input else None
    gres = torch.empty_like(x) if want_gres else None
    check(lib.bigdl_bn_bwd(ptr(gy), ptr(x), ptr(y if relu else None), ptr(gx), ptr(gres), _ll(M), C.c_int(C_),
                           ptr(gamma), ptr(save_mean), ptr(save_invstd), ptr(gg_acc), ptr(gb_acc), _f(scale),
                           ptr(cbias_acc), _f(cbias_scale), ptr(ws), ptr(coef), C.c_int(1 if relu else 0), _s()),
          "bn_bwd")
    return gx, gres


# ------------------------------------------------------------------------------------------------ softmax / CE
def _targets_i32(target_1b, B):
    t = target_1b.reshape(-1)
    if t.numel() != B:
        return None
    return t.to(torch.int32).contiguous()


@register("cross_entropy_fused")
def cross_entropy_fused(x, target_1b, weights=None, size_average=True, padding_value=-1):
    if x.dim() != 2 or not x.is_contiguous() or x.dtype not in (_bf16, _f32):
        return NotImplemented
    B, K = x.shape
    t = _targets_i32(target_1b.to(x.device), B)
    if t is None:
        return NotImplemented
    w = None
    if weights is not None:
        w = weights.to(x.device, _f32).contiguous()
        if w.numel() != K:
            return NotImplemented
    ws = torch.empty(3 * B, dtype=_f32, device=x.device)
    out = torch.empty(2, dtype=_f32, device=x.device)
    gx = torch.empty_like(x)
    check(_lib().bigdl_cross_entropy(ptr(x), ptr(t), ptr(w), ptr(gx), _ll(B), C.c_int(K), C.c_int(int(padding_value)),
                                     C.c_int(1 if size_average else 0), C.c_int(1 if x.dtype == _bf16 else 0),
                                     ptr(ws), ptr(out), _s()), "cross_entropy")
    return out[0], gx


@register("log_softmax_forward")
def log_softmax_forward(x):
    if not x.is_contiguous() or x.dtype not in (_bf16, _f32) or x.dim() < 1 or x.numel() == 0:
        return NotImplemented
    K = x.shape[-1]
    rows = x.numel() // K
    y = torch.empty_like(x)
    check(_lib().bigdl_logsoftmax(ptr(x), ptr(None), ptr(y), _ll(rows), C.c_int(K), C.c_int(0),
                                  C.c_int(1 if x.dtype == _bf16 else 0), _s()), "logsoftmax")
    return y


@register("log_softmax_backward")
def log_softmax_backward(gy, y):
    if not (gy.is_contiguous() and y.is_contiguous()) or gy.dtype != y.dtype or y.dtype not in (_bf16, _f32) \
            or gy.shape != y.shape:
        return NotImplemented
    K = y.shape[-1]
    rows = y.numel() // K
    gx = torch.empty_like(y)
    check(_lib().bigdl_logsoftmax(ptr(gy), ptr(y), ptr(gx), _ll(rows), C.c_int(K), C.c_int(1),
                                  C.c_int(1 if y.dtype == _bf16 else 0), _s()), "logsoftmax_bwd")
    return gx


# ------------------------------------------------------------------------------------------------ optimizers
def _vec_ok(*ts, n):
    for t in ts:
        if t is None:
            continue
        if not (t.is_cuda and t.is_contiguous() and t.numel() == n and _al16(t)):
            return False
    return True


@register("sgd_step")
def sgd_step(w, g, buf, lr, momentum, dampening, weight_decay, nesterov, first_step, grad_scale=1.0, shadow=None,
             lrs=None, wds=None):
    n = w.numel()
    if w.dtype != _f32 or g.dtype != _f32 or n % 4 or not _vec_ok(w, g, buf, lrs, wds, n=n):
        return NotImplemented
    if shadow is not None and not (shadow.dtype == _bf16 and shadow.is_contiguous() and shadow.numel() == n
                                   and shadow.data_ptr() % 8 == 0):
        return NotImplemented
    if momentum != 0 and buf is None:
        return NotImplemented
    check(_lib().bigdl_sgd(ptr(w), ptr(g), ptr(buf if momentum != 0 else None), ptr(shadow), ptr(lrs), ptr(wds),
                           _ll(n), _f(lr), _f(momentum), _f(dampening), _f(weight_decay), C.c_int(int(bool(nesterov))),
                           C.c_int(int(bool(first_step))), _f(grad_scale), _s()), "sgd")
    return w


@register("adam_step")
def adam_step(w, g, m, v, lr, beta1, beta2, eps, step, weight_decay=0.0, grad_scale=1.0, shadow=None):
    import math
    n = w.numel()
    if w.dtype != _f32 or n % 4 or not _vec_ok(w, g, m, v, n=n):
        return NotImplemented
    if shadow is not None and not (shadow.dtype == _bf16 and shadow.is_contiguous() and shadow.data_ptr() % 8 == 0):
        return NotImplemented
    step_size = lr * math.sqrt(1 - beta2 ** step) / (1 - beta1 ** step)
    check(_lib().bigdl_adam(ptr(w), ptr(g), ptr(m), ptr(v), ptr(shadow), _ll(n), _f(step_size), _f(beta1), _f(beta2),
                            _f(eps), _f(weight_decay), _f(grad_scale), _s()), "adam")
    return w
