"""Python wrappers for the native HIP kernels.

Every wrapper checks dtype / layout / alignment / sizes on the host before launching and returns
``NotImplemented`` for configurations the kernel does not cover (the dispatcher then uses the
reference op).  No wrapper launches a kernel whose shape assumptions were not verified here.
"""
from __future__ import annotations

import contextlib
import ctypes as C
from typing import Optional

import torch

from . import native as N
from . import reference as R_
from . import fp32x3 as F3
from ..utils import config
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
@register("zero_fill")
def zero_fill(t):
    """t[:] = 0 for a contiguous 32-bit device tensor (the per-step gradient-arena clear) with the
    native 16-B store kernel, so no torch fill kernel runs in the training step."""
    if not (t.is_cuda and t.is_contiguous() and t.element_size() == 4 and _al16(t)) or not hasattr(_lib(), "bigdl_fill32"):
        return NotImplemented
    check(_lib().bigdl_fill32(ptr(t), _ll(t.numel()), C.c_uint32(0), _s()), "fill32")
    return t


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
    if not _dense(x) or not _al16(x):
        return NotImplemented
    if x.dtype == _f32:  # the reference's precision (DL/nn/Threshold.scala:46-421)
        y = x if inplace else torch.empty_like(x)
        check(_lib().bigdl_threshold_fwd_f32(ptr(x), ptr(y), _ll(x.numel()), _f(threshold), _f(value), _s()),
              "threshold_fwd_f32")
        return y
    if x.dtype != _bf16 or x.numel() % 8:
        return NotImplemented
    y = x if inplace else torch.empty_like(x)
    check(_lib().bigdl_threshold_fwd_bf16(ptr(x), ptr(y), _ll(x.numel()), _f(threshold), _f(value), _s()),
          "threshold_fwd")
    return y


@register("relu_backward")
def relu_backward(gy, ref, threshold=0.0):
    if gy.dtype != ref.dtype or gy.dtype not in (_bf16, _f32) or gy.shape != ref.shape:
        return NotImplemented
    if not (_dense(gy) and _dense(ref)) or gy.stride() != ref.stride():
        return NotImplemented
    if not (_al16(gy) and _al16(ref)):
        return NotImplemented
    gx = torch.empty_like(gy)
    if gy.dtype == _f32:
        check(_lib().bigdl_threshold_bwd_f32(ptr(gy), ptr(ref), ptr(gx), _ll(gy.numel()), _f(threshold), _s()),
              "threshold_bwd_f32")
        return gx
    if gy.numel() % 8:
        return NotImplemented
    check(_lib().bigdl_threshold_bwd_bf16(ptr(gy), ptr(ref), ptr(gx), _ll(gy.numel()), _f(threshold), _s()),
          "threshold_bwd")
    return gx


# ------------------------------------------------------------------------------------------------ batchnorm
def _bn_ok(x, C_):
    return x.dtype == _bf16 and C_ % 8 == 0 and _al16(x) and C_ <= 8192


def _f32vec(t, C_):
    return t is None or (t.dtype == _f32 and t.is_contiguous() and t.numel() == C_ and t.is_cuda)


def _bn32_ok(x, C_, *more):
    """fp32 NHWC tensors of the fp32 compute mode (csrc/batchnorm.hip k_bn32_*)."""
    return (x.dtype == _f32 and C_ % 8 == 0 and C_ <= 8192 and _al16(x) and F3.enabled(x)
            and all(t is None or (t.dtype == _f32 and t.shape == x.shape and t.stride() == x.stride() and _al16(t))
                    for t in more))


@register("batchnorm_forward_train")
def batchnorm_forward_train(x, gamma, beta, running_mean, running_var, momentum, eps, relu=False, residual=None,
                            in_bias=None, coef_out=None, bits_out=None):
    rc = _rows_c(x)
    if rc is None:
        return NotImplemented
    M, C_ = rc
    if _bn32_ok(x, C_, residual) and all(_f32vec(t, C_) for t in (gamma, beta, running_mean, running_var, in_bias)):
        G = _lib().bigdl_bn_num_partials(_ll(M), C.c_int(C_))
        ws = torch.empty(2 * G * C_, dtype=_f32, device=x.device)
        coef = coef_out if _coef_ok(coef_out, C_) else torch.empty(2 * C_, dtype=_f32, device=x.device)
        mean = torch.empty(C_, dtype=_f32, device=x.device)
        invstd = torch.empty(C_, dtype=_f32, device=x.device)
        y = torch.empty_like(x)
        sp = F3.split_buffer(M, C_, x.device)  # the next conv's [hi | lo] operand, written by the apply pass
        mb = torch.empty(M * (C_ // 8), dtype=torch.uint8, device=x.device) if relu else None  # ReLU mask bits
        check(_lib().bigdl_bn32_fwd_train(ptr(x), ptr(residual), ptr(y), _ll(M), C.c_int(C_), ptr(gamma), ptr(beta),
                                          ptr(in_bias), ptr(running_mean), ptr(running_var), _f(momentum), _f(eps),
                                          ptr(mean), ptr(invstd), ptr(ws), ptr(coef), C.c_int(1 if relu else 0),
                                          ptr(sp), ptr(mb), _s()), "bn32_fwd_train")
        F3.note_split(y, sp, mb)
        return y, mean, invstd
    if not _bn_ok(x, C_) or not all(_f32vec(t, C_) for t in (gamma, beta, running_mean, running_var, in_bias)):
        return NotImplemented
    if residual is not None and (residual.shape != x.shape or residual.stride() != x.stride() or
                                 residual.dtype != _bf16 or not _al16(residual)):
        return NotImplemented
    lib = _lib()
    G = lib.bigdl_bn_num_partials(_ll(M), C.c_int(C_))
    ws = torch.empty(2 * G * C_, dtype=_f32, device=x.device)
    coef = coef_out if _coef_ok(coef_out, C_) else torch.empty(2 * C_, dtype=_f32, device=x.device)
    mean = torch.empty(C_, dtype=_f32, device=x.device)
    invstd = torch.empty(C_, dtype=_f32, device=x.device)
    y = torch.empty_like(x)
    check(lib.bigdl_bn_fwd_train(ptr(x), ptr(residual), ptr(y), _ll(M), C.c_int(C_), ptr(gamma), ptr(beta),
                                 ptr(in_bias), ptr(running_mean), ptr(running_var), _f(momentum), _f(eps), ptr(mean),
                                 ptr(invstd), ptr(ws), ptr(coef), C.c_int(1 if relu else 0),
                                 ptr(_bits_ok(bits_out, M, C_, relu)), _s()), "bn_fwd_train")
    return y, mean, invstd


def _bits_ok(bits, M, C_, relu):
    """The ReLU-mask byte buffer (M·C/8 uint8) if usable, else None."""
    if bits is None or not relu:
        return None
    if bits.dtype != torch.uint8 or not bits.is_contiguous() or bits.numel() != M * C_ // 8 or not bits.is_cuda:
        return None
    return bits


def _fold_scratch(G, C_, dev):
    f = N._load().bigdl_bn_fold_scratch  # the raw CDLL symbol (restype must stick)
    f.restype = C.c_longlong
    n = f(C.c_int(G), C.c_int(C_))
    return torch.empty(n, dtype=_f32, device=dev) if n > 0 else None


def _coef_ok(t, C_):
    return t is not None and t.dtype == _f32 and t.is_contiguous() and t.numel() >= 2 * C_ and t.is_cuda


def batchnorm_forward_train_partials(x, partial, G, gamma, beta, running_mean, running_var, momentum, eps,
                                    relu=False, residual=None, in_bias=None, coef_out=None, shift=None, bits_out=None,
                                    rezero=False, zero_next=None, mean_out=None, apply=True):
    """Training BN whose statistics were produced by the preceding conv's epilogue
    (:func:`conv2d_forward_stats`): finalize + apply only.  ``rezero``: ``partial`` is a replicated
    atomic-statistics buffer ([2][G][C], G replicas) that the finalize clears after reading.
    ``apply=False``: finalize only (coef_out required) and y = None — the caller defers the apply;
    ``residual`` may be such a deferred BN output (:class:`~bigdl.ops.reference.BNOut`), applied
    inside this BN's pass."""
    rc = _rows_c(x)
    if rc is None:
        return NotImplemented
    M, C_ = rc
    deferred = isinstance(residual, R_.BNOut)
    if (not apply and not deferred and residual is None and rezero and 1 <= G <= 512 and _bn32_ok(x, C_, None)
            and partial is not None and partial.dtype == _f32 and partial.numel() == 2 * G * C_
            and _f32vec(shift, C_) and _coef_ok(coef_out, C_)
            and all(_f32vec(t, C_) for t in (gamma, beta, running_mean, running_var, in_bias))):
        # fp32 compute, finalize only: the consuming conv applies BN + ReLU in its operand prologues
        # (bigdl.fp32.bnPrologue), so the BN output is never written
        mean = torch.empty(C_, dtype=_f32, device=x.device)
        invstd = torch.empty(C_, dtype=_f32, device=x.device)
        check(_lib().bigdl_bn32_fwd_train_partials(ptr(x), None, None, _ll(M), C.c_int(C_), ptr(gamma), ptr(beta),
                                                   ptr(in_bias), ptr(running_mean), ptr(running_var), _f(momentum),
                                                   _f(eps), ptr(mean), ptr(invstd), ptr(partial), C.c_int(G),
                                                   ptr(shift), ptr(coef_out), C.c_int(1 if relu else 0), None, None,
                                                   _s()), "bn32_fwd_train_partials(finalize)")
        return None, mean, invstd
    if deferred or not apply:
        # the bf16 replicated / partial-rows path only (the fused block tail of the training step)
        if not (_bn_ok(x, C_) and all(_f32vec(t, C_) for t in (gamma, beta, running_mean, running_var, in_bias))
                and G >= 1 and partial is not None and partial.numel() == 2 * G * C_ and partial.dtype == _f32
                and (not rezero or G <= 512)):
            return NotImplemented
        if deferred and not (residual.x.shape == x.shape and residual.x.stride() == x.stride()
                             and residual.x.dtype == _bf16 and _al16(residual.x) and _f32vec(residual.coef, 2 * C_)):
            return NotImplemented
        if not apply and not _coef_ok(coef_out, C_):
            return NotImplemented
        coef = coef_out if _coef_ok(coef_out, C_) else torch.empty(2 * C_, dtype=_f32, device=x.device)
        mean = mean_out if (mean_out is not None and _f32vec(mean_out, C_)) else torch.empty(C_, dtype=_f32,
                                                                                               device=x.device)
        invstd = torch.empty(C_, dtype=_f32, device=x.device)
        y = torch.empty_like(x) if apply else None
        res_t, rcoef = (residual.x, residual.coef) if deferred else (residual, None)
        check(_lib().bigdl_bn_fwd_train_partials2(ptr(x), ptr(res_t), ptr(rcoef), ptr(y), _ll(M), C.c_int(C_),
                                                  ptr(gamma), ptr(beta), ptr(in_bias), ptr(running_mean),
                                                  ptr(running_var), _f(momentum), _f(eps), ptr(mean), ptr(invstd),
                                                  ptr(partial), C.c_int(G), ptr(shift if _f32vec(shift, C_) else None),
                                                  ptr(coef), C.c_int(1 if relu else 0),
                                                  ptr(_fold_scratch(G, C_, x.device)),
                                                  ptr(_bits_ok(bits_out, M, C_, relu) if apply else None),
                                                  C.c_int(1 if rezero else 0), _s()), "bn_fwd_train_partials2")
        return y, mean, invstd
    if (rezero and 1 <= G <= 512 and _bn32_ok(x, C_, residual) and partial is not None and partial.dtype == _f32
            and partial.numel() == 2 * G * C_ and _f32vec(shift, C_)
            and all(_f32vec(t, C_) for t in (gamma, beta, running_mean, running_var, in_bias))):
        # fp32 compute: the replicated sums of the fp32-output conv (fp32x3.conv_forward_stats)
        coef = coef_out if _coef_ok(coef_out, C_) else torch.empty(2 * C_, dtype=_f32, device=x.device)
        mean = torch.empty(C_, dtype=_f32, device=x.device)
        invstd = torch.empty(C_, dtype=_f32, device=x.device)
        y = torch.empty_like(x)
        sp = F3.split_buffer(M, C_, x.device)
        mb = torch.empty(M * (C_ // 8), dtype=torch.uint8, device=x.device) if relu else None
        check(_lib().bigdl_bn32_fwd_train_partials(ptr(x), ptr(residual), ptr(y), _ll(M), C.c_int(C_), ptr(gamma),
                                                   ptr(beta), ptr(in_bias), ptr(running_mean), ptr(running_var),
                                                   _f(momentum), _f(eps), ptr(mean), ptr(invstd), ptr(partial),
                                                   C.c_int(G), ptr(shift), ptr(coef), C.c_int(1 if relu else 0),
                                                   ptr(sp), ptr(mb), _s()), "bn32_fwd_train_partials")
        F3.note_split(y, sp, mb)
        return y, mean, invstd
    if not _bn_ok(x, C_) or not all(_f32vec(t, C_) for t in (gamma, beta, running_mean, running_var, in_bias)):
        return NotImplemented
    if G == 0:  # atomically accumulated sums [2C + 1] (conv epilogue, stats_atomic)
        if partial is None or partial.numel() != 2 * C_ + 1 or partial.dtype != _f32 or C_ > 8192:
            return NotImplemented
    elif partial is None or partial.numel() != 2 * G * C_ or partial.dtype != _f32:
        return NotImplemented
    if residual is not None and (residual.shape != x.shape or residual.stride() != x.stride() or
                                 residual.dtype != _bf16 or not _al16(residual)):
        return NotImplemented
    coef = coef_out if _coef_ok(coef_out, C_) else torch.empty(2 * C_, dtype=_f32, device=x.device)
    mean = mean_out if (mean_out is not None and _f32vec(mean_out, C_)) else torch.empty(C_, dtype=_f32,
                                                                                           device=x.device)
    invstd = torch.empty(C_, dtype=_f32, device=x.device)
    y = torch.empty_like(x)
    if (rezero and G >= 1 and zero_next is not None and zero_next.numel() == partial.numel() and shift is not None
            and _f32vec(shift, C_) and shift.data_ptr() not in (running_mean.data_ptr(), mean.data_ptr())
            and C_ <= 8192 and 2 * G * C_ <= 32768 and _al16(zero_next)):
        # ONE launch: each block reduces the conv's replicated statistics itself (no finalize kernel),
        # block 0 updates the running statistics and clears the next step's replica set
        check(_lib().bigdl_bn_fwd_train_rep_fin(ptr(x), ptr(residual), ptr(y), _ll(M), C.c_int(C_), ptr(gamma),
                                                ptr(beta), ptr(in_bias), ptr(running_mean), ptr(running_var),
                                                _f(momentum), _f(eps), ptr(mean), ptr(invstd), ptr(partial),
                                                C.c_int(G), ptr(zero_next), ptr(shift), ptr(coef),
                                                C.c_int(1 if relu else 0), ptr(_bits_ok(bits_out, M, C_, relu)), _s()),
              "bn_fwd_train_rep_fin")
        return y, mean, invstd
    if G == 0:
        check(_lib().bigdl_bn_fwd_train_sums_apply(ptr(x), ptr(residual), ptr(y), _ll(M), C.c_int(C_), ptr(gamma),
                                                   ptr(beta), ptr(in_bias), ptr(running_mean), ptr(running_var),
                                                   _f(momentum), _f(eps), ptr(mean), ptr(invstd), ptr(partial),
                                                   ptr(shift if _f32vec(shift, C_) else None), ptr(coef),
                                                   C.c_int(1 if relu else 0), ptr(_bits_ok(bits_out, M, C_, relu)),
                                                   _s()), "bn_fwd_train_sums_apply")
        return y, mean, invstd
    check(_lib().bigdl_bn_fwd_train_partials(ptr(x), ptr(residual), ptr(y), _ll(M), C.c_int(C_), ptr(gamma),
                                             ptr(beta), ptr(in_bias), ptr(running_mean), ptr(running_var),
                                             _f(momentum), _f(eps), ptr(mean), ptr(invstd), ptr(partial),
                                             C.c_int(G), ptr(shift if _f32vec(shift, C_) else None), ptr(coef),
                                             C.c_int(1 if relu else 0),
                                             ptr(_fold_scratch(G, C_, x.device)),
                                             ptr(_bits_ok(bits_out, M, C_, relu)), C.c_int(1 if rezero else 0), _s()),
          "bn_fwd_train_partials")
    return y, mean, invstd


def batchnorm_backward_partials(gm, x, gamma, save_mean, save_invstd, partial, G, need_input=True, gg_acc=None,
                                gb_acc=None, scale=1.0, cbias_acc=None, cbias_scale=1.0, lazy=False, rezero=False,
                                zero_next=None):
    """BN backward whose reductions came from the consumer conv's dgrad epilogue; ``gm`` is the
    already ReLU-masked gradient.  Returns gradInput (or None) / NotImplemented; ``lazy`` returns
    it as a :class:`~bigdl.ops.reference.BNGrad` (coefficients only, no apply pass)."""
    rc = _rows_c(x)
    if rc is None:
        return NotImplemented
    M, C_ = rc
    if (rezero and 1 <= G <= 512 and _bn32_ok(x, C_, gm) and partial is not None and partial.dtype == _f32
            and partial.numel() == 2 * G * C_
            and all(_f32vec(t, C_) for t in (gamma, save_mean, save_invstd, gg_acc, gb_acc, cbias_acc))):
        # fp32 compute: the replicated sums of the consumer's fp32 dgrad epilogue (fp32x3.conv_backward)
        coef = torch.empty(3 * C_, dtype=_f32, device=x.device)
        gx = torch.empty_like(x) if need_input else None
        sp = F3.split_buffer(M, C_, x.device) if need_input else None
        check(_lib().bigdl_bn32_bwd_partials(ptr(gm), ptr(x), ptr(gx), _ll(M), C.c_int(C_), ptr(gamma),
                                             ptr(save_mean), ptr(save_invstd), ptr(gg_acc), ptr(gb_acc), _f(scale),
                                             ptr(cbias_acc), _f(cbias_scale), ptr(partial), C.c_int(G), ptr(coef),
                                             ptr(sp), _s()), "bn32_bwd_partials")
        F3.note_split(gx, sp)
        return gx
    if not _bn_ok(x, C_) or gm.dtype != _bf16 or gm.shape != x.shape or gm.stride() != x.stride() or not _al16(gm):
        return NotImplemented
    if not all(_f32vec(t, C_) for t in (gamma, save_mean, save_invstd, gg_acc, gb_acc, cbias_acc)):
        return NotImplemented
    coef = torch.empty(3 * C_, dtype=_f32, device=x.device)
    gx = torch.empty_like(x) if (need_input and not lazy) else None
    if (rezero and G >= 1 and zero_next is not None and partial is not None and zero_next.numel() == partial.numel()
            and C_ <= 4096 and 2 * G * C_ <= 32768 and _al16(zero_next)):
        # ONE launch (no finalize kernel): coefficients from the dgrad's replicated sums in every block,
        # dγ / dβ / the folded bias by block 0, which also clears the next step's replica set
        check(_lib().bigdl_bn_bwd_rep_fin(ptr(gm), ptr(x), ptr(gx), _ll(M), C.c_int(C_), ptr(gamma), ptr(save_mean),
                                          ptr(save_invstd), ptr(gg_acc if scale != 0 else None),
                                          ptr(gb_acc if scale != 0 else None), _f(scale),
                                          ptr(cbias_acc if cbias_scale != 0 else None), _f(cbias_scale), ptr(partial),
                                          C.c_int(G), ptr(zero_next), ptr(coef), _s()), "bn_bwd_rep_fin")
        if need_input and lazy:
            return R_.BNGrad(gm, x, coef)
        return gx
    if G == 0:  # atomically accumulated [Σg', Σg'·(x − μ), counter] from the dgrad epilogue
        if partial is None or partial.numel() != 2 * C_ + 1 or partial.dtype != _f32 or C_ > 4096:
            return NotImplemented
        check(_lib().bigdl_bn_bwd_sums_apply(ptr(gm), ptr(x), ptr(gx), _ll(M), C.c_int(C_), ptr(gamma),
                                             ptr(save_mean), ptr(save_invstd), ptr(gg_acc), ptr(gb_acc), _f(scale),
                                             ptr(cbias_acc), _f(cbias_scale), ptr(partial), ptr(coef), _s()),
              "bn_bwd_sums_apply")
        if need_input and lazy:
            return R_.BNGrad(gm, x, coef)
        return gx
    check(_lib().bigdl_bn_bwd_partials(ptr(gm), ptr(x), ptr(gx), _ll(M), C.c_int(C_), ptr(gamma), ptr(save_mean),
                                       ptr(save_invstd), ptr(gg_acc), ptr(gb_acc), _f(scale), ptr(cbias_acc),
                                       _f(cbias_scale), ptr(partial), C.c_int(G), ptr(coef),
                                       ptr(_fold_scratch(G, C_, x.device)), C.c_int(1 if rezero else 0), _s()),
          "bn_bwd_partials")
    if need_input and lazy:
        return R_.BNGrad(gm, x, coef)
    return gx


# ---- SyncBN (cross-rank statistics; the caller all-reduces the 2·C sums between the halves) ----
def bn_local_sums(x, shift, partial=None, G=0, rezero=False):
    """This rank's shifted sums [Σ(x−K), Σ(x−K)², rows] (fp32 [2C + 1]) with K = ``shift`` (the
    running mean, identical on every rank): from a producing conv's epilogue partials
    (``partial``/``G``, which must have been computed with the same shift) or a stats pass over x.
    The row count rides in the buffer the all-reduce sums, so every rank issues the same collective
    every step whatever its batch, and the global count never needs a host read.  NotImplemented
    when the native path cannot run."""
    rc = _rows_c(x)
    if rc is None:
        return NotImplemented
    M, C_ = rc
    if not _bn_ok(x, C_) or not _f32vec(shift, C_):
        return NotImplemented
    out = torch.empty(2 * C_ + 1, dtype=_f32, device=x.device)
    if partial is not None:
        if partial.numel() != 2 * G * C_ or partial.dtype != _f32:
            return NotImplemented
        check(_lib().bigdl_bn_partials_sums(ptr(partial), C.c_int(G), C.c_int(C_),
                                            ptr(_fold_scratch(G, C_, x.device)), ptr(out), _f(M),
                                            C.c_int(1 if rezero else 0), _s()),
              "bn_partials_sums")
        return out
    lib = _lib()
    Gs = lib.bigdl_bn_num_partials(_ll(M), C.c_int(C_))
    ws = torch.empty(2 * Gs * C_, dtype=_f32, device=x.device)
    check(lib.bigdl_bn_stats_sums(ptr(x), _ll(M), C.c_int(C_), ptr(shift), ptr(ws), ptr(_fold_scratch(Gs, C_, x.device)),
                                  ptr(out), _f(M), _s()), "bn_stats_sums")
    return out


_TICKETS: dict = {}


def _ticket(dev):
    """A zeroed arrival-ticket word of the device (the one-launch finalize+apply kernels' last-block
    election; the last arriver re-zeroes it, so stream-ordered launches share it)."""
    t = _TICKETS.get(dev)
    if t is None:
        t = _TICKETS[dev] = torch.zeros(32, dtype=torch.int32, device=dev)  # root + 16 leaves (batchnorm.hip)
    return t


def bn_forward_from_sums(x, sums, count, shift, gamma, beta, running_mean, running_var, momentum, eps, relu=False,
                         residual=None, in_bias=None, coef_out=None, bits_out=None, mean_out=None, apply=True):
    """Training BN from GLOBAL shifted sums over ``count`` rows (0: the all-reduced count at
    ``sums[2C]``): (y, save_mean, save_invstd).  ``bits_out`` (uint8 [M·C/8], with ``relu``): the
    output's ReLU mask as bits for a block-tail consumer's dgrad epilogue.  ``apply=False``: finalize
    only (``coef_out`` required, y = None: a deferred shortcut BN); ``residual`` may be such a deferred
    BN output (:class:`~bigdl.ops.reference.BNOut`), applied inside this pass."""
    rc = _rows_c(x)
    if rc is None:
        return NotImplemented
    M, C_ = rc
    if not _bn_ok(x, C_) or not all(_f32vec(t, C_) for t in (gamma, beta, running_mean, running_var, in_bias, shift)):
        return NotImplemented
    rcoef = None
    if isinstance(residual, R_.BNOut):
        if residual.relu or not (residual.x.shape == x.shape and residual.x.stride() == x.stride()
                                 and residual.x.dtype == _bf16 and _al16(residual.x) and _f32vec(residual.coef, 2 * C_)):
            return NotImplemented
        residual, rcoef = residual.x, residual.coef
    if residual is not None and (residual.shape != x.shape or residual.stride() != x.stride() or
                                 residual.dtype != _bf16 or not _al16(residual)):
        return NotImplemented
    if not apply and (residual is not None or bits_out is not None or not _coef_ok(coef_out, C_)):
        return NotImplemented
    coef = coef_out if _coef_ok(coef_out, C_) else torch.empty(2 * C_, dtype=_f32, device=x.device)
    mean = mean_out if _f32vec(mean_out, C_) and mean_out is not None else torch.empty(C_, dtype=_f32, device=x.device)
    invstd = torch.empty(C_, dtype=_f32, device=x.device)
    y = torch.empty_like(x) if apply else None
    check(_lib().bigdl_bn_fwd_train_sums(ptr(x), ptr(residual), ptr(rcoef), ptr(y), _ll(M), _ll(count), C.c_int(C_), ptr(gamma),
                                         ptr(beta), ptr(in_bias), ptr(running_mean), ptr(running_var), _f(momentum),
                                         _f(eps), ptr(mean), ptr(invstd), ptr(sums), ptr(shift), ptr(coef),
                                         C.c_int(1 if relu else 0), ptr(bits_out if relu else None),
                                         ptr(_ticket(x.device)), _s()),
          "bn_fwd_train_sums")
    return y, mean, invstd


def bn_bwd_local_sums(gy, x, save_mean, y=None, relu=False):
    """This rank's [Σg', Σg'·(x − mean)] twice (fp32 [4C + 1]: the local sums, then a copy for the
    in-place all-reduce followed by this rank's row count); g' = gy·[y > 0] when ``relu``."""
    rc = _rows_c(x)
    if rc is None:
        return NotImplemented
    M, C_ = rc
    if not _bn_ok(x, C_) or gy.dtype != _bf16 or gy.shape != x.shape or gy.stride() != x.stride() or not _al16(gy):
        return NotImplemented
    if relu and (y is None or y.dtype != _bf16 or y.stride() != x.stride() or not _al16(y)):
        return NotImplemented
    lib = _lib()
    G = lib.bigdl_bn_num_partials(_ll(M), C.c_int(C_))
    ws = torch.empty(2 * G * C_, dtype=_f32, device=x.device)
    out = torch.empty(4 * C_ + 1, dtype=_f32, device=x.device)
    check(lib.bigdl_bn_bwd_sums(ptr(gy), ptr(x), ptr(y if relu else None), _ll(M), C.c_int(C_), ptr(save_mean), ptr(ws),
                                ptr(_fold_scratch(G, C_, x.device)), ptr(out), C.c_int(1 if relu else 0), _f(M), _s()),
          "bn_bwd_sums")
    return out


def bn_bwd_partials_sums(partial, G, C_, dev, rows=None, rezero=False):
    """[Σg', Σg'·(x − mean)] twice (fp32 [4C + 1], ``rows`` last) from the consumer conv's
    dgrad-epilogue partials (``_pending_grad``): no pass over the activations."""
    if partial is None or partial.dtype != _f32 or partial.numel() != 2 * G * C_ or rows is None:
        return NotImplemented
    out = torch.empty(4 * C_ + 1, dtype=_f32, device=dev)
    check(_lib().bigdl_bn_partials_sums2(ptr(partial), C.c_int(G), C.c_int(C_), ptr(_fold_scratch(G, C_, dev)),
                                         ptr(out), ptr(out[2 * C_:]), _f(rows), C.c_int(1 if rezero else 0), _s()), "bn_partials_sums2")
    return out


def bn_backward_from_sums(gy, x, gamma, save_mean, save_invstd, local_sums, global_sums, count, y=None, relu=False,
                          need_input=True, gg_acc=None, gb_acc=None, scale=1.0, cbias_acc=None, cbias_scale=1.0):
    """SyncBN backward: local sums → this rank's dγ/dβ; global sums over ``count`` rows (0: the
    all-reduced count at ``global_sums[2C]``) → gradInput; ``cbias_acc`` receives this rank's share
    of a folded producer bias's gradient (fp32 closed form)."""
    rc = _rows_c(x)
    if rc is None:
        return NotImplemented
    M, C_ = rc
    if not all(_f32vec(t, C_) for t in (gamma, save_mean, save_invstd, gg_acc, gb_acc, cbias_acc)):
        return NotImplemented
    coef = torch.empty(3 * C_, dtype=_f32, device=x.device)
    scratch = torch.empty(3 * C_, dtype=_f32, device=x.device)
    gx = torch.empty_like(x) if need_input else None
    check(_lib().bigdl_bn_bwd_apply_sums(ptr(gy), ptr(x), ptr(y if relu else None), ptr(gx), _ll(M), _ll(count),
                                         C.c_int(C_), ptr(gamma), ptr(save_mean), ptr(save_invstd),
                                         ptr(gg_acc if scale != 0 else None), ptr(gb_acc if scale != 0 else None),
                                         _f(scale), ptr(local_sums), ptr(global_sums), ptr(coef), ptr(scratch),
                                         C.c_int(1 if relu else 0), ptr(cbias_acc if cbias_scale != 0 else None),
                                         _f(cbias_scale), ptr(_ticket(x.device)), _s()), "bn_bwd_apply_sums")
    return gx


@register("batchnorm_forward_infer")
def batchnorm_forward_infer(x, gamma, beta, running_mean, running_var, eps, relu=False, in_bias=None):
    rc = _rows_c(x)
    if rc is None:
        return NotImplemented
    M, C_ = rc
    if _bn32_ok(x, C_) and all(_f32vec(t, C_) for t in (gamma, beta, running_mean, running_var, in_bias)):
        coef = torch.empty(2 * C_, dtype=_f32, device=x.device)
        y = torch.empty_like(x)
        check(_lib().bigdl_bn32_fwd_infer(ptr(x), ptr(y), _ll(M), C.c_int(C_), ptr(gamma), ptr(beta),
                                          ptr(running_mean), ptr(running_var), ptr(in_bias), _f(eps), ptr(coef),
                                          C.c_int(1 if relu else 0), _s()), "bn32_fwd_infer")
        return y
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
    mb = F3.producer_bits(y) if relu else None  # the forward's ReLU mask bits (1 bit instead of 4 B)
    if (_bn32_ok(x, C_, gy, y if relu and mb is None else None) and (y is not None or not relu)
            and all(_f32vec(t, C_) for t in (gamma, save_mean, save_invstd, gg_acc, gb_acc, cbias_acc))):
        G = _lib().bigdl_bn_num_partials(_ll(M), C.c_int(C_))
        ws = torch.empty(2 * G * C_, dtype=_f32, device=x.device)
        coef = torch.empty(3 * C_, dtype=_f32, device=x.device)
        gx = torch.empty_like(x) if need_input else None
        gres = torch.empty_like(x) if want_gres else None
        sp = F3.split_buffer(M, C_, x.device) if need_input else None  # the producing conv's dY split
        check(_lib().bigdl_bn32_bwd(ptr(gy), ptr(x), ptr(y if relu else None), ptr(gx), ptr(gres), _ll(M), C.c_int(C_),
                                    ptr(gamma), ptr(save_mean), ptr(save_invstd), ptr(gg_acc), ptr(gb_acc), _f(scale),
                                    ptr(cbias_acc), _f(cbias_scale), ptr(ws), ptr(coef), C.c_int(1 if relu else 0),
                                    ptr(sp), ptr(mb), _s()), "bn32_bwd")
        F3.note_split(gx, sp)
        return gx, gres
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
    # float labels already on the device are read by the kernel as they are (no per-step int cast)
    tf = target_1b.reshape(-1) if target_1b.dtype == _f32 and target_1b.device == x.device else None
    if tf is not None and (tf.numel() != B or not tf.is_contiguous() or not hasattr(_lib(), "bigdl_cross_entropy_ft")):
        tf = None
    t = None if tf is not None else _targets_i32(target_1b.to(x.device), B)
    if tf is None and t is None:
        return NotImplemented
    w = None
    if weights is not None:
        w = weights.to(x.device, _f32).contiguous()
        if w.numel() != K:
            return NotImplemented
    ws = torch.empty(3 * B, dtype=_f32, device=x.device)
    out = torch.empty(2, dtype=_f32, device=x.device)
    gx = torch.empty_like(x)
    fn = _lib().bigdl_cross_entropy_ft if tf is not None else _lib().bigdl_cross_entropy
    check(fn(ptr(x), ptr(tf if tf is not None else t), ptr(w), ptr(gx), _ll(B), C.c_int(K), C.c_int(int(padding_value)),
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


# ------------------------------------------------------------------------------------------------ convolution
def _krsc(w4):
    """(O, I, kH, kW) view → contiguous (O, kH, kW, I) tensor (a view when already KRSC)."""
    k = w4.permute(0, 2, 3, 1)
    return k if k.is_contiguous() else k.contiguous()


def _pad_taps(wk, K, taps, C_, cp, ldw):
    """KRSC bf16 weights → [K][ldw] rows, each tap's channels zero-padded to ``cp`` and the row to
    ``ldw`` (one native pass; the weights change every step, so nothing is cached)."""
    wp = torch.empty((K, ldw), dtype=wk.dtype, device=wk.device)
    if wk.is_cuda and wk.dtype == _bf16 and wk.is_contiguous() and hasattr(_lib(), "bigdl_pad_taps_bf16"):
        check(_lib().bigdl_pad_taps_bf16(ptr(wk), ptr(wp), C.c_int(K), C.c_int(taps), C.c_int(C_), C.c_int(cp),
                                         C.c_int(ldw), _s()), "pad_taps_bf16")
        return wp
    wp.zero_()
    wp[:, :taps * cp].view(K, taps, cp)[..., :C_] = wk.reshape(K, taps, C_)
    return wp


def _pad_channels(x_nhwc_4d, c_to, slot=None, reuse=False):
    """Zero-pad the channel dim of a channels-last NCHW-logical tensor to ``c_to``.

    ``slot`` is the calling layer's one-entry holder: the forward (``reuse=False``) always pads
    afresh and parks (source, version, padded) there; the same layer's backward (``reuse=True``)
    takes the forward's copy when it still describes the same input.  The copy therefore lives
    exactly as long as the layer's forward→backward pair and, under HIP-graph capture, is produced
    by a captured kernel of the same graph (no process-global cache)."""
    if slot is not None and isinstance(slot[0], tuple) and len(slot[0]) == 4:
        # the backward of the same input, or an input the layout conversion produced padded
        src, ver, ct, padded = slot[0]
        if src is x_nhwc_4d and ver == x_nhwc_4d._version and ct == c_to and (reuse or padded.dim() == 4 and
                                                                             padded.shape[1] == c_to and
                                                                             padded.data_ptr() == src.data_ptr()):
            return padded
    n, c, h, w = x_nhwc_4d.shape
    out = torch.empty((n, h, w, c_to), dtype=x_nhwc_4d.dtype, device=x_nhwc_4d.device)
    if (x_nhwc_4d.is_cuda and x_nhwc_4d.dtype == _bf16 and c_to <= 8 and _al16(out)
            and x_nhwc_4d.is_contiguous(memory_format=torch.channels_last)):
        # one HIP pass: read C, write C_to (8-B / 16-B stores), no separate zero fill
        check(_lib().bigdl_pad_channels(ptr(x_nhwc_4d), ptr(out), _ll(n * h * w), C.c_int(c), C.c_int(c_to), _s()),
              "pad_channels")
    else:
        out[..., c:].zero_()
        out[..., :c] = x_nhwc_4d.permute(0, 2, 3, 1)
    res = out.permute(0, 3, 1, 2)
    if slot is not None:
        slot[0] = (x_nhwc_4d, x_nhwc_4d._version, c_to, res)
    return res


def _conv_geom_ok(x, w4, groups, dilation):
    return (groups == 1 and x.dim() == 4 and x.dtype == _bf16 and w4.dtype == _bf16 and
            x.is_contiguous(memory_format=torch.channels_last) and _al16(x))


def _conv_geom_ok_slot(x, w4, groups, dilation, slot):
    """:func:`_conv_geom_ok`, also accepting a few-channel input view whose channel-padded
    channels-last copy the layout conversion parked in the layer's pad ``slot``."""
    if _conv_geom_ok(x, w4, groups, dilation):
        return True
    pre = _prepadded(x, slot)
    return pre is not None and x.dtype == _bf16 and _conv_geom_ok(pre, w4, groups, dilation)


def _depthwise_ok(x, w4, groups):
    """groups == C == K (one filter per channel): the depthwise stencil kernels (depthwise.hip)."""
    return (groups > 1 and x.dim() == 4 and x.dtype == _bf16 and x.shape[1] == groups and w4.shape[0] == groups
            and w4.shape[1] == 1 and groups % 8 == 0 and w4.shape[2] * w4.shape[3] <= 25
            and x.is_contiguous(memory_format=torch.channels_last) and _al16(x))


def _dw_weight(w4):
    C_, _, R, S = w4.shape
    return w4.detach().float().reshape(C_, R * S).t().contiguous()  # [R·S][C] fp32


def _dw_out_hw(H, W, R, S, stride, pad, dilation):
    return ((H + 2 * pad[0] - dilation[0] * (R - 1) - 1) // stride[0] + 1,
            (W + 2 * pad[1] - dilation[1] * (S - 1) - 1) // stride[1] + 1)


def _depthwise_fwd(x, w4, b, stride, pad, dilation, relu=False):
    N_, C_, H, W = x.shape
    R, S = w4.shape[2], w4.shape[3]
    P, Q = _dw_out_hw(H, W, R, S, stride, pad, dilation)
    if P <= 0 or Q <= 0:
        return NotImplemented
    y = torch.empty((N_, C_, P, Q), dtype=_bf16, device=x.device, memory_format=torch.channels_last)
    bias = None if b is None else b.detach().float().contiguous()
    check(_lib().bigdl_dw_fwd(ptr(x), ptr(_dw_weight(w4)), ptr(bias), ptr(y), N_, H, W, C_, P, Q, R, S, stride[0],
                              stride[1], pad[0], pad[1], dilation[0], dilation[1], int(bool(relu)), _s()), "dw_fwd")
    return y


def _depthwise_bwd(gy, x, w4, stride, pad, dilation, need_input, gw_acc, gb_acc, scale):
    N_, C_, H, W = x.shape
    R, S = w4.shape[2], w4.shape[3]
    P, Q = gy.shape[2], gy.shape[3]
    if not (gy.dtype == _bf16 and gy.is_contiguous(memory_format=torch.channels_last) and _al16(gy)):
        gy = gy.to(_bf16).contiguous(memory_format=torch.channels_last)
    gi = None
    if need_input:
        gi = torch.empty(x.shape, dtype=_bf16, device=x.device, memory_format=torch.channels_last)
        check(_lib().bigdl_dw_dgrad(ptr(gy), ptr(_dw_weight(w4)), ptr(gi), N_, H, W, C_, P, Q, R, S, stride[0],
                                    stride[1], pad[0], pad[1], dilation[0], dilation[1], _s()), "dw_dgrad")
    if gw_acc is not None and scale != 0:
        tmp = torch.zeros((R * S, C_), dtype=_f32, device=x.device)
        check(_lib().bigdl_dw_wgrad(ptr(x), ptr(gy), ptr(tmp), _f(1.0), N_, H, W, C_, P, Q, R, S, stride[0], stride[1],
                                    pad[0], pad[1], dilation[0], dilation[1], _s()), "dw_wgrad")
        gw_acc.add_(tmp.t().reshape(C_, 1, R, S), alpha=scale)
    if gb_acc is not None and scale != 0:
        gb_acc.add_(gy.float().sum((0, 2, 3)), alpha=scale)
    return gi


def _grouped_ok(x, w4, groups):
    return (groups > 1 and x.dim() == 4 and x.dtype == _bf16 and w4.dtype == _bf16 and x.shape[1] % groups == 0
            and w4.shape[0] % groups == 0 and w4.shape[1] == x.shape[1] // groups)


def _group_slice(t, g, n):
    """channel slice g (width n) of an NCHW-shaped tensor as its own channels-last tensor (one copy)."""
    return t[:, g * n:(g + 1) * n].contiguous(memory_format=torch.channels_last)


def _group_pack(G, Cg, Kg):
    """Groups per launch group ("pack"): a divisor of G whose packed widths gps·Cg and gps·Kg are
    multiples of 8 (16-B chunks), as large as fits one 64-channel output tile.  A pack runs as one
    dense conv on a block-diagonal filter: the MFMA tile pays 64 output channels per pixel however
    the groups are split, so packing small groups adds no work and fills the k loop.  None when no
    divisor gives 8-aligned widths."""
    best = None
    for gps in range(1, G + 1):
        if G % gps or (gps * Cg) % 8 or (gps * Kg) % 8:
            continue
        if best is None or gps * Kg <= 64:
            best = gps
    return best


def _packed_filter(w4, G, gps):
    """[K][Cg][R][S] grouped filter → [G/gps · gps·Kg][R][S][gps·Cg] bf16: each pack's groups on the
    block diagonal (zeros elsewhere)."""
    K, Cg, R, S = w4.shape
    Kg = K // G
    if gps == 1:
        return _krsc(w4.to(_bf16))
    wv = w4.detach().to(_bf16).reshape(G // gps, gps, Kg, Cg, R, S)
    eye = torch.eye(gps, dtype=_bf16, device=w4.device)
    bd = torch.einsum("aikcrs,ij->aikrsjc", wv, eye)  # exact: products with 0 / 1
    return bd.reshape(K, R, S, gps * Cg).contiguous()


def _conv_fwd_grouped_1(x, w4, b, stride, pad, dilation, groups, relu=False, out_hw=None):
    """Grouped convolution (SpatialConvolution.scala:93-98 nGroup) in ONE launch: packs of groups
    (``_group_pack``) are the grid's y index, x is read in place (pixel stride C), y written in
    place (pixel stride K).  NotImplemented when no 8-aligned packing exists."""
    N_, C_, H, W = x.shape
    K, Cg, R, S = w4.shape
    Kg = K // groups
    gps = _group_pack(groups, Cg, Kg)
    if gps is None or not (x.is_contiguous(memory_format=torch.channels_last) and _al16(x)):
        return NotImplemented
    if out_hw is None:
        out_hw = _dw_out_hw(H, W, R, S, stride, pad, dilation)
    P, Q = out_hw
    if P <= 0 or Q <= 0:
        return NotImplemented
    wp = _packed_filter(w4, groups, gps)
    y = torch.empty((N_, K, P, Q), dtype=_bf16, device=x.device, memory_format=torch.channels_last)
    bias = None if b is None else b.detach().float().contiguous()
    check(_lib().bigdl_conv_fwd_grouped(ptr(x), ptr(wp), ptr(bias), ptr(y), N_, H, W, C_, gps * Cg, gps * Kg,
                                        groups // gps, R, S, P, Q, stride[0], stride[1], pad[0], pad[1],
                                        dilation[0], dilation[1], int(bool(relu)), K, _s()), "conv_fwd_grouped")
    return y


def _conv_bwd_grouped_1(gy, x, w4, stride, pad, dilation, groups, need_input, gw_acc, gb_acc, scale):
    """Backward of ``_conv_fwd_grouped_1``: data gradient = the grouped forward of dY with each
    group's flipped, transposed filter (strided convs scatter dY onto the stride lattice first);
    weight gradient = one grouped wgrad launch over the packs, block diagonals extracted."""
    N_, C_, H, W = x.shape
    K, Cg, R, S = w4.shape
    Kg = K // groups
    P, Q = gy.shape[2], gy.shape[3]
    gps = _group_pack(groups, Cg, Kg)
    if gps is None or _group_pack(groups, Kg, Cg) is None:
        return NotImplemented
    if not (x.is_contiguous(memory_format=torch.channels_last) and _al16(x)):
        return NotImplemented
    if not (gy.is_contiguous(memory_format=torch.channels_last) and _al16(gy)):
        gy = gy.to(_bf16).contiguous(memory_format=torch.channels_last)
    gi = None
    if need_input:
        src = gy
        if tuple(stride) != (1, 1):
            src = torch.empty((N_, K, (P - 1) * stride[0] + 1, (Q - 1) * stride[1] + 1), dtype=_bf16,
                              device=gy.device, memory_format=torch.channels_last).zero_()
            src[:, :, ::stride[0], ::stride[1]] = gy
        wt = w4.detach().reshape(groups, Kg, Cg, R, S).flip(3, 4).transpose(1, 2).reshape(C_, Kg, R, S)
        pd = (dilation[0] * (R - 1) - pad[0], dilation[1] * (S - 1) - pad[1])
        gi = _conv_fwd_grouped_1(src, wt, None, (1, 1), pd, dilation, groups, out_hw=(H, W))
        if gi is NotImplemented:
            return NotImplemented
    if gw_acc is not None and scale != 0:
        NS, KS, CS = groups // gps, gps * Kg, gps * Cg
        tmp = torch.zeros((NS, KS, R, S, CS), dtype=_f32, device=x.device)
        check(_lib().bigdl_conv_wgrad_grouped(ptr(x), ptr(gy), ptr(tmp), _f(1.0), N_, H, W, C_, CS, K, KS, NS, R, S,
                                              P, Q, stride[0], stride[1], pad[0], pad[1], dilation[0], dilation[1],
                                              _s()), "conv_wgrad_grouped")
        if gps > 1:  # the packs' block diagonals: [NS][gps][Kg][R][S][gps][Cg] → [K][Cg][R][S]
            d = torch.diagonal(tmp.view(NS, gps, Kg, R, S, gps, Cg), dim1=1, dim2=5)  # [NS][Kg][R][S][Cg][gps]
            gw = d.permute(0, 5, 1, 4, 2, 3).reshape(K, Cg, R, S)
        else:
            gw = tmp.view(K, R, S, Cg).permute(0, 3, 1, 2)
        gw_acc.add_(gw, alpha=scale)
    if gb_acc is not None and scale != 0:
        gb_acc.add_(gy.float().sum((0, 2, 3)), alpha=scale)
    return gi


def _conv_fwd_grouped(x, w4, b, stride, pad, dilation, groups, pad_slot=None, relu=False):
    """Grouped convolution (the reference's nGroup, SpatialConvolution.scala:93-98): one launch over
    all groups (``_conv_fwd_grouped_1``); only a grouping with no 8-aligned packing falls back to
    one groups=1 launch per group on channel slices."""
    y = _conv_fwd_grouped_1(x, w4, b, stride, pad, dilation, groups, relu)
    if y is not NotImplemented:
        return y
    N_, C_, H, W = x.shape
    K = w4.shape[0]
    Cg, Kg = C_ // groups, K // groups
    P = (H + 2 * pad[0] - dilation[0] * (w4.shape[2] - 1) - 1) // stride[0] + 1
    Q = (W + 2 * pad[1] - dilation[1] * (w4.shape[3] - 1) - 1) // stride[1] + 1
    y = torch.empty((N_, K, P, Q), dtype=_bf16, device=x.device, memory_format=torch.channels_last)
    for g in range(groups):
        xg = _group_slice(x, g, Cg)
        wg = w4[g * Kg:(g + 1) * Kg]
        bg = None if b is None else b[g * Kg:(g + 1) * Kg]
        tgt = y[:, g * Kg:(g + 1) * Kg] if (Kg % 8 == 0 and K % 8 == 0) else None
        r = _conv_fwd_impl(xg, wg, bg, stride, pad, dilation, 1, relu=relu, out=tgt)
        if r is NotImplemented:
            return NotImplemented
        if tgt is None:
            y[:, g * Kg:(g + 1) * Kg] = r
    return y


# ------------------------------------------------------------------------------------------------ kernel selection
#: per-geometry tile choice (BN, BK, BM) of the implicit-GEMM forward, filled by the compile phase's
#: autotuner (nn/compiled.py ``autotune``) and passed with each launch (no launcher-global state);
#: ``record`` collects (geometry, relaunch-with-tile) pairs while a planned forward runs.  Empty
#: table = the launcher's shape heuristic everywhere.
_TILE = {"table": {}, "record": None}


def _stat_target(part, atomic):
    """Where a statistics epilogue writes: the real buffer, except while kernel selection re-times a
    recorded launch whose tiles ADD into the consumer's sums (a repeat would corrupt the next step's
    statistics): then a throwaway zeroed copy."""
    if atomic and _TILE.get("retiming"):
        return torch.zeros_like(part)
    return part


def _tiled_launch(key, fn):
    """``fn(tile)`` launches the conv with ``tile`` = (BN, BK, BM) (zeros: the launcher's
    heuristic); the tile is this geometry's entry of the kernel-selection table, if any."""
    rec = _TILE["record"]
    if rec is not None:
        # first launch per geometry only: a closure pins its launch's operands (dY, partials, …) until
        # retiming ends, so recording every repeat would hold a whole step's worth of tensors
        if isinstance(rec, dict):
            rec.setdefault(key, fn)
        else:
            rec.append((key, fn))
    fn(_TILE["table"].get(key, (0, 0, 0)))


def conv_tile_table() -> dict:
    return _TILE["table"]


def _conv_fwd_impl(x, w4, b, stride, pad, dilation=(1, 1), groups=1, res=None, stats=False, relu=False, out=None,
                   pad_slot=None, shift=None, sums=None):
    """``out`` (optional): a channel slice ``big[:, c0:c0+K]`` of a channels-last tensor the conv
    writes into directly (zero-copy concat); returned as the result."""
    if groups > 1 and res is None and not stats and out is None and _depthwise_ok(x, w4, groups):
        return _depthwise_fwd(x, w4, b, stride, pad, dilation, relu)
    if groups > 1 and res is None and not stats and out is None and _grouped_ok(x, w4, groups):
        return _conv_fwd_grouped(x, w4, b, stride, pad, dilation, groups, pad_slot, relu)
    if not _conv_geom_ok_slot(x, w4, groups, dilation, pad_slot):
        return NotImplemented
    N_, C_, H, W = x.shape
    K, Ci, R, S = w4.shape
    if Ci != C_:
        return NotImplemented
    if (res is not None or stats) and K % 8:
        return NotImplemented
    wk = _krsc(w4)
    c4 = C_ <= 4 and out is None and tuple(dilation) == (1, 1)
    ldw = 0
    if c4:
        # RGB stem: pad 3 → 4 channels (not 8) and run the two-taps-per-chunk C4 gather; weight rows
        # are zero-padded to a multiple of 8 elements so every 16-B weight chunk stays aligned
        x = _pad_channels(x, 4, pad_slot)
        kg = R * S * 4
        ldw = (kg + 7) // 8 * 8
        wp = _pad_taps(wk, K, R * S, C_, 4, ldw)
        wk, C_ = wp, 4
    elif C_ % 8:
        cp = (C_ + 7) // 8 * 8
        x = _pad_channels(x, cp, pad_slot)
        wp = _pad_taps(wk, K, R * S, C_, cp, R * S * cp).view(K, R, S, cp)
        wk, C_ = wp, cp
    P = (H + 2 * pad[0] - dilation[0] * (R - 1) - 1) // stride[0] + 1
    Q = (W + 2 * pad[1] - dilation[1] * (S - 1) - 1) // stride[1] + 1
    if P <= 0 or Q <= 0 or not _al16(wk):
        return NotImplemented
    if res is not None and not (res.shape == (N_, K, P, Q) and res.dtype == _bf16 and
                                res.is_contiguous(memory_format=torch.channels_last) and _al16(res)):
        return NotImplemented
    ldy = K
    if out is not None:
        if not (out.dim() == 4 and tuple(out.shape) == (N_, K, P, Q) and out.dtype == _bf16 and not stats
                and res is None and out.stride(1) == 1 and out.stride(3) % 8 == 0 and K % 8 == 0
                and out.stride(2) == out.stride(3) * Q and out.stride(0) == out.stride(2) * P and _al16(out)):
            return NotImplemented
        y, ldy = out, out.stride(3)
    else:
        y = torch.empty((N_, K, P, Q), dtype=_bf16, device=x.device, memory_format=torch.channels_last)
    bias = b if (b is None or (b.dtype == _f32 and b.is_contiguous())) else b.float().contiguous()
    part, G = None, 0
    if shift is not None and not (stats and res is None and not relu and out is None and tuple(dilation) == (1, 1)
                                  and _f32vec(shift, K)):
        shift = None
    atomic = 0
    if stats:
        if isinstance(sums, tuple) and shift is not None and sums[0].dtype == _f32 and sums[0].is_cuda \
                and 1 <= sums[1] <= 512 and sums[0].numel() == 2 * sums[1] * K:
            # replicated atomic statistics: tile tm ADDS into replica tm % R of the BN's zeroed
            # [2][R][K] buffer; the BN finalizes from the R rows (no fold pass) and clears them
            part, atomic, G = sums[0], sums[1], sums[1]
        elif sums is not None and not isinstance(sums, tuple) and shift is not None and sums.dtype == _f32 \
                and sums.numel() == 2 * K + 1 and sums.is_cuda:
            # the tiles ADD their partial sums into the consumer BN's zeroed [2K + 1] buffer (G = 0
            # marks it for the one-launch finalize+apply, ops/csrc/batchnorm.hip k_bn_apply_fin)
            part, atomic = sums, 1
        else:
            G = _lib().bigdl_conv_num_row_tiles(_ll(N_ * P * Q))
            part = torch.empty(2 * G * K, dtype=_f32, device=x.device)
    if c4:
        if shift is not None:
            check(_lib().bigdl_conv_fwd_c4_stats_shift(ptr(x), ptr(wk), ldw, ptr(bias), ptr(y), ptr(part), ptr(shift),
                                                       N_, H, W, K, R, S, P, Q, stride[0], stride[1], pad[0], pad[1],
                                                       atomic, _s()), "conv_fwd_c4_stats_shift")
            return y, part, G
        check(_lib().bigdl_conv_fwd_c4(ptr(x), ptr(wk), ldw, ptr(bias), ptr(res), ptr(y), ptr(part), N_, H, W, K, R, S,
                                       P, Q, stride[0], stride[1], pad[0], pad[1], int(relu), _s()), "conv_fwd_c4")
        return (y, part, G) if stats else y
    # geometry only: a tile tuned on the plain forward also serves the BN-statistics / residual
    # epilogues of the same conv (training), which every tile shape instantiates
    key = (N_, H, W, C_, K, R, S, tuple(stride), tuple(pad), tuple(dilation))
    if shift is not None:
        _tiled_launch(key, lambda t: check(_lib().bigdl_conv_fwd_stats_shift_t(
            ptr(x), ptr(wk), ptr(bias), ptr(y), ptr(_stat_target(part, atomic)), ptr(shift), N_, H, W, C_, K, R, S,
            P, Q, stride[0], stride[1], pad[0], pad[1], 1, 1, t[0], t[1], t[2], atomic, _s()),
            "conv_fwd_stats_shift"))
        return y, part, G
    _tiled_launch(key, lambda t: check(_lib().bigdl_conv_fwd_ldy_t(
        ptr(x), ptr(wk), ptr(bias), ptr(res), ptr(y), ptr(part), N_, H, W, C_, K, R, S, P, Q, stride[0], stride[1],
        pad[0], pad[1], dilation[0], dilation[1], int(relu), ldy, t[0], t[1], t[2], _s()), "conv_fwd"))
    if stats:
        return y, part, G
    return y


def conv2d_forward_q(x, w4, b, stride, pad, relu, q_scale, u8=False, pad_slot=None):
    """The RGB (C ≤ 4) stem conv with its output quantised in the epilogue (bias, ReLU, static
    int8 scale ``q_scale``; ``u8``: the unsigned offset code with its 0x80 tail) — the first layer
    of a calibrated int8 chain in one pass instead of a bf16 conv plus a quantisation pass.  Returns
    the tagged int8 NHWC activation, or NotImplemented."""
    if not (x.is_cuda and x.dtype == _bf16 and x.dim() == 4 and x.shape[1] <= 4 and w4.shape[1] == x.shape[1]):
        return NotImplemented
    if not _conv_geom_ok_slot(x, w4, 1, (1, 1), pad_slot):
        return NotImplemented
    N_, C_, H, W = x.shape
    K, _, R, S = w4.shape
    if K % 8:
        return NotImplemented
    wk = _krsc(w4)
    xp = _pad_channels(x, 4, pad_slot)
    kg = R * S * 4
    ldw = (kg + 7) // 8 * 8
    wp = torch.zeros((K, ldw), dtype=wk.dtype, device=wk.device)
    wp[:, :kg].view(K, R, S, 4)[..., :C_] = wk
    P = (H + 2 * pad[0] - R) // stride[0] + 1
    Q = (W + 2 * pad[1] - S) // stride[1] + 1
    if P <= 0 or Q <= 0:
        return NotImplemented
    y = _i8_act(N_, K, P, Q, x.device, u8)
    bias = b if (b is None or (b.dtype == _f32 and b.is_contiguous())) else b.float().contiguous()
    check(_lib().bigdl_conv_fwd_c4_q(ptr(xp), ptr(wp), ldw, ptr(bias), ptr(y), C.c_float(q_scale), C.c_int(int(u8)),
                                     N_, H, W, K, R, S, P, Q, stride[0], stride[1], pad[0], pad[1], int(relu), _s()),
          "conv_fwd_c4_q")
    return _tag(y, q_scale, u8)


@register("conv2d_forward")
def conv2d_forward(x, w4, b, stride, pad, dilation=(1, 1), groups=1, relu=False, out=None, res=None, pad_slot=None,
                   pro=None):
    """``pro`` (fp32 compute): ``x`` is the INPUT of a training BN + ReLU whose deferred output this conv
    consumes, ``pro`` that BN's [scale | shift] — the direct fp32 kernels apply it on load
    (NotImplemented when they cannot: the caller then materialises the BN output)."""
    if pro is not None:
        if x.dtype != _f32 or res is not None or out is not None or not F3.enabled(x):
            return NotImplemented
        return F3.conv_forward(x, w4, b, stride, pad, dilation, groups, relu, slot=pad_slot, pro=pro)
    if x.dtype == _f32 and res is None and out is None and F3.enabled(x):
        r = F3.conv_forward(x, w4, b, stride, pad, dilation, groups, relu, slot=pad_slot)
        if r is not NotImplemented:
            return r
    if res is not None and (res.dtype != _bf16 or not res.is_contiguous(memory_format=torch.channels_last)):
        res = res.to(_bf16).contiguous(memory_format=torch.channels_last)
    return _conv_fwd_impl(x, w4, b, stride, pad, dilation, groups, res=res, relu=relu, out=out, pad_slot=pad_slot)


def conv2d_forward_stats(x, w4, b, stride, pad, dilation=(1, 1), groups=1, pad_slot=None, shift=None, sums=None,
                         pro=None):
    """Forward conv whose epilogue also emits per-row-tile Σ(y−K)/Σ(y−K)² partials for a following
    BN (128-row tiles; the BN finalize combines them in fp64).  ``shift`` (fp32 [K], e.g. the BN's
    running mean) is K; the same array must reach the finalize.  ``sums`` (fp32 [2K + 1], zero): the
    tiles atomically ADD into it instead (returned G = 0) for the one-launch BN finalize+apply.
    Returns ``(y, partials, G)`` or NotImplemented."""
    if x.dtype == _f32 and F3.enabled(x):  # fp32 compute: the bf16x3 conv's fp32 epilogue (replicas only)
        if groups != 1 or b is not None:
            return NotImplemented
        return F3.conv_forward_stats(x, w4, stride, pad, dilation, sums, shift, slot=pad_slot, pro=pro)
    if pro is not None:
        return NotImplemented
    return _conv_fwd_impl(x, w4, b, stride, pad, dilation, groups, stats=True, pad_slot=pad_slot, shift=shift,
                          sums=sums)


def _dgrad_s1(gy, w4, x_shape, pad, dilation, residual=None, bn_fuse=None):
    """stride-1 backward-data as a forward conv of gy with the flipped, transposed kernel; an optional
    ``residual`` gradient (same shape as x) is summed in the epilogue."""
    N_, C_, H, W = x_shape
    K, Ci, R, S = w4.shape
    if K % 8:
        return None
    ax = acoef = None
    if isinstance(gy, R_.BNGrad):  # the BN input gradient, applied in the A-operand prologue
        gy, ax, acoef = gy.g, gy.x, gy.coef
    # W'[c][r][s][k] = W[k][R-1-r][S-1-s][c]: one cached-index gather from the KRSC storage (a
    # flip + transpose copy would be two launches per layer per step)
    ent = _S1_XFORM.get((K, Ci, R, S))
    if ent is None:
        ent = _S1_XFORM[(K, Ci, R, S)] = [(0, 0, list(range(R)), list(range(S)))]
    wt = _subfilters(w4, ent, ("s1", K, Ci, R, S))[0]
    P, Q = gy.shape[2], gy.shape[3]
    ph = dilation[0] * (R - 1) - pad[0]
    pw = dilation[1] * (S - 1) - pad[1]
    if ph < 0 or pw < 0:
        return None
    rs = None  # strided residual geometry (res_sh, res_sw, res_H, res_W)
    if isinstance(residual, R_.StridedGrad):
        t = residual.t
        if not (C_ % 8 == 0 and residual.shape == (N_, C_, H, W) and t.dtype == _bf16 and t.shape[:2] == (N_, C_)
                and t.is_contiguous(memory_format=torch.channels_last) and _al16(t)):
            return None
        rs = (residual.stride[0], residual.stride[1], t.shape[2], t.shape[3])
        residual = t
    elif residual is not None and not (C_ % 8 == 0 and residual.shape == (N_, C_, H, W)
                                       and residual.dtype == _bf16
                                       and residual.is_contiguous(memory_format=torch.channels_last)
                                       and _al16(residual)):
        return None
    gx = torch.empty((N_, C_, H, W), dtype=_bf16, device=gy.device, memory_format=torch.channels_last)
    # the dgrad IS a forward conv of gy (N, P, Q, K → C): it shares the forward geometry key space of
    # the kernel-selection table
    dkey = (N_, P, Q, K, C_, R, S, (1, 1), (ph, pw), tuple(dilation))
    if bn_fuse is not None and C_ % 8 == 0:
        # BN-backward prologue in the epilogue: either the ReLU mask recomputed from the BN input
        # (conv → BN+ReLU → this conv), or an explicit mask tensor with the residual gradient summed
        # first (ResNet block tail: mask = block output)
        bx, mu, mask = bn_fuse["x"], bn_fuse["mean"], bn_fuse.get("mask")
        sc, sh = bn_fuse.get("scale"), bn_fuse.get("shift")
        bits = bn_fuse.get("bits") if mask is not None else None
        if bits is not None and not (bits.dtype == torch.uint8 and bits.is_cuda and bits.is_contiguous()
                                     and bits.numel() == N_ * H * W * C_ // 8):
            bits = None

        def _act_ok(t):
            return (t.shape == (N_, C_, H, W) and t.dtype == _bf16
                    and t.is_contiguous(memory_format=torch.channels_last) and _al16(t))
        ok = _act_ok(bx) and mu is not None and _f32vec(mu, C_)
        ok = ok and (_act_ok(mask) if mask is not None else (residual is None and sc is not None and sh is not None
                                                             and _f32vec(sc, C_) and _f32vec(sh, C_)))
        sums = bn_fuse.get("sums")
        if ok and ax is None and isinstance(sums, tuple) and sums[0].dtype == _f32 and sums[0].is_cuda \
                and 1 <= sums[1] <= 512 and sums[0].numel() == 2 * sums[1] * C_:
            # replicated atomic statistics ([2][R][C], tile tm → replica tm % R); the BN backward
            # finalizes from the R rows and clears them
            buf, rep = sums
            _tiled_launch(dkey, lambda t: check(_lib().bigdl_conv_fwd_bnbwd(
                ptr(gy), ptr(wt), ptr(residual), ptr(gx), ptr(_stat_target(buf, 1)), rep, N_, P, Q, K, C_, R, S, H,
                W, 1, 1, ph, pw, dilation[0], dilation[1], ptr(bx), ptr(sc), ptr(sh), ptr(mu), ptr(mask),
                ptr(bits), *(rs or (0, 0, 0, 0)), t[0], t[1], t[2], _s()), "conv_dgrad_bnbwd_rep"))
            bn_fuse["partial"], bn_fuse["G"] = buf, rep
            return gx
        if ok and ax is None and sums is not None and not isinstance(sums, tuple) and sums.dtype == _f32 \
                and sums.numel() == 2 * C_ + 1 and sums.is_cuda:
            # the tiles ADD Σg', Σg'·(x − μ) into the BN's zeroed [2C + 1] buffer (G = 0): the BN
            # backward is then one finalize+apply launch (batchnorm.hip k_bn_bwd_apply_fin)
            _tiled_launch(dkey, lambda t: check(_lib().bigdl_conv_fwd_bnbwd(
                ptr(gy), ptr(wt), ptr(residual), ptr(gx), ptr(_stat_target(sums, 1)), 1, N_, P, Q, K, C_, R, S, H,
                W, 1, 1, ph, pw, dilation[0], dilation[1], ptr(bx), ptr(sc), ptr(sh), ptr(mu), ptr(mask),
                ptr(bits), *(rs or (0, 0, 0, 0)), t[0], t[1], t[2], _s()), "conv_dgrad_bnbwd_at"))
            bn_fuse["partial"], bn_fuse["G"] = sums, 0
            return gx
        if ok:
            G = _lib().bigdl_conv_num_row_tiles(_ll(N_ * H * W))
            part = torch.empty(2 * G * C_, dtype=_f32, device=gy.device)
            if ax is not None:
                check(_lib().bigdl_conv_fwd_full3(ptr(gy), ptr(ax), ptr(acoef), ptr(wt), ptr(residual), ptr(gx),
                                                  ptr(part), N_, P, Q, K, C_, R, S, H, W, 1, 1, ph, pw, dilation[0],
                                                  dilation[1], ptr(bx), ptr(sc), ptr(sh), ptr(mu), ptr(mask),
                                                  ptr(bits), *(rs or (0, 0, 0, 0)), _s()), "conv_dgrad_bnbwd3")
            elif rs is not None or bits is not None:
                _tiled_launch(dkey, lambda t: check(_lib().bigdl_conv_fwd_full2(
                    ptr(gy), ptr(wt), ptr(residual), ptr(gx), ptr(part), N_, P, Q, K, C_, R, S, H, W, 1, 1, ph, pw,
                    dilation[0], dilation[1], ptr(bx), ptr(sc), ptr(sh), ptr(mu), ptr(mask), ptr(bits),
                    *(rs or (0, 0, 0, 0)), t[0], t[1], t[2], _s()), "conv_dgrad_bnbwd2"))
            else:
                _tiled_launch(dkey, lambda t: check(_lib().bigdl_conv_fwd_full(
                    ptr(gy), ptr(wt), ptr(None), ptr(residual), ptr(gx), ptr(part), N_, P, Q, K, C_, R, S, H, W, 1,
                    1, ph, pw, dilation[0], dilation[1], 0, 1, 1, 0, 0, H, W, ptr(bx), ptr(sc), ptr(sh), ptr(mu),
                    ptr(mask), t[0], t[1], t[2], _s()), "conv_dgrad_bnbwd"))
            bn_fuse["partial"], bn_fuse["G"] = part, G
            return gx
    if ax is not None:
        check(_lib().bigdl_conv_fwd_full3(ptr(gy), ptr(ax), ptr(acoef), ptr(wt), ptr(residual), ptr(gx), ptr(None),
                                          N_, P, Q, K, C_, R, S, H, W, 1, 1, ph, pw, dilation[0], dilation[1],
                                          ptr(None), ptr(None), ptr(None), ptr(None), ptr(None), ptr(None),
                                          *(rs or (0, 0, 0, 0)), _s()), "conv_dgrad_at")
        return gx
    if rs is not None:
        _tiled_launch(dkey, lambda t: check(_lib().bigdl_conv_fwd_full2(
            ptr(gy), ptr(wt), ptr(residual), ptr(gx), ptr(None), N_, P, Q, K, C_, R, S, H, W, 1, 1, ph, pw,
            dilation[0], dilation[1], ptr(None), ptr(None), ptr(None), ptr(None), ptr(None), ptr(None), *rs,
            t[0], t[1], t[2], _s()), "conv_dgrad_rs"))
        return gx
    _tiled_launch(dkey, lambda t: check(_lib().bigdl_conv_fwd_ex(
        ptr(gy), ptr(wt), ptr(None), ptr(residual), ptr(gx), ptr(None), N_, P, Q, K, C_, R, S, H, W, 1, 1, ph, pw,
        dilation[0], dilation[1], 0, t[0], t[1], t[2], _s()), "conv_dgrad"))
    return gx


_SUBFILTER_IDX: dict = {}

# ---- dgrad weight transforms of a whole step in one launch (weight_xform.hip k_w_xform_multi) ----
# Transforms of weights that live in a parameter arena's bf16 shadow are cached per (weight, class
# list) with the arena's shadow generation; after an optimizer update the first dgrad refreshes
# every cached transform of that arena in ONE batched launch instead of one launch per layer.
_XFC: dict = {}
_XF_ARENAS: dict = {}   # shadow storage data_ptr → weakref(arena)
_XF_TABLE: dict = {}    # id(arena) → (device job table, njobs, total blocks, entry list)


def register_shadow_arena(arena) -> None:
    import weakref
    _XF_ARENAS[arena.shadow.untyped_storage().data_ptr()] = weakref.ref(arena)


def _shadow_arena(t):
    try:
        sp = t.untyped_storage().data_ptr()
    except RuntimeError:
        return None
    ref = _XF_ARENAS.get(sp)
    a = ref() if ref is not None else None
    if a is None or a.shadow is None or a.shadow.untyped_storage().data_ptr() != sp:
        return None
    return a


def _xf_refresh(arena) -> None:
    """Re-run every cached dgrad weight transform of ``arena`` in one launch (job table built once,
    outside HIP-graph capture; without a table, the stale entries are left for per-layer launches)."""
    entries = [c for c in _XFC.values() if c["arena"] == id(arena)]
    if not entries:
        return
    tab = _XF_TABLE.get(id(arena))
    if tab is None:
        if torch.cuda.is_current_stream_capturing():
            return
        lib = _lib()
        rec = int(lib.bigdl_w_xform_job_size())
        buf = (C.c_ubyte * (rec * len(entries)))()
        first = 0
        nb = C.c_longlong(0)
        for i, c in enumerate(entries):
            K, R, S, C_, ncls, a_ro, a_so, a_rm, a_sm, a_off = c["args"]
            check(lib.bigdl_w_xform_job(C.byref(buf, i * rec), ptr(c["phys"]), ptr(c["out"]), K, R, S, C_, ncls, a_ro,
                                        a_so, a_rm, a_sm, a_off, C.c_longlong(first), C.byref(nb)), "w_xform_job")
            first += nb.value
        host = torch.frombuffer(bytearray(bytes(buf)), dtype=torch.uint8)
        dev = torch.empty(host.numel() + 16, dtype=torch.uint8, device=entries[0]["out"].device)
        off = (-dev.data_ptr()) % 16
        table = dev[off:off + host.numel()]
        table.copy_(host)
        tab = _XF_TABLE[id(arena)] = (table, len(entries), first, entries, dev)
    table, nj, total, ents, _keep = tab
    check(_lib().bigdl_w_xform_multi(ptr(table), C.c_int(nj), C.c_longlong(total), _s()), "w_xform_multi")
    for c in ents:
        c["gen"] = arena.shadow_gen


_S1_XFORM = {}  # (K, C, R, S) → the single full-filter class list of a stride-1 dgrad


def _subfilters(w4, classes, gkey=None):
    """All parity sub-filters of a strided dgrad in ONE gather: W'_ab[c][j'][i'][k] =
    W[k][c][rs[Ra-1-j']][ss[Sb-1-i']], indexed straight from the weight's physical storage (KRSC
    in the arena) with a cached index vector — one small kernel per layer per step."""
    K, C_, R, S = w4.shape
    krsc = w4.permute(0, 2, 3, 1)
    phys = krsc if krsc.is_contiguous() else krsc.contiguous()
    # HIP transform kernel (weight_xform.hip): every class in one launch, no index tensor.  The
    # ctypes argument block is built once per (shape, geometry) — this runs per layer per step, so
    # the hot path is one dict lookup.  ``gkey`` is the caller's hashable geometry key (the internal
    # callers have one); without it the key is derived from the class list's contents.
    if gkey is None:
        gkey = tuple((a, b, tuple(rs), tuple(ss)) for (a, b, rs, ss, *_r) in classes)
    key = ("xf", K, C_, R, S, gkey)
    ent = _SUBFILTER_IDX.get(key)
    live = [c for c in classes if c[2] and c[3]] if ent is None else None
    if (phys.dtype == _bf16 and phys.is_cuda and C_ % 8 == 0 and K % 8 == 0 and _al16(phys)
            and (ent is not None or (0 < len(live) <= 4 and max(max(len(c[2]), len(c[3])) for c in live) <= 8))):
        if ent is None:
            n = [len(rs) * len(ss) * C_ * K if (rs and ss) else 0 for (a, b, rs, ss, *_r) in classes]
            ros, sos, rm, sm, offs = [], [], [0] * 32, [0] * 32, []
            off = 0
            for (a, b, rs, ss, *_r), ni in zip(classes, n):
                if ni:
                    q = len(ros)
                    ros.append(len(rs))
                    sos.append(len(ss))
                    rm[q * 8:q * 8 + len(rs)] = rs[::-1]
                    sm[q * 8:q * 8 + len(ss)] = ss[::-1]
                    offs.append(off)
                off += ni
            IA, LA = C.c_int * 32, C.c_longlong * 4
            ent = (n, sum(n), len(ros), IA(*ros), IA(*sos), IA(*rm), IA(*sm), LA(*offs))
            _SUBFILTER_IDX[key] = ent
        n, total, ncls, a_ro, a_so, a_rm, a_sm, a_off = ent
        arena = _shadow_arena(phys)
        ck = (phys.data_ptr(), key)
        if arena is not None:
            c = _XFC.get(ck)
            if c is not None:
                if c["gen"] != arena.shadow_gen:
                    _xf_refresh(arena)
                if c["gen"] == arena.shadow_gen:
                    return c["views"]
        out = torch.empty(total, dtype=_bf16, device=w4.device)
        check(_lib().bigdl_w_dgrad_xform(ptr(phys), ptr(out), K, R, S, C_, ncls, a_ro, a_so, a_rm, a_sm, a_off, _s()),
              "w_dgrad_xform")
        res, off = [], 0
        for (a, b, rs, ss, *_r), ni in zip(classes, n):
            res.append(out[off:off + ni].view(C_, len(rs), len(ss), K) if ni else None)
            off += ni
        if arena is not None:
            _XFC[ck] = {"gen": arena.shadow_gen, "out": out, "views": res, "arena": id(arena), "phys": phys,
                        "args": (K, R, S, C_, ncls, a_ro, a_so, a_rm, a_sm, a_off)}
            _XF_TABLE.pop(id(arena), None)  # the job table gains an entry
        return res
    key = (K, C_, R, S, tuple((a, b, tuple(rs), tuple(ss)) for (a, b, rs, ss, *_r) in classes), w4.device)
    ent = _SUBFILTER_IDX.get(key)
    if ent is None:
        parts, sizes = [], []
        kk = torch.arange(K).view(1, 1, 1, K)
        cc = torch.arange(C_).view(C_, 1, 1, 1)
        for (a, b, rs, ss, *_r) in classes:
            if not rs or not ss:
                sizes.append(0)
                continue
            rr = torch.tensor(rs[::-1]).view(1, len(rs), 1, 1)
            sv = torch.tensor(ss[::-1]).view(1, 1, len(ss), 1)
            idx = ((kk * R + rr) * S + sv) * C_ + cc  # [C][Ra][Sb][K] → offset in (K, R, S, C)
            parts.append(idx.reshape(-1))
            sizes.append(idx.numel())
        ent = (torch.cat(parts).to(w4.device), sizes)
        _SUBFILTER_IDX[key] = ent
    idx, sizes = ent
    flat = phys.reshape(-1)[idx]
    out, off = [], 0
    for (a, b, rs, ss, *_r), n in zip(classes, sizes):
        out.append(flat[off:off + n].view(C_, len(rs), len(ss), K) if n else None)
        off += n
    return out


_STRIDED_CLASSES = {}  # geometry → parity-class list (one object per geometry: _subfilters keys on it)


def _parity_classes(H, W, R, S, sh, sw, ph, pw):
    classes = []
    for a in range(sh):
        ra = (a + ph) % sh
        rs = list(range(ra, R, sh))
        for b in range(sw):
            sb = (b + pw) % sw
            ss = list(range(sb, S, sw))
            ho = (H - a + sh - 1) // sh
            wo = (W - b + sw - 1) // sw
            if ho <= 0 or wo <= 0:
                continue
            classes.append((a, b, rs, ss, ho, wo, (a + ph - ra) // sh, (b + pw - sb) // sw))
    return classes


def _dgrad_strided(gy, w4, x_shape, stride, pad, dilation, residual=None, lazy=False):
    """Strided backward-data by sub-pixel decomposition: the input-gradient pixels of parity
    (a, b) = (h mod sh, w mod sw) receive only the filter taps r ≡ a + ph (mod sh), s ≡ b + pw
    (mod sw), so each parity class is a STRIDE-1 convolution of gy with a flipped sub-filter whose
    output is scattered to pixels (sh·ho + a, sw·wo + b) — sh·sw launches of the implicit-GEMM
    kernel and no zero-stuffed FLOPs (reference: SpatialConvolution.updateGradInput's col2im,
    DL/nn/SpatialConvolution.scala:656-735)."""
    N_, C_, H, W = x_shape
    K, Ci, R, S = w4.shape
    sh, sw = stride
    ph, pw = pad
    if tuple(dilation) != (1, 1) or C_ % 8 or K % 8 or gy.shape[1] != K:
        return None
    if residual is not None and not (residual.shape == (N_, C_, H, W) and residual.dtype == _bf16 and
                                     residual.is_contiguous(memory_format=torch.channels_last) and _al16(residual)):
        return None
    P, Q = gy.shape[2], gy.shape[3]
    ckey = (H, W, R, S, sh, sw, ph, pw)
    classes = _STRIDED_CLASSES.get(ckey)
    if classes is None:
        classes = _STRIDED_CLASSES[ckey] = _parity_classes(H, W, R, S, sh, sw, ph, pw)
    if lazy and residual is None and R == 1 and S == 1 and ph == 0 and pw == 0:
        # 1×1 stride-s: only parity (0, 0) has a tap — return its pixels densely packed and let the
        # consumer read them as a strided residual (no zero-filled full-resolution tensor)
        (a, b, rs, ss, ho, wo, ea, eb) = classes[0]
        wt = _subfilters(w4, classes, ckey)[0]
        tmp = torch.empty((N_, C_, ho, wo), dtype=_bf16, device=gy.device, memory_format=torch.channels_last)
        _tiled_launch((N_, P, Q, K, C_, 1, 1, (1, 1), (0, 0), (1, 1)), lambda t: check(_lib().bigdl_conv_fwd_ex(
            ptr(gy), ptr(wt), ptr(None), ptr(None), ptr(tmp), ptr(None), N_, P, Q, K, C_, 1, 1, ho, wo, 1, 1, 0, 0, 1,
            1, 0, t[0], t[1], t[2], _s()), "conv_dgrad_1x1s_lazy"))
        return R_.StridedGrad(tmp, stride, (N_, C_, H, W))
    gx = torch.empty((N_, C_, H, W), dtype=_bf16, device=gy.device, memory_format=torch.channels_last)
    if any(not rs or not ss for (_, _, rs, ss, *_r) in classes):
        # some parity receives no tap (e.g. 1x1 stride 2): those pixels are exactly zero / the residual
        if residual is not None:
            gx.copy_(residual)
        else:
            gx.zero_()
    subs = _subfilters(w4, classes, ckey)
    for ci, (a, b, rs, ss, ho, wo, ea, eb) in enumerate(classes):
        if not rs or not ss:
            continue
        wt = subs[ci]
        Ra, Sb = len(rs), len(ss)
        res_ok = residual is not None  # tap-less parities already hold the residual (copied above)
        check(_lib().bigdl_conv_fwd_scatter(ptr(gy), ptr(wt), ptr(None), ptr(residual if res_ok else None), ptr(gx),
                                            ptr(None), N_, P, Q, K, C_, Ra, Sb, ho, wo, 1, 1, Ra - 1 - ea,
                                            Sb - 1 - eb, 1, 1, 0, sh, sw, a, b, H, W, 0, 0, 0, _s()),
              "conv_dgrad_strided")
    return gx


def _dgrad_1x1_strided(gy, w4, x_shape, stride):
    """1×1 stride-s backward-data: GEMM into the strided positions, zeros elsewhere."""
    N_, C_, H, W = x_shape
    K = w4.shape[0]
    if C_ % 4 or K % 8:
        return None
    wt = w4.reshape(K, C_).t().contiguous()  # [C][K] = [C][1][1][K]
    P, Q = gy.shape[2], gy.shape[3]
    tmp = torch.empty((N_, C_, P, Q), dtype=_bf16, device=gy.device, memory_format=torch.channels_last)
    check(_lib().bigdl_conv_fwd(ptr(gy), ptr(wt), ptr(None), ptr(tmp), N_, P, Q, K, C_, 1, 1, P, Q, 1, 1, 0, 0, 1, 1,
                                0, _s()), "conv_dgrad_1x1s")
    gx = torch.empty((N_, C_, H, W), dtype=_bf16, device=gy.device, memory_format=torch.channels_last)
    gx.zero_()
    gx[:, :, ::stride[0], ::stride[1]] = tmp
    return gx


# ------------------------------------------------------------------------------------------------ async wgrad
# Backward-weight convolutions are compute-bound and independent of the backward-data chain, which
# alternates with memory-bound BatchNorm passes: inside an optimizer step they run on a second HIP
# stream so the two overlap (cdna_hip_programming.md Guideline 15).  The optimizer joins the side
# stream before anything reads the gradients (update, reduce-scatter).  Off outside optimizer steps
# (a plain module.backward() leaves every gradient complete on the current stream) and during
# HIP-graph capture.
_WG = {"on": False, "streams": {}}


def async_wgrad(on: bool) -> None:
    _WG["on"] = bool(on) and bool(config.get_property("bigdl.conv.asyncWgrad"))


def _new_side_stream(dev):
    """The wgrad side stream.  ``BIGDL_WGRAD_CUMASK=keep/period`` (e.g. ``3/4``) restricts it to the
    CUs with ``i % period < keep`` (hipExtStreamCreateWithCUMask), so the weight gradients can never
    hold every CU while the backward-data chain on the step stream waits for workgroup slots."""
    spec = __import__("os").environ.get("BIGDL_WGRAD_CUMASK", "")
    if spec:
        keep, period = (int(v) for v in spec.split("/"))
        f = N._load().bigdl_stream_create_cumask  # the raw CDLL symbol: a 64-bit handle
        f.restype = C.c_longlong
        with torch.cuda.device(dev):
            h = f(C.c_int(keep), C.c_int(period))
        if h:
            return torch.cuda.ExternalStream(h, device=dev)
        __import__("logging").getLogger("bigdl.ops").warning("CU-masked wgrad stream %s unavailable; using a plain stream", spec)
    return torch.cuda.Stream(device=dev)


def _wgrad_side_stream(t):
    if not _WG["on"] or not t.is_cuda or torch.cuda.is_current_stream_capturing():
        return None
    dev = t.device
    st = _WG["streams"].get(dev)
    if st is None:
        st = _WG["streams"][dev] = _new_side_stream(dev)
    st.wait_stream(torch.cuda.current_stream(dev))  # gy / x / zeroed gradients are ready
    return st


def join_wgrad(stream=None) -> None:
    """Make ``stream`` (default: the current stream) wait for every wgrad queued on the side stream."""
    if not _WG["streams"] or torch.cuda.is_current_stream_capturing():
        return
    cur = stream or torch.cuda.current_stream()
    st = _WG["streams"].get(cur.device)
    if st is not None:
        cur.wait_stream(st)


#: total blocks the wgrad kernel aims for (split-K over pixels); 0 = per-shape heuristic below.
#: tools/bench_conv.py --wgrad-sweep A/Bs fixed values.
_WGRAD_TARGET_BLOCKS = [int(__import__("os").environ.get("BIGDL_WGRAD_BLOCKS", "0"))]


def _wgrad_blocks(M, C_, K):
    """Split-K target measured on the ResNet-50 shapes (profiles/r1_wgrad_sweep.txt): 384 blocks
    (1.5 per CU) minimises atomic traffic for most layers; the very tall, narrow 56² layers and the
    C=3 stem need more blocks to fill the chip."""
    if _WGRAD_TARGET_BLOCKS[0] > 0:
        return _WGRAD_TARGET_BLOCKS[0]
    if C_ <= 8:
        return 2048
    if M >= 400000 and (C_ <= 64 or K <= 64):
        return 768
    return 384


def _wgrad_launch(x, gy, w4, gw_acc, scale, stride, pad, dilation, pad_slot):
    """Backward-weight conv on the current stream; returns the activation operand it read."""
    N_, C_, H, W = x.shape
    K, Ci, R, S = w4.shape
    xx, cc = x, C_
    if C_ % 8:
        cc = 4 if (C_ <= 4 and tuple(dilation) == (1, 1)) else (C_ + 7) // 8 * 8
        xx = _pad_channels(x, cc, pad_slot, reuse=True)
    direct = (cc == C_ and gw_acc.dtype == _f32 and gw_acc.permute(0, 2, 3, 1).is_contiguous())
    if direct:
        target = gw_acc.permute(0, 2, 3, 1)
    else:
        target = torch.empty((K, R, S, cc), dtype=_f32, device=x.device)
        if zero_fill(target) is NotImplemented:
            target.zero_()
    P, Q = gy.shape[2], gy.shape[3]
    if isinstance(gy, R_.BNGrad):  # dY = the BN input gradient, applied while loading dY
        check(_lib().bigdl_conv_wgrad_bnbwd(ptr(xx), ptr(gy.g), ptr(gy.x), ptr(gy.coef), ptr(target),
                                            _f(scale if direct else 1.0), N_, H, W, cc, K, R, S, P, Q, stride[0],
                                            stride[1], pad[0], pad[1], dilation[0], dilation[1],
                                            -_wgrad_blocks(N_ * P * Q, cc, K), _s()), "conv_wgrad_bnbwd")
    else:
        # kernel selection key: ("wg", geometry) → (target blocks, k-tile pixel depth); 0 = heuristic
        wkey = ("wg", N_, H, W, cc, K, R, S, tuple(stride), tuple(pad), tuple(dilation))
        _tiled_launch(wkey, lambda t: check(_lib().bigdl_conv_wgrad_t(
            ptr(xx), ptr(gy), ptr(target), _f(scale if direct else 1.0), N_, H, W, cc, K, R, S, P, Q, stride[0],
            stride[1], pad[0], pad[1], dilation[0], dilation[1], -(t[0] or _wgrad_blocks(N_ * P * Q, cc, K)), t[1],
            _s()), "conv_wgrad"))
    if not direct:
        if cc == 4 and C_ <= 4 and gw_acc.dtype == _f32 and gw_acc.dim() == 4:
            # the RGB stem's C4 gradient folded onto the KCRS master gradient natively (weight_x3.hip)
            check(_lib().bigdl_c4_wgrad_fold(ptr(target), ptr(gw_acc), K, C_, R, S,
                                             *(C.c_longlong(v) for v in gw_acc.stride()), _f(scale), _s()),
                  "c4_wgrad_fold")
        else:
            gw_acc.add_(target[..., :C_].permute(0, 3, 1, 2), alpha=scale)
    return xx


def bngrad_consumable(g, x, w4, stride, pad, groups=1):
    """A deferred BN gradient can feed this conv's backward prologues: 1×1, stride 1, unpadded,
    one group, channel counts the pointwise kernel tiles exactly (K % 32, C % 8), dense bf16."""
    if not isinstance(g, R_.BNGrad) or groups != 1 or tuple(stride) != (1, 1) or tuple(pad) != (0, 0):
        return False
    K, Ci, R, S = w4.shape
    if R != 1 or S != 1 or K % 32 or x.dim() != 4 or x.shape[1] % 8 or g.shape[1] != K:
        return False
    cl = torch.channels_last
    return all(t.is_cuda and t.dtype == _bf16 and t.is_contiguous(memory_format=cl) and _al16(t) for t in (g.g, g.x)) \
        and g.g.shape == g.x.shape and _f32vec(g.coef, 3 * K) and x.dtype == _bf16 \
        and x.is_contiguous(memory_format=cl) and _al16(x)


@register("conv2d_backward")
def conv2d_backward(gy, x, w4, stride, pad, dilation=(1, 1), groups=1, need_input=True, gw_acc=None, gb_acc=None,
                    scale=1.0, residual=None, bn_fuse=None, pad_slot=None, lazy_strided=False, pro=None):
    """``lazy_strided``: a 1×1 stride-s unpadded conv may return its input gradient as a
    :class:`~bigdl.ops.reference.StridedGrad` (the caller sums it as a strided residual).  ``gy`` may
    be a deferred :class:`~bigdl.ops.reference.BNGrad` (consumed in the operand prologues of a 1×1
    stride-1 conv, materialised otherwise)."""
    if isinstance(gy, torch.Tensor) and gy.dtype == _f32 and x.dtype == _f32 and F3.enabled(gy):
        # fp32 (bf16x3): the bf16 epilogue fusions are optional — bn_fuse is left unconsumed (the BN
        # runs its own backward), a lazy strided gradient is returned dense
        r = F3.conv_backward(gy, x, w4, stride, pad, dilation, groups, need_input, gw_acc, gb_acc, scale, residual,
                             slot=pad_slot, bn_fuse=bn_fuse, lazy_strided=lazy_strided, pro=pro)
        if r is not NotImplemented or pro is not None:
            return r
    if pro is not None:
        return NotImplemented
    if isinstance(gy, R_.BNGrad) and not (bngrad_consumable(gy, x, w4, stride, pad, groups) and gb_acc is None):
        gy = gy.dense()
    if isinstance(gy, R_.BNGrad):
        if need_input:
            gi = _dgrad_s1(gy, w4, x.shape, pad, dilation, residual, bn_fuse)
            if gi is None:
                return conv2d_backward(gy.dense(), x, w4, stride, pad, dilation, groups, need_input, gw_acc, gb_acc,
                                       scale, residual, bn_fuse, pad_slot, lazy_strided)
        else:
            gi = None
        if gw_acc is not None and scale != 0:
            side = _wgrad_side_stream(gy.g) if _WG["on"] else None
            if side is None:
                _wgrad_launch(x, gy, w4, gw_acc, scale, stride, pad, dilation, pad_slot)
            else:
                with torch.cuda.stream(side):
                    xx = _wgrad_launch(x, gy, w4, gw_acc, scale, stride, pad, dilation, pad_slot)
                for t in (x, xx, gy.g, gy.x, gy.coef):
                    t.record_stream(side)
        return gi
    if isinstance(residual, R_.StridedGrad) and (tuple(stride) != (1, 1) or groups > 1 or gy.dtype != _bf16):
        residual = residual.dense()
    if groups > 1 and residual is None and bn_fuse is None and _depthwise_ok(x, w4, groups):
        return _depthwise_bwd(gy, x, w4, stride, pad, dilation, need_input, gw_acc, gb_acc, scale)
    if groups > 1 and residual is None and bn_fuse is None and _grouped_ok(x, w4, groups) and gy.dtype == _bf16:
        r = _conv_bwd_grouped_1(gy, x, w4, stride, pad, dilation, groups, need_input, gw_acc, gb_acc, scale)
        if r is not NotImplemented:
            return r
        # no 8-aligned packing: one groups=1 backward per channel slice (gradient-weight rows of a
        # group are a contiguous block of the arena, so they accumulate in place)
        C_, K = x.shape[1], w4.shape[0]
        Cg, Kg = C_ // groups, K // groups
        gi = torch.empty(x.shape, dtype=_bf16, device=x.device,
                         memory_format=torch.channels_last) if need_input else None
        for g in range(groups):
            r = conv2d_backward(_group_slice(gy, g, Kg), _group_slice(x, g, Cg), w4[g * Kg:(g + 1) * Kg], stride,
                                pad, dilation, 1, need_input,
                                None if gw_acc is None else gw_acc[g * Kg:(g + 1) * Kg],
                                None if gb_acc is None else gb_acc[g * Kg:(g + 1) * Kg], scale)
            if r is NotImplemented:
                return NotImplemented
            if need_input:
                gi[:, g * Cg:(g + 1) * Cg] = r
        return gi
    if not _conv_geom_ok_slot(x, w4, groups, dilation, pad_slot) or gy.dtype != _bf16:
        return NotImplemented
    if not gy.is_contiguous(memory_format=torch.channels_last) or not _al16(gy):
        return NotImplemented
    N_, C_, H, W = x.shape
    K, Ci, R, S = w4.shape
    if K % 8:
        # odd output-channel count (LeNet's 6 / 12 maps): zero-pad the gradient's channels (and
        # the filter bank) to a multiple of 8 — padded channels contribute exactly zero
        if residual is not None or bn_fuse is not None:
            return NotImplemented
        K8 = (K + 7) // 8 * 8
        P, Q = gy.shape[2], gy.shape[3]
        gyp = torch.zeros((N_, P, Q, K8), dtype=_bf16, device=gy.device).permute(0, 3, 1, 2)
        gyp[:, :K] = gy
        wk = torch.zeros((K8, R, S, Ci), dtype=w4.dtype, device=w4.device)
        wk[:K] = w4.permute(0, 2, 3, 1)
        tmp = None
        if gw_acc is not None and scale != 0:
            tmp = torch.zeros((K8, R, S, Ci), dtype=_f32, device=x.device).permute(0, 3, 1, 2)
        gi = conv2d_backward(gyp, x, wk.permute(0, 3, 1, 2), stride, pad, dilation, groups, need_input, tmp, None,
                             scale, pad_slot=pad_slot)
        if gi is NotImplemented:
            return NotImplemented
        if tmp is not None:
            gw_acc.add_(tmp[:K])
        if gb_acc is not None and scale != 0:
            gb_acc.add_(gy.float().sum((0, 2, 3)), alpha=scale)
        return gi
    gi = None
    wg_done = False
    if gw_acc is not None and scale != 0 and _WG["on"] and _WG_FIRST[0]:
        # fork the weight gradient BEFORE the data gradient: the side stream's wait then covers only
        # what produced gy / x, so the wgrad runs beside this layer's dgrad instead of after it
        wg_done = _wgrad_async_or_inline(x, gy, w4, gw_acc, scale, stride, pad, dilation, pad_slot)
    if need_input:
        res_done = False
        if stride == (1, 1) or tuple(stride) == (1, 1):
            gi = _dgrad_s1(gy, w4, x.shape, pad, dilation, residual, bn_fuse)
            res_done = gi is not None
            if gi is None and residual is not None:
                gi = _dgrad_s1(gy, w4, x.shape, pad, dilation)
        else:
            gi = _dgrad_strided(gy, w4, x.shape, tuple(stride), tuple(pad), dilation, residual,
                                lazy=lazy_strided and bn_fuse is None)
            res_done = gi is not None
        if gi is None:  # dilated strided backward-data: library path
            N.note_fallback("conv2d_backward.dgrad", "dilated-strided", (gy, x, w4))
            gi = R_.conv2d_backward(gy, x, w4, stride, pad, dilation, groups, True, None, None, 0.0)
        if residual is not None and not res_done:
            gi = R_.as_dense(gi) + R_.as_dense(residual)
    if gw_acc is not None and scale != 0 and not wg_done:
        _wgrad_async_or_inline(x, gy, w4, gw_acc, scale, stride, pad, dilation, pad_slot)
    if gb_acc is not None and scale != 0:
        gb_acc.add_(gy.float().sum((0, 2, 3)), alpha=scale)
    return gi


#: conv2d_backward forks its weight gradient onto the side stream BEFORE the data gradient is
#: enqueued, so the two run side by side (BIGDL_WGRAD_FIRST=0: after, the round-3 order; 22.08 vs
#: 22.94 ms/step, profiles/r4_bn_replicas_ab.txt)
_WG_FIRST = [__import__("os").environ.get("BIGDL_WGRAD_FIRST", "1") == "1"]


def _wgrad_async_or_inline(x, gy, w4, gw_acc, scale, stride, pad, dilation, pad_slot) -> bool:
    side = _wgrad_side_stream(gy) if _WG["on"] else None
    if side is None:
        _wgrad_launch(x, gy, w4, gw_acc, scale, stride, pad, dilation, pad_slot)
    else:
        with torch.cuda.stream(side):
            xx = _wgrad_launch(x, gy, w4, gw_acc, scale, stride, pad, dilation, pad_slot)
        # the caching allocator must not hand these blocks to the compute stream while the side
        # stream still reads them
        for t in (x, xx, gy):
            t.record_stream(side)
    return True


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
             lrs=None, wds=None, first_dev=None):
    """Fused SGD over a flat fp32 slice; ``g`` is fp32 or bf16 (the bf16-wire reduce-scatter output,
    read directly by the kernel instead of being unpacked into an fp32 shard first)."""
    F3.mark_dirty(w)
    n = w.numel()
    if w.dtype != _f32 or g.dtype not in (_f32, _bf16) or not _vec_ok(w, buf, lrs, wds, n=n):
        return NotImplemented
    g16 = g.dtype == _bf16
    if not (g.is_cuda and g.is_contiguous() and g.numel() == n and g.data_ptr() % (8 if g16 else 16) == 0):
        return NotImplemented
    if shadow is not None and not (shadow.dtype == _bf16 and shadow.is_contiguous() and shadow.numel() == n
                                   and shadow.data_ptr() % 8 == 0):
        return NotImplemented
    if momentum != 0 and buf is None:
        return NotImplemented
    if first_dev is not None and not (first_dev.is_cuda and first_dev.dtype == _f32):
        return NotImplemented
    fn = _lib().bigdl_sgd_g16 if g16 else _lib().bigdl_sgd
    check(fn(ptr(w), ptr(g), ptr(buf if momentum != 0 else None), ptr(shadow), ptr(lrs), ptr(wds),
             _ll(n), _f(lr), _f(momentum), _f(dampening), _f(weight_decay), C.c_int(int(bool(nesterov))),
             C.c_int(int(bool(first_step))), _f(grad_scale), ptr(first_dev), _s()), "sgd")
    return w


@register("adam_step")
def adam_step(w, g, m, v, lr, beta1, beta2, eps, step, weight_decay=0.0, grad_scale=1.0, shadow=None):
    import math
    F3.mark_dirty(w)
    n = w.numel()
    if w.dtype != _f32 or g.dtype != _f32 or not _vec_ok(w, g, m, v, n=n):
        return NotImplemented
    if shadow is not None and not (shadow.dtype == _bf16 and shadow.is_contiguous() and shadow.numel() == n
                                   and shadow.data_ptr() % 8 == 0):
        return NotImplemented
    step_size = lr * math.sqrt(1 - beta2 ** step) / (1 - beta1 ** step)
    check(_lib().bigdl_adam(ptr(w), ptr(g), ptr(m), ptr(v), ptr(shadow), _ll(n), _f(step_size), _f(beta1), _f(beta2),
                            _f(eps), _f(weight_decay), _f(grad_scale), _s()), "adam")
    return w


@register("adam_step_dev")
def adam_step_dev(w, g, m, v, dev_n, lr, lr_decay, beta1, beta2, eps, weight_decay=0.0, grad_scale=1.0, shadow=None):
    """Adam whose iteration count ``dev_n`` (fp32 [1], before this step) is read on the device —
    the replay-safe form for HIP-graph capture; the caller advances ``dev_n`` afterwards."""
    F3.mark_dirty(w)
    n = w.numel()
    if w.dtype != _f32 or g.dtype != _f32 or not _vec_ok(w, g, m, v, n=n) or not (dev_n.is_cuda and
                                                                                  dev_n.dtype == _f32):
        return NotImplemented
    if shadow is not None and not (shadow.dtype == _bf16 and shadow.is_contiguous() and shadow.numel() == n
                                   and shadow.data_ptr() % 8 == 0):
        return NotImplemented
    check(_lib().bigdl_adam_dev(ptr(w), ptr(g), ptr(m), ptr(v), ptr(shadow), _ll(n), ptr(dev_n), _f(lr), _f(lr_decay),
                                _f(beta1), _f(beta2), _f(eps), _f(weight_decay), _f(grad_scale), _s()), "adam_dev")
    return w


@register("adagrad_step")
def adagrad_step(w, g, s, lr, lr_decay, n, weight_decay=0.0, grad_scale=1.0, shadow=None, dev_n=None):
    """Fused Adagrad update (bigdl_adagrad); ``dev_n`` (fp32 [1] on the device, the iteration count
    before this step) makes it replay-safe under HIP-graph capture, else ``n`` (host) is used."""
    F3.mark_dirty(w)
    numel = w.numel()
    g16 = g.dtype == _bf16  # the DistriOptimizer's bf16 wire shard, widened on load
    if w.dtype != _f32 or s.dtype != _f32 or not _vec_ok(w, s, n=numel):
        return NotImplemented
    if g16:
        if not (g.is_cuda and g.is_contiguous() and g.numel() == numel and g.data_ptr() % 8 == 0):
            return NotImplemented
    elif g.dtype != _f32 or not _vec_ok(g, n=numel):
        return NotImplemented
    if dev_n is not None and not (dev_n.is_cuda and dev_n.dtype == _f32):
        return NotImplemented
    if shadow is not None and not (shadow.dtype == _bf16 and shadow.is_contiguous() and shadow.numel() == numel
                                   and shadow.data_ptr() % 8 == 0):
        return NotImplemented
    clr = lr / (1 + n * lr_decay)
    fn = _lib().bigdl_adagrad_g16 if g16 else _lib().bigdl_adagrad
    check(fn(ptr(w), ptr(g), ptr(s), ptr(shadow), _ll(numel), _f(clr), ptr(dev_n), _f(lr), _f(lr_decay),
             _f(weight_decay), _f(grad_scale), _s()), "adagrad")
    return w


# ------------------------------------------------------------------------------------------------ LSTM
def _row_view(t, rows, cols):
    """(row stride) of a 2-D view with unit column stride, else None."""
    if t is None:
        return 0
    if t.dim() != 2 or t.shape[0] != rows or t.shape[1] != cols or t.stride(1) != 1:
        return None
    return t.stride(0)


def _f32c(t, n):
    return t is None or (t.dtype == _f32 and t.is_contiguous() and t.numel() == n and t.is_cuda)


@register("lstm_cell_forward")
def lstm_cell_forward(xg, hg, c_prev, h_out=None, c_out=None, act_out=None, tc_out=None):
    B, G = xg.shape
    H = G // 4
    dt = xg.dtype
    if dt not in (_bf16, _f32) or G != 4 * H or (hg is not None and hg.dtype != dt):
        return NotImplemented
    if c_prev.dtype != _f32 or not c_prev.is_contiguous() or c_prev.shape != (B, H):
        return NotImplemented
    ldx, ldhg = _row_view(xg, B, G), _row_view(hg, B, G)
    if ldx is None or ldhg is None:
        return NotImplemented
    h = h_out if h_out is not None else torch.empty(B, H, device=xg.device, dtype=dt)
    ldh = _row_view(h, B, H)
    if ldh is None or h.dtype != dt:
        return NotImplemented
    c = c_out if c_out is not None else torch.empty(B, H, device=xg.device, dtype=_f32)
    act = act_out if act_out is not None else torch.empty(B, G, device=xg.device, dtype=_f32)
    tc = tc_out if tc_out is not None else torch.empty(B, H, device=xg.device, dtype=_f32)
    if not (_f32c(c, B * H) and _f32c(act, B * G) and _f32c(tc, B * H)):
        return NotImplemented
    check(_lib().bigdl_lstm_fwd(ptr(xg), C.c_long(ldx), ptr(hg), C.c_long(ldhg), ptr(c_prev), ptr(h), C.c_long(ldh),
                                ptr(c), ptr(act), ptr(tc), B, H, 0 if dt == _bf16 else 1, _s()), "lstm_fwd")
    return h, c, act, tc


@register("lstm_cell_backward")
def lstm_cell_backward(gh, gh2, gc_next, act, tc, c_prev, dg_out=None):
    B, H = gh.shape
    dt = gh.dtype
    if dt not in (_bf16, _f32):
        return NotImplemented
    ldgh = _row_view(gh, B, H)
    if ldgh is None:
        return NotImplemented
    if gh2 is not None and (gh2.dtype != dt or not gh2.is_contiguous() or gh2.shape != (B, H)):
        return NotImplemented
    if not (_f32c(gc_next, B * H) and _f32c(act, B * 4 * H) and _f32c(tc, B * H) and _f32c(c_prev, B * H)):
        return NotImplemented
    dg = dg_out if dg_out is not None else torch.empty(B, 4 * H, device=gh.device, dtype=dt)
    lddg = _row_view(dg, B, 4 * H)
    if lddg is None or dg.dtype != dt:
        return NotImplemented
    dc = torch.empty(B, H, device=gh.device, dtype=_f32)
    check(_lib().bigdl_lstm_bwd(ptr(gh), C.c_long(ldgh), ptr(gh2), ptr(gc_next), ptr(act), ptr(tc), ptr(c_prev),
                                ptr(dg), C.c_long(lddg), ptr(dc), B, H, 0 if dt == _bf16 else 1, _s()), "lstm_bwd")
    return dg, dc


# ------------------------------------------------------------------------------------------------ int8 (K26)
@register("quant_rows")
def quant_rows(x2d, kp=None):
    if x2d.dim() != 2 or x2d.dtype not in (_bf16, _f32) or x2d.stride(1) != 1:
        return NotImplemented
    M, K = x2d.shape
    kp = kp or (K + 63) // 64 * 64
    if kp % 16 or kp < K or M == 0 or K == 0:
        return NotImplemented
    q = torch.empty((M, kp), dtype=torch.int8, device=x2d.device)
    sc = torch.empty(M, dtype=_f32, device=x2d.device)
    check(_lib().bigdl_quant_rows(ptr(x2d), C.c_int(1 if x2d.dtype == _bf16 else 0), _ll(M), C.c_int(K),
                                  _ll(x2d.stride(0)), ptr(q), C.c_int(kp), ptr(sc), _s()), "quant_rows")
    return q, sc


# ---- int8 implicit-GEMM convolution (conv_i8.hip) ----------------------------------------------
def conv_i8_supported(C_, R, S, groups=1) -> bool:
    return groups == 1 and (C_ == 64 or C_ % 16 == 0) and R * S <= 64


def conv_i8_weight(qweight, K, C_, R, S):
    """Per-output-channel int8 weights of the (c, kh, kw)-ordered GEMM view → the kernel's
    [K][ldw] rows in (r, s, c) order, zero-padded to whole 128-byte k-tiles.  Returns (w, ldw)."""
    kg = C_ * R * S
    w = qweight[:, :kg].reshape(K, C_, R, S).permute(0, 2, 3, 1).reshape(K, R * S, C_)
    if C_ == 64:
        KT = (R * S + 1) // 2
        ldw = KT * 128
        out = torch.zeros((K, ldw), dtype=torch.int8, device=qweight.device)
        out[:, :kg] = w.reshape(K, kg)
        return out, ldw
    cp = (C_ + 127) // 128 * 128  # each tap's channels padded to whole 128-byte k-tiles
    ldw = R * S * cp
    out = torch.zeros((K, R * S, cp), dtype=torch.int8, device=qweight.device)
    out[:, :, :C_] = w
    return out.reshape(K, ldw), ldw


def quant_images(x):
    """Per-image dynamic int8 quantisation of an NHWC bf16 activation: (xq int8 same layout, sx
    fp32 [N] dequantisation scales = amax / 127)."""
    N_ = x.shape[0]
    per = x.numel() // N_
    xq = torch.empty_like(x, dtype=torch.int8)
    sx = torch.empty(N_, dtype=_f32, device=x.device)
    amax = torch.empty(N_, dtype=_f32, device=x.device)
    check(_lib().bigdl_quant_img(ptr(x), C.c_int(N_), _ll(per), ptr(amax), ptr(xq), ptr(sx), _s()), "quant_img")
    return xq, sx


def conv2d_i8_forward(x, wq, ldw, w_scale, bias, K, R, S, stride, pad, dilation, out_hw, relu=False):
    """int8 conv of a channels-last bf16 activation (quantised per image here) with prepared
    weights (:func:`conv_i8_weight`); ``pad`` = (top, left), ``out_hw`` = (P, Q) from the full
    padding.  Returns the bf16 output (N, K, P, Q), channels-last memory, or NotImplemented."""
    if not (x.is_cuda and x.dim() == 4 and x.dtype == _bf16 and x.is_contiguous(memory_format=torch.channels_last)):
        return NotImplemented
    N_, C_, H, W = x.shape
    if not conv_i8_supported(C_, R, S) or K % 8 or not _al16(x):
        return NotImplemented
    P, Q = out_hw
    xq, sx = quant_images(x)
    y = torch.empty((N_, K, P, Q), dtype=_bf16, device=x.device, memory_format=torch.channels_last)
    b = bias.float().contiguous() if bias is not None else None
    check(_lib().bigdl_conv_i8_fwd(ptr(xq), ptr(wq), C.c_int(ldw), ptr(sx), ptr(w_scale), ptr(b), ptr(y), C.c_int(K),
                                   N_, H, W, C_, K, R, S, P, Q, stride[0], stride[1], pad[0], pad[1], dilation[0],
                                   dilation[1], C.c_int(1 if relu else 0), _s()), "conv_i8_fwd")
    return y


def _i8_act(N_, C_, H, W, dev, tail):
    """An int8 NHWC activation (logical NCHW, channels-last); ``tail``: 16 more bytes after it in
    the same allocation, which the kernels that write the unsigned code fill with 0x80 (the code of
    0, read by a consumer conv for its padded taps)."""
    n = N_ * C_ * H * W
    if not tail:
        return torch.empty((N_, C_, H, W), dtype=torch.int8, device=dev, memory_format=torch.channels_last)
    buf = torch.empty(n + 16, dtype=torch.int8, device=dev)
    return buf[:n].view(N_, H, W, C_).permute(0, 3, 1, 2)


def _tag(t, scale, u8):
    t._qscale = float(scale) if scale is not None else None
    t._qzero = 128 if u8 else 0
    t._qtail = bool(u8)
    return t


def quant_static(x, scale, u8=False):
    """Calibrated (static) int8 quantisation of a channels-last fp32 / bf16 activation with one
    scale: int8 tensor of the same logical shape and memory layout, tagged ``_qscale``.  ``u8``: the
    input is non-negative (post-ReLU) and is stored as unsigned 8-bit offset by −128 (tagged
    ``_qzero = 128``: x = (q + 128)·scale, with the 0x80 padding tail), doubling the resolution of
    the signed code."""
    if not (x.is_cuda and x.dtype in (_f32, _bf16) and x.numel() % 16 == 0 and _al16(x)):
        return NotImplemented
    cl = x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last)
    if not (cl or x.is_contiguous()):
        return NotImplemented
    if u8 and not cl:
        return NotImplemented
    xq = _i8_act(*x.shape, x.device, True) if u8 else torch.empty_like(x, dtype=torch.int8)
    check(_lib().bigdl_quant_static2(ptr(x), C.c_int(0 if x.dtype == _f32 else 1), _ll(x.numel()), C.c_float(scale),
                                     ptr(xq), C.c_int(1 if u8 else 0), _s()), "quant_static")
    return _tag(xq, scale, u8)


def maxpool_i8(x, kh, kw, sh, sw, ph, pw, P, Q):
    """Max pooling of an int8 NHWC activation (the scale carries over: max commutes with the
    monotone quantisation).  Returns the pooled int8 tensor tagged with the input's ``_qscale``."""
    if not (x.is_cuda and x.dtype == torch.int8 and x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last)
            and x.shape[1] % 16 == 0 and _al16(x)):
        return NotImplemented
    N_, C_, H, W = x.shape
    u8 = bool(getattr(x, "_qzero", 0))  # the offset code is monotone too
    y = _i8_act(N_, C_, P, Q, x.device, u8)
    check(_lib().bigdl_maxpool_i8_t(ptr(x), ptr(y), N_, H, W, C_, P, Q, kh, kw, sh, sw, ph, pw, C.c_int(int(u8)), _s()),
          "maxpool_i8")
    return _tag(y, getattr(x, "_qscale", None), u8)


def conv_i8_u8_bias(wq, ldw, K, R, S, C_, sx, w_scale, bias):
    """The bias of the int8 conv for an unsigned (offset −128) input of scale ``sx``: the offset's
    share of the dot product, 128·Σ_(taps, c) w · sx · sw, is a per-channel constant (padded taps
    read the code of 0 from the input's tail) folded in here."""
    w = wq.view(torch.int8).reshape(K, ldw).to(torch.int32).sum(-1).double()  # (padding entries are 0)
    b = bias.double() if bias is not None else torch.zeros(K, dtype=torch.float64, device=wq.device)
    return (b + 128.0 * w * float(sx) * w_scale.double()).float().contiguous()


def conv2d_i8_forward_static(x, wq, ldw, w_scale, bias, K, R, S, stride, pad, dilation, out_hw, relu=False,
                             in_scale=None, out_scale=None, in_u8=False, out_u8=False, u8_bias=None, residual=None,
                             out=None):
    """int8 conv with calibrated scales: ``x`` int8 NHWC (tagged ``_qscale``, the producer's
    requantised output) or fp32/bf16 quantised here with ``in_scale`` in one static pass; with
    ``out_scale`` the epilogue writes the int8 NHWC input of the next quantised layer (bias, ReLU
    and requantisation fused), else bf16.  ``in_u8`` (fp32/bf16 input known non-negative) / an int8
    input tagged ``_qzero``: offset −128 u8 input (its bias ``u8_bias``, :func:`conv_i8_u8_bias`);
    ``out_u8``: write the (ReLU'd) output that way.  ``residual`` (NHWC [N][K][P][Q], int8 tagged
    ``_qscale`` / ``_qzero`` or bf16): summed before the ReLU in the epilogue — the conv + sum of a
    residual block tail.  NotImplemented when the kernel does not apply."""
    if not (x.is_cuda and x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last) and _al16(x)):
        return NotImplemented
    N_, C_, H, W = x.shape
    if not conv_i8_supported(C_, R, S) or K % 8 or (out_scale is not None and K % 16):
        return NotImplemented
    if x.dtype == torch.int8:
        sx = getattr(x, "_qscale", None)
        if sx is None:
            return NotImplemented
        xq = x
    else:
        if in_scale is None:
            return NotImplemented
        xq = quant_static(x, in_scale, u8=in_u8)
        if xq is NotImplemented:
            return NotImplemented
        sx = in_scale
    x_u8 = bool(getattr(xq, "_qzero", 0))
    if x_u8 and not getattr(xq, "_qtail", False):
        return NotImplemented  # no padding tail to point the padded taps at
    if out_u8 and not (relu and out_scale is not None):
        raise ValueError("conv2d_i8_forward_static: out_u8 needs a fused ReLU and an int8 output")
    P, Q = out_hw
    ldy = K
    if out is not None and out_scale is not None:
        # a channel slice [N][K][P][Q] of a wider channels-last int8 tensor (zero-copy concat)
        if not (out.dtype == torch.int8 and tuple(out.shape) == (N_, K, P, Q) and out.stride(1) == 1
                and out.stride(2) == Q * out.stride(3) and out.stride(0) == P * Q * out.stride(3)
                and out.stride(3) % 16 == 0 and out.data_ptr() % 16 == 0):
            return NotImplemented
        y, ldy = out, out.stride(3)
    elif out_scale is not None:
        y = _i8_act(N_, K, P, Q, x.device, out_u8)
    else:
        y = torch.empty((N_, K, P, Q), dtype=_bf16, device=x.device, memory_format=torch.channels_last)
    rkind, rscale, rzero = 0, 1.0, 0.0
    if residual is not None:
        if (residual.dim() != 4 or tuple(residual.shape) != (N_, K, P, Q) or not residual.is_cuda
                or not residual.is_contiguous(memory_format=torch.channels_last) or residual.data_ptr() % 8):
            return NotImplemented
        if residual.dtype == torch.int8 and getattr(residual, "_qscale", None) is not None:
            rkind, rscale, rzero = 1, float(residual._qscale), float(getattr(residual, "_qzero", 0))
        elif residual.dtype == _bf16:
            rkind = 2
        else:
            return NotImplemented
    b = bias.float().contiguous() if bias is not None else None
    if x_u8:
        b = u8_bias if u8_bias is not None else conv_i8_u8_bias(wq, ldw, K, R, S, C_, sx, w_scale, bias)
    check(_lib().bigdl_conv_i8_fwd4(ptr(xq), ptr(wq), C.c_int(ldw), None, C.c_float(sx), ptr(w_scale), ptr(b),
                                    None if out_scale is not None else ptr(y), ptr(y) if out_scale is not None else None,
                                    C.c_float(out_scale if out_scale is not None else 1.0), C.c_int(ldy), N_, H, W, C_, K,
                                    R, S, P, Q, stride[0], stride[1], pad[0], pad[1], dilation[0], dilation[1],
                                    C.c_int(1 if relu else 0), C.c_int(int(x_u8)),
                                    C.c_int(int(out_u8)), ptr(residual), C.c_int(rkind), C.c_int(K), C.c_float(rscale),
                                    C.c_float(rzero), _s()), "conv_i8_fwd4")
    if out_scale is not None:
        _tag(y, out_scale, out_u8)
    return y


@register("gemm_i8")
def gemm_i8(qa, sa, qb, sb, bias=None, out_dtype=torch.float32, relu=False):
    if qa.dtype != torch.int8 or qb.dtype != torch.int8 or qa.shape[1] != qb.shape[1] or qa.shape[1] % 16:
        return NotImplemented
    if not (qa.is_contiguous() and qb.is_contiguous() and _al16(qa) and _al16(qb)):
        return NotImplemented
    if out_dtype not in (_f32, _bf16):
        return NotImplemented
    M, Kp = qa.shape
    N = qb.shape[0]
    sa = sa.float().contiguous()
    sb = sb.float().contiguous()
    b = bias.float().contiguous() if bias is not None else None
    out = torch.empty((M, N), dtype=out_dtype, device=qa.device)
    check(_lib().bigdl_gemm_i8(ptr(qa), ptr(qb), C.c_int(M), C.c_int(N), C.c_int(Kp), ptr(sa), ptr(sb), ptr(b),
                               ptr(out), C.c_int(1 if out_dtype == _bf16 else 0), C.c_int(1 if relu else 0), _s()),
          "gemm_i8")
    return out


def _i8_splits(M, N, Kp):
    """Split-K factor of an int8 GEMM: whole-K 128×128 tiles fill ≥ 2 waves of the 256 CUs already,
    else split the reduction (≥ 4 k-tiles per split) until they do."""
    tiles = -(-M // 128) * -(-N // 128)
    kt = -(-Kp // 128)
    if tiles >= 512 or kt < 8:
        return 1
    return max(1, min(kt // 4, -(-512 // tiles)))


def gemm_i8_static(qa, sa0, qb, sb, bias=None, out_dtype=torch.bfloat16, relu=False, out_scale=None, out_u8=False):
    """int8 GEMM of a statically quantised activation ``qa`` [M][Kp] (one scale ``sa0``) with per-row
    int8 weights ``qb`` [N][Kp] (scales ``sb``): bias, ReLU, then ``out_dtype`` or — ``out_scale`` — the
    next quantised layer's int8 input (tagged; ``out_u8``: the offset unsigned code of a ReLU'd
    output).  Split-K for small-M, long-K products (classifier heads)."""
    if qa.dtype != torch.int8 or qb.dtype != torch.int8 or qa.dim() != 2 or qa.shape[1] != qb.shape[1] \
            or qa.shape[1] % 16 or not (sa0 and sa0 > 0):
        return NotImplemented
    if not (qa.is_contiguous() and qb.is_contiguous() and _al16(qa) and _al16(qb)) or out_dtype not in (_f32, _bf16):
        return NotImplemented
    M, Kp = qa.shape
    N = qb.shape[0]
    sb = sb.float().contiguous()
    b = bias.float().contiguous() if bias is not None else None
    if out_scale is not None:
        out = torch.empty((M, N), dtype=torch.int8, device=qa.device)
    else:
        out = torch.empty((M, N), dtype=out_dtype, device=qa.device)
    splits = _i8_splits(M, N, Kp)
    work = torch.empty(splits * M * N, dtype=torch.int32, device=qa.device) if splits > 1 else None
    check(_lib().bigdl_gemm_i8_ex(ptr(qa), ptr(qb), C.c_int(M), C.c_int(N), C.c_int(Kp), None, C.c_float(sa0), ptr(sb),
                                  ptr(b), ptr(out), C.c_int(1 if out_dtype == _bf16 else 0), C.c_int(1 if relu else 0),
                                  C.c_float(out_scale if out_scale is not None else 0.0),
                                  C.c_int(1 if (out_scale is not None and out_u8) else 0), C.c_int(splits), ptr(work),
                                  _s()), "gemm_i8_ex")
    if out_scale is not None:
        _tag(out, out_scale, out_u8)
        out._qtail = False
    return out


# ------------------------------------------------------------------------------------------------ image (K25)
@register("image_crop_flip_norm")
def image_crop_flip_norm(src, oy, ox, flip, out_h, out_w, mean, std, to_rgb, out_dtype=torch.float32):
    if src.dim() != 4 or src.dtype not in (torch.uint8, _f32) or not src.is_contiguous():
        return NotImplemented
    if out_dtype not in (_f32, _bf16):
        return NotImplemented
    B, H, W, Cc = src.shape
    if Cc > 4:
        return NotImplemented
    oy_c, ox_c, fl_c = (torch.as_tensor(v).reshape(-1).cpu().int() for v in (oy, ox, flip))
    if len(oy_c) != B or len(ox_c) != B or len(fl_c) != B:
        return NotImplemented
    if int(oy_c.max()) + out_h > H or int(ox_c.max()) + out_w > W or int(oy_c.min()) < 0 or int(ox_c.min()) < 0:
        raise ValueError("crop window outside the image")
    dev = src.device
    oy_d, ox_d, fl_d = (t.to(dev, non_blocking=True) for t in (oy_c, ox_c, fl_c))
    mean_f = (C.c_float * 4)(*[float(v) for v in list(mean)[:Cc]])
    std_f = (C.c_float * 4)(*[float(v) for v in list(std)[:Cc]])
    out = torch.empty((B, Cc, out_h, out_w), dtype=out_dtype, device=dev, memory_format=torch.channels_last)
    check(_lib().bigdl_image_crop_flip_norm(ptr(src), C.c_int(1 if src.dtype == torch.uint8 else 0), C.c_int(B),
                                            C.c_int(H), C.c_int(W), C.c_int(Cc), ptr(oy_d), ptr(ox_d), ptr(fl_d),
                                            C.c_int(out_h), C.c_int(out_w), mean_f, std_f,
                                            C.c_int(1 if to_rgb else 0), ptr(out),
                                            C.c_int(1 if out_dtype == _bf16 else 0), _s()), "image_crop_flip_norm")
    return out


# ------------------------------------------------------------------------------------------------ pooling (K10)
def _pool_out(size, k, s, p, ceil_mode):
    if ceil_mode:
        o = -(-(size + 2 * p - k) // s) + 1
        if (o - 1) * s >= size + p:
            o -= 1
    else:
        o = (size + 2 * p - k) // s + 1
    return o


class _Int8Idx:
    """argmax offsets from the native max-pool forward (int8, NHWC) — only the native backward reads it."""
    __slots__ = ("t",)

    def __init__(self, t):
        self.t = t


@register("maxpool2d_forward")
def maxpool2d_forward(x, k, s, p, ceil_mode, need_indices=True):
    """``need_indices=False`` (inference) skips the int8 argmax: 1/3 less traffic.  fp32 NHWC
    (bigdl.compute.dtype=fp32) runs the fp32 instantiation of the same kernel (per-element kernels when
    C % 8 != 0, e.g. LeNet's 6 / 12 maps)."""
    if (x.dim() == 4 and x.dtype == _f32 and x.is_contiguous(memory_format=torch.channels_last)
            and k[0] * k[1] <= 127 and p[0] * 2 <= k[0] and p[1] * 2 <= k[1]):
        N_, C_, H, W = x.shape
        P = _pool_out(H, k[0], s[0], p[0], ceil_mode)
        Q = _pool_out(W, k[1], s[1], p[1], ceil_mode)
        if P > 0 and Q > 0:
            y = torch.empty((N_, C_, P, Q), dtype=_f32, device=x.device, memory_format=torch.channels_last)
            idx = torch.empty((N_, P, Q, C_), dtype=torch.int8, device=x.device) if need_indices else None
            check(_lib().bigdl_maxpool32_fwd(ptr(x), ptr(y), ptr(idx), N_, H, W, C_, P, Q, k[0], k[1], s[0], s[1],
                                             p[0], p[1], _s()), "maxpool32_fwd")
            return y, (_Int8Idx(idx) if need_indices else None)
    if x.dim() != 4 or x.dtype != _bf16 or not x.is_contiguous(memory_format=torch.channels_last) or not _al16(x):
        return NotImplemented
    N_, C_, H, W = x.shape
    if k[0] * k[1] > 127 or p[0] * 2 > k[0] or p[1] * 2 > k[1] or (C_ % 8 and not x.is_contiguous(
            memory_format=torch.channels_last)):
        return NotImplemented
    P = _pool_out(H, k[0], s[0], p[0], ceil_mode)
    Q = _pool_out(W, k[1], s[1], p[1], ceil_mode)
    y = torch.empty((N_, C_, P, Q), dtype=_bf16, device=x.device, memory_format=torch.channels_last)
    idx = torch.empty((N_, P, Q, C_), dtype=torch.int8, device=x.device) if need_indices else None
    check(_lib().bigdl_maxpool_fwd(ptr(x), ptr(y), ptr(idx), N_, H, W, C_, P, Q, k[0], k[1], s[0], s[1], p[0], p[1],
                                   _s()), "maxpool_fwd")
    return y, (_Int8Idx(idx) if need_indices else None)


@register("maxpool2d_backward")
def maxpool2d_backward(gy, x, idx, k, s, p, ceil_mode):
    if not isinstance(idx, _Int8Idx):
        return NotImplemented
    N_, C_, H, W = x.shape
    P, Q = gy.shape[2], gy.shape[3]
    if x.dtype == _f32:
        gy = gy.float().contiguous(memory_format=torch.channels_last)
        gx = torch.empty((N_, C_, H, W), dtype=_f32, device=x.device, memory_format=torch.channels_last)
        check(_lib().bigdl_maxpool32_bwd(ptr(gy), ptr(idx.t), ptr(gx), N_, H, W, C_, P, Q, k[0], k[1], s[0], s[1],
                                         p[0], p[1], _s()), "maxpool32_bwd")
        return gx
    if gy.dtype != _bf16:
        gy = gy.to(_bf16)
    gy = gy.contiguous(memory_format=torch.channels_last)
    gx = torch.empty((N_, C_, H, W), dtype=_bf16, device=x.device, memory_format=torch.channels_last)
    check(_lib().bigdl_maxpool_bwd(ptr(gy), ptr(idx.t), ptr(gx), N_, H, W, C_, P, Q, k[0], k[1], s[0], s[1], p[0],
                                   p[1], _s()), "maxpool_bwd")
    return gx


# ---------------------------------------------------------------------------------- K18 LRN
def _lrn_ok(x, size):
    return (x.dim() == 4 and x.dtype in (_bf16, _f32) and x.is_contiguous(memory_format=torch.channels_last)
            and _al16(x) and x.shape[1] % 8 == 0 and size % 2 == 1 and x.numel() > 0)


@register("lrn_forward")
def lrn_forward(x, size, alpha, beta, k):
    """bf16 or fp32 NHWC (the fp32 kernel: the reference's precision, DL/nn/SpatialCrossMapLRN.scala:96-200)."""
    if x.dim() == 4 and x.dtype == _f32 and not x.is_contiguous(memory_format=torch.channels_last):
        x = x.contiguous(memory_format=torch.channels_last)
    if not _lrn_ok(x, size) or size > 17:
        return NotImplemented
    y = torch.empty_like(x, memory_format=torch.channels_last)
    n, c, h, w = x.shape
    fn = _lib().bigdl_lrn_fwd_f32 if x.dtype == _f32 else _lib().bigdl_lrn_fwd
    check(fn(ptr(x), ptr(y), _ll(n * h * w), c, size, C.c_float(alpha), C.c_float(beta), C.c_float(k), _s()),
          "lrn_fwd")
    return y


@register("lrn_backward")
def lrn_backward(gy, x, size, alpha, beta, k):
    if x.dim() == 4 and x.dtype == _f32 and not x.is_contiguous(memory_format=torch.channels_last):
        x = x.contiguous(memory_format=torch.channels_last)
    if not _lrn_ok(x, size) or size > 9:
        return NotImplemented
    gy = gy.to(x.dtype).contiguous(memory_format=torch.channels_last)
    if gy.shape != x.shape or not _al16(gy):
        return NotImplemented
    gx = torch.empty_like(x, memory_format=torch.channels_last)
    n, c, h, w = x.shape
    fn = _lib().bigdl_lrn_bwd_f32 if x.dtype == _f32 else _lib().bigdl_lrn_bwd
    check(fn(ptr(x), ptr(gy), ptr(gx), _ll(n * h * w), c, size, C.c_float(alpha), C.c_float(beta), C.c_float(k),
             _s()), "lrn_bwd")
    return gx


# ---------------------------------------------------------------------------------- K17 dropout
class _DropMask:
    """Stands in for the dropout mask: the kernel regenerates the keep decisions from ``seed``
    (or, under HIP-graph capture, from the device-side seed snapshot ``dev``)."""
    __slots__ = ("seed", "cl", "shape", "dev")

    def __init__(self, seed, cl, shape, dev=None):
        self.seed, self.cl, self.shape, self.dev = seed, cl, shape, dev


_DEV_SEED = {}


def _device_seed(device) -> torch.Tensor:
    """Per-device int64 seed counter advanced on the stream (captured into graphs)."""
    t = _DEV_SEED.get(device)
    if t is None:
        t = torch.tensor([int(torch.randint(0, 2 ** 62, (1,)))], dtype=torch.int64, device=device)
        _DEV_SEED[device] = t
    return t


def _dense_layout(t):
    if t.is_contiguous():
        return False
    if t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last):
        return True
    return None


@register("dropout_forward")
def dropout_forward(x, p, generator=None):
    if p <= 0 or p >= 1 or x.dtype not in (_bf16, _f32) or not _al16(x) or x.numel() == 0:
        return NotImplemented
    cl = _dense_layout(x)
    if cl is None:
        return NotImplemented
    y = torch.empty_like(x)
    if torch.cuda.is_current_stream_capturing():
        snap = _device_seed(x.device).clone()
        check(_lib().bigdl_dropout_devseed(ptr(x), ptr(y), _ll(x.numel()), 0 if x.dtype == _bf16 else 1, C.c_float(p),
                                           ptr(snap), _s()), "dropout_fwd")
        _device_seed(x.device).add_(1)
        return y, _DropMask(None, cl, tuple(x.shape), snap)
    seed = int(torch.randint(0, 2 ** 62, (1,), generator=generator if (generator is not None and
                                                                         generator.device.type == "cpu") else None))
    check(_lib().bigdl_dropout(ptr(x), ptr(y), _ll(x.numel()), 0 if x.dtype == _bf16 else 1, C.c_float(p),
                               C.c_ulonglong(seed), _s()), "dropout_fwd")
    return y, _DropMask(seed, cl, tuple(x.shape))


@register("dropout_backward")
def dropout_backward(gy, mask, p):
    if not isinstance(mask, _DropMask):
        return NotImplemented
    if tuple(gy.shape) != mask.shape:
        raise ValueError(f"dropout backward: gradient shape {tuple(gy.shape)} != forward {mask.shape}")
    if gy.dtype not in (_bf16, _f32):
        gy = gy.float()
    gy = gy.contiguous(memory_format=torch.channels_last) if mask.cl else gy.contiguous()
    if not _al16(gy):
        gy = gy.clone()
    gx = torch.empty_like(gy)
    if mask.dev is not None:
        check(_lib().bigdl_dropout_devseed(ptr(gy), ptr(gx), _ll(gy.numel()), 0 if gy.dtype == _bf16 else 1,
                                           C.c_float(p), ptr(mask.dev), _s()), "dropout_bwd")
        return gx
    check(_lib().bigdl_dropout(ptr(gy), ptr(gx), _ll(gy.numel()), 0 if gy.dtype == _bf16 else 1, C.c_float(p),
                               C.c_ulonglong(mask.seed), _s()), "dropout_bwd")
    return gx


# ---------------------------------------------------------------------------------- K4 dense GEMM
def _mat_ok(t, cols=None):
    """2-D bf16 device matrix with unit column stride, 16-B aligned rows (row stride % 8)."""
    return (t is not None and t.dim() == 2 and t.dtype == _bf16 and t.is_cuda and t.stride(1) == 1
            and t.stride(0) % 8 == 0 and t.stride(0) >= t.shape[1] and _al16(t)
            and (cols is None or t.shape[1] == cols))


def _bias_f32(b, n):
    if b is None:
        return None
    if b.dtype != _f32 or not b.is_contiguous() or not _al16(b):
        b = b.float().contiguous()
    return b if b.numel() == n else None


def gemm(a, b, bias=None, act=0, out=None, d=None, alpha=1.0, beta=0.0):
    """C = act(alpha·A·Bᵀ + bias + D) (+ beta·C for an fp32 ``out``) on the MFMA GEMM kernel
    (gemm.hip).  A [M][K], B [N][K] bf16 rows; ``out`` bf16 or fp32 [M][N] (row stride % 4)."""
    if not (_mat_ok(a) and _mat_ok(b)) or a.shape[1] != b.shape[1]:
        return NotImplemented
    M, K = a.shape
    N = b.shape[0]
    if K % 8 or N % 4 or M == 0:
        return NotImplemented
    bb = _bias_f32(bias, N)
    if bias is not None and bb is None:
        return NotImplemented
    if out is None:
        out = torch.empty((M, N), dtype=_bf16, device=a.device)
    if out.dim() != 2 or tuple(out.shape) != (M, N) or out.stride(1) != 1 or out.stride(0) % 4 or \
            out.dtype not in (_bf16, _f32) or out.data_ptr() % (16 if out.dtype == _f32 else 8):
        return NotImplemented
    if d is not None and (d.dtype != _bf16 or d.dim() != 2 or tuple(d.shape) != (M, N) or d.stride(1) != 1
                          or d.stride(0) % 4 or d.data_ptr() % 8):
        return NotImplemented
    S = _gemm_splits(M, N, K)
    slab = torch.empty(S * M * N, dtype=_f32, device=a.device) if S > 1 else None
    check(_lib().bigdl_gemm_splitk(ptr(a), _ll(a.stride(0)), ptr(b), _ll(b.stride(0)), ptr(bb), ptr(d),
                                   _ll(d.stride(0) if d is not None else 0), ptr(out), _ll(out.stride(0)), C.c_int(M),
                                   C.c_int(N), C.c_int(K), C.c_int(act), C.c_int(1 if out.dtype == _f32 else 0),
                                   _f(alpha), _f(beta), ptr(slab), C.c_int(S), _s()), "gemm")
    return out


def _gemm_splits(M, N, K):
    """K slices for gemm(): a GEMM whose 64×64 tile grid cannot fill the chip (under 256 tiles) and
    whose K is long (≥ 2048: a classifier head, batch × 25088 · 4096) splits K so that ~512 blocks
    run, each slice ≥ 8 k-tiles; the fp32 partial slabs are summed by the epilogue kernel."""
    if M * N >= 256 * 128 * 128 or K < 2048:
        return 1
    tiles = ((M + 63) // 64) * ((N + 63) // 64)
    if tiles >= 256:
        return 1
    return max(1, min(16, 512 // tiles, K // 512))


def transpose_bf16(src):
    """[R][C] bf16 (unit column stride) → contiguous [C][R]."""
    R_, C_ = src.shape
    dst = torch.empty((C_, R_), dtype=_bf16, device=src.device)
    check(_lib().bigdl_transpose_bf16(ptr(src), _ll(src.stride(0)), ptr(dst), _ll(R_), C.c_int(R_), C.c_int(C_),
                                      _s()), "transpose")
    return dst


def colsum_acc(x, out, scale=1.0):
    """out[n] += scale · Σ_m x[m][n]  (bias gradient, bf16 or fp32 rows → fp32)."""
    M, N_ = x.shape
    if x.dtype == _f32:
        if not (x.is_cuda and x.stride(1) == 1 and x.stride(0) % 4 == 0 and x.stride(0) >= N_ and _al16(x)
                and N_ % 4 == 0 and out.dtype == _f32 and out.is_contiguous() and out.numel() == N_):
            return NotImplemented
        check(_lib().bigdl_colsum_f32(ptr(x), _ll(x.stride(0)), ptr(out), C.c_int(M), C.c_int(N_), _f(scale), _s()),
              "colsum_f32")
        return out
    if not (_mat_ok(x) and N_ % 8 == 0 and out.dtype == _f32 and out.is_contiguous() and out.numel() == N_):
        return NotImplemented
    check(_lib().bigdl_colsum_bf16(ptr(x), _ll(x.stride(0)), ptr(out), C.c_int(M), C.c_int(N_), _f(scale), _s()),
          "colsum")
    return out


def wgrad_rows(gy, x, gw_acc, scale):
    """gw_acc[N][K] += scale · gyᵀ·x for row-major gy [M][N], x [M][K] (the 1×1 case of the conv
    wgrad kernel: transposed LDS reads, split-K over rows with fp32 atomics)."""
    M, N_ = gy.shape
    K = x.shape[1]
    if not (gy.is_contiguous() and x.is_contiguous() and gy.dtype == _bf16 and x.dtype == _bf16 and _al16(gy)
            and _al16(x) and N_ % 8 == 0 and K % 8 == 0 and gw_acc.dtype == _f32 and gw_acc.is_contiguous()
            and gw_acc.numel() == N_ * K):
        return NotImplemented
    check(_lib().bigdl_conv_wgrad(ptr(x), ptr(gy), ptr(gw_acc), _f(scale), M, 1, 1, K, N_, 1, 1, 1, 1, 1, 1, 0, 0, 1, 1,
                                  -_wgrad_blocks(M, K, N_), _s()), "linear_wgrad")
    return gw_acc


def _r8(n):
    return (n + 7) // 8 * 8


def _padded(t, rows, cols):
    """``t`` as a dense bf16 [rows][cols] matrix, zero-padded (a copy only when needed)."""
    if tuple(t.shape) == (rows, cols) and _mat_ok(t):
        return t
    out = torch.zeros((rows, cols), dtype=_bf16, device=t.device)
    out[:t.shape[0], :t.shape[1]] = t
    return out


@register("linear_forward")
def linear_forward(x, w, b, act=0):
    if x.dtype == _f32 and F3.enabled(x):
        r = F3.linear_forward(x, w, b, act)
        if r is not NotImplemented:
            return r
    if x.dim() != 2 or w.dim() != 2 or x.dtype != _bf16 or w.dtype != _bf16 or x.shape[1] != w.shape[1]:
        return NotImplemented
    M, K = x.shape
    N_ = w.shape[0]
    if M == 0:
        return NotImplemented
    # odd sizes (LeNet's 100 → 10 classifier): zero-pad K to a multiple of 8 and N to 4, slice after
    K8, N4 = _r8(K), (N_ + 3) // 4 * 4
    xp, wp = _padded(x, M, K8), _padded(w, N4, K8)
    bp = b
    if b is not None and N4 != N_:
        bp = torch.zeros(N4, dtype=_f32, device=x.device)
        bp[:N_] = b
    y = gemm(xp, wp, bp, act=act)
    if y is NotImplemented or N4 == N_:
        return y
    return y[:, :N_].contiguous()


@register("linear_backward")
def linear_backward(gy, x, w, need_input=True, gw_acc=None, gb_acc=None, scale=1.0):
    if gy.dtype == _f32 and x.dtype == _f32 and F3.enabled(gy):
        r = F3.linear_backward(gy, x, w, need_input, gw_acc, gb_acc, scale)
        if r is not NotImplemented:
            return r
    if gy.dim() != 2 or x.dim() != 2 or w.dim() != 2 or not (gy.dtype == x.dtype == w.dtype == _bf16):
        return NotImplemented
    M, N_ = gy.shape
    K = x.shape[1]
    if x.shape[0] != M or tuple(w.shape) != (N_, K) or M == 0:
        return NotImplemented
    do_w = gw_acc is not None and scale != 0
    do_b = gb_acc is not None and scale != 0
    if do_w and not (gw_acc.dtype == _f32 and gw_acc.is_contiguous() and gw_acc.numel() == N_ * K):
        return NotImplemented
    if do_b and not (gb_acc.dtype == _f32 and gb_acc.is_contiguous() and gb_acc.numel() == N_):
        return NotImplemented
    N8, K8 = _r8(N_), _r8(K)
    gyp = _padded(gy, M, N8)
    gi = None
    if need_input:
        # gx = gy·W = gy · (Wᵀ)ᵀ: transposed weight copy [K][N] (zero-padded to [K8][N8] if odd)
        wt = transpose_bf16(w) if (N8 == N_ and _mat_ok(w)) else None
        wt = _padded(wt if wt is not None else w.t(), K8, N8)
        gi = gemm(gyp, wt)
        if gi is NotImplemented:
            return NotImplemented
        if K8 != K:
            gi = gi[:, :K].contiguous()
    if do_w:
        # the wgrad kernel reads dense rows: strided views (e.g. a gate slice) are packed first
        if N8 == N_ and K8 == K:
            r = wgrad_rows(gyp.contiguous(), x.contiguous(), gw_acc, scale)
        else:
            tmp = torch.zeros(N8 * K8, dtype=_f32, device=x.device)
            r = wgrad_rows(gyp.contiguous(), _padded(x, M, K8).contiguous(), tmp, scale)
            gw_acc.view(N_, K).add_(tmp.view(N8, K8)[:N_, :K])
        if r is NotImplemented:
            return NotImplemented
    if do_b:
        if N8 == N_:
            colsum_acc(gyp, gb_acc, scale)
        else:
            tmp = torch.zeros(N8, dtype=_f32, device=x.device)
            colsum_acc(gyp, tmp, scale)
            gb_acc.add_(tmp[:N_])
    return gi


# ---------------------------------------------------------------------------------- K12 softmax
def _rowwise(x):
    return x.is_cuda and x.dtype in (_bf16, _f32) and x.dim() >= 1 and x.numel() > 0 and x.is_contiguous()


@register("softmax_forward")
def softmax_forward(x):
    if not _rowwise(x):
        return NotImplemented
    K = x.shape[-1]
    y = torch.empty_like(x)
    check(_lib().bigdl_softmax(ptr(x), ptr(None), ptr(y), _ll(x.numel() // K), C.c_int(K), C.c_int(0),
                               C.c_int(1 if x.dtype == _bf16 else 0), _s()), "softmax")
    return y


@register("softmax_backward")
def softmax_backward(gy, y):
    if not (_rowwise(y) and gy.shape == y.shape):
        return NotImplemented
    if gy.dtype != y.dtype or not gy.is_contiguous():
        gy = gy.to(y.dtype).contiguous()
    K = y.shape[-1]
    gx = torch.empty_like(y)
    check(_lib().bigdl_softmax(ptr(gy), ptr(y), ptr(gx), _ll(y.numel() // K), C.c_int(K), C.c_int(1),
                               C.c_int(1 if y.dtype == _bf16 else 0), _s()), "softmax_bwd")
    return gx


def softmax_channels_nhwc(x, backward_gy=None):
    """Channel-dim softmax (SoftMax on a 4-D batch) on the NHWC device layout: channels are the
    contiguous dim, so it is the row-wise kernel over N·H·W rows."""
    if x.dim() != 4 or not x.is_contiguous(memory_format=torch.channels_last) or x.dtype not in (_bf16, _f32):
        return NotImplemented
    n, c, h, w = x.shape
    rows = x.permute(0, 2, 3, 1).reshape(-1, c)
    if backward_gy is None:
        r = softmax_forward(rows)
    else:
        g = backward_gy.to(x.dtype).contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1).reshape(-1, c)
        r = softmax_backward(g, rows)
    if r is NotImplemented:
        return r
    return r.reshape(n, h, w, c).permute(0, 3, 1, 2)


# ---------------------------------------------------------------------------------- K11 avg-pool
@register("avgpool2d_forward")
def avgpool2d_forward(x, k, s, p, ceil_mode, count_include_pad, divisor=None):
    if (x.dim() != 4 or x.dtype not in (_bf16, _f32) or not x.is_contiguous(memory_format=torch.channels_last)
            or not _al16(x)):
        return NotImplemented
    N_, C_, H, W = x.shape
    if C_ % 8 or p[0] * 2 > k[0] or p[1] * 2 > k[1]:
        return NotImplemented
    P = _pool_out(H, k[0], s[0], p[0], ceil_mode)
    Q = _pool_out(W, k[1], s[1], p[1], ceil_mode)
    if P <= 0 or Q <= 0:
        return NotImplemented
    y = torch.empty((N_, C_, P, Q), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
    fn = _lib().bigdl_avgpool32_fwd if x.dtype == _f32 else _lib().bigdl_avgpool_fwd  # fp32: the reference precision
    check(fn(ptr(x), ptr(y), N_, H, W, C_, P, Q, k[0], k[1], s[0], s[1], p[0], p[1],
                                   int(bool(count_include_pad)), int(divisor or 0), _s()), "avgpool_fwd")
    return y


@register("avgpool2d_backward")
def avgpool2d_backward(gy, x, k, s, p, ceil_mode, count_include_pad, divisor=None):
    if x.dim() != 4 or x.dtype not in (_bf16, _f32) or gy.dim() != 4:
        return NotImplemented
    N_, C_, H, W = x.shape
    if C_ % 8 or p[0] * 2 > k[0] or p[1] * 2 > k[1]:
        return NotImplemented
    P = _pool_out(H, k[0], s[0], p[0], ceil_mode)
    Q = _pool_out(W, k[1], s[1], p[1], ceil_mode)
    if tuple(gy.shape) != (N_, C_, P, Q):
        return NotImplemented
    gy = gy.to(x.dtype).contiguous(memory_format=torch.channels_last)
    if not _al16(gy):
        gy = gy.clone(memory_format=torch.channels_last)
    gx = torch.empty((N_, C_, H, W), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
    fn = _lib().bigdl_avgpool32_bwd if x.dtype == _f32 else _lib().bigdl_avgpool_bwd
    check(fn(ptr(gy), ptr(gx), N_, H, W, C_, P, Q, k[0], k[1], s[0], s[1], p[0], p[1],
                                   int(bool(count_include_pad)), int(divisor or 0), _s()), "avgpool_bwd")
    return gx


# ---------------------------------------------------------------------------------- K16 embedding
_ITYPE = {_f32: 0, torch.int64: 1, torch.int32: 2}


# Out-of-range ids (the reference requires 1 <= id <= nIndex, LookupTable.scala:96-98,227-229):
# the forward kernel ORs a per-device error flag; after each launch the flag is copied to pinned
# host memory behind an event, and the NEXT embedding call (or embedding_check) raises once that
# copy has landed — no host/device synchronisation on the hot path.  bigdl.embedding.syncCheck
# checks synchronously after every launch (debugging).
_EMB = {}


def _emb_state(dev):
    st = _EMB.get(dev)
    if st is None:
        st = _EMB[dev] = {"flag": torch.zeros(1, dtype=torch.int32, device=dev),
                          "host": torch.zeros(1, dtype=torch.int32, pin_memory=True), "event": None, "n_index": 0}
    return st


def embedding_check(dev=None, sync: bool = False) -> None:
    """Raise if an embedding lookup since the last check saw an id outside [1, nIndex]."""
    for d, st in list(_EMB.items()):
        if dev is not None and d != dev:
            continue
        ev = st["event"]
        if ev is None:
            continue
        if sync:
            ev.synchronize()
        elif not ev.query():
            continue
        st["event"] = None
        if int(st["host"][0]) != 0:
            st["flag"].zero_()
            st["host"].zero_()
            raise IndexError(f"LookupTable: an input id is outside [1, {st['n_index']}] "
                             "(elements of input should be >= 1 and <= nIndex)")


@register("embedding_forward")
def embedding_forward(weight, idx_1b, padding_value=0, mask_zero=False):
    """Gather rows ``weight[id - 1]``; ids must lie in [1, nIndex] (``mask_zero``: the padding id is
    also accepted — the layer zeroes its rows)."""
    if weight.dim() != 2 or weight.dtype not in (_bf16, _f32) or not weight.is_contiguous() or not _al16(weight):
        return NotImplemented
    if not idx_1b.is_cuda or idx_1b.dtype not in _ITYPE or idx_1b.numel() == 0:
        return NotImplemented
    idx = idx_1b if idx_1b.is_contiguous() else idx_1b.contiguous()
    n = idx.numel()
    D = weight.shape[1]
    capturing = torch.cuda.is_current_stream_capturing()
    st = _emb_state(weight.device)
    if not capturing:
        embedding_check(weight.device)
    out = torch.empty((*idx_1b.shape, D), dtype=weight.dtype, device=weight.device)
    check(_lib().bigdl_embedding_fwd(ptr(weight), ptr(idx), C.c_int(_ITYPE[idx.dtype]), ptr(out), _ll(n),
                                     _ll(weight.shape[0]), C.c_int(D), C.c_int(0 if weight.dtype == _bf16 else 1),
                                     ptr(st["flag"]), C.c_int(1 if mask_zero else 0), _f(padding_value), _s()),
          "embedding_fwd")
    st["n_index"] = int(weight.shape[0])
    if not capturing and st["event"] is None:
        st["host"].copy_(st["flag"], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        st["event"] = ev
        if config.get_property("bigdl.embedding.syncCheck"):
            embedding_check(weight.device, sync=True)
    return out


@register("embedding_backward")
def embedding_backward(grad_weight, idx_1b, gy, scale=1.0, padding_value=0):
    if grad_weight.dtype != _f32 or not grad_weight.is_contiguous() or grad_weight.dim() != 2:
        return NotImplemented
    if not idx_1b.is_cuda or idx_1b.dtype not in _ITYPE:
        return NotImplemented
    D = grad_weight.shape[1]
    n = idx_1b.numel()
    if gy.numel() != n * D or gy.dtype not in (_bf16, _f32):
        return NotImplemented
    if scale == 0 or n == 0:
        return grad_weight
    idx = idx_1b.contiguous()
    g = gy.contiguous()
    check(_lib().bigdl_embedding_bwd(ptr(grad_weight), ptr(idx), C.c_int(_ITYPE[idx.dtype]), ptr(g), _ll(n),
                                     _ll(grad_weight.shape[0]), C.c_int(D), C.c_int(0 if g.dtype == _bf16 else 1),
                                     _f(scale), C.c_int(1 if padding_value != 0 else 0), _f(padding_value), _s()),
          "embedding_bwd")
    return grad_weight


# ---------------------------------------------------------------------------------- K14/K15 fused recurrent step
_RNN_CELLS = {"lstm_fwd": 0, "lstm_bwd": 1, "gru_fwd1": 2, "gru_fwd2": 3, "gru_bwd1": 4, "gru_bwd2": 5}


def _ld(t):
    return 0 if t is None else t.stride(0)


def rnn_step(cell, a, u, M, K, Hs, xg=None, hprev=None, c_prev=None, h_out=None, c_out=None, act=None, tc=None,
             gy=None, gc_next=None, dg=None, dc_prev=None, s0=None, s1=None, s2=None, rh=None):
    """One fused recurrent step (rnn_step.hip).  Row operands are 2-D views (unit column stride);
    fp32 state tensors are contiguous [M][Hs] (act [M][4Hs]).  The launcher re-validates every
    alignment / stride the kernel assumes and returns an error instead of launching."""
    x_f32 = 1 if (xg is not None and xg.dtype == _f32) else 0
    check(_lib().bigdl_rnn_step(C.c_int(_RNN_CELLS[cell]), ptr(a), _ll(_ld(a)), ptr(u), C.c_int(M), C.c_int(K),
                                C.c_int(Hs), ptr(xg), _ll(_ld(xg)), C.c_int(x_f32), ptr(hprev), _ll(_ld(hprev)),
                                ptr(c_prev), ptr(h_out), _ll(_ld(h_out)), ptr(c_out), ptr(act), ptr(tc), ptr(gy),
                                _ll(_ld(gy)), ptr(gc_next), ptr(dg), _ll(_ld(dg)), ptr(dc_prev), ptr(s0), ptr(s1),
                                ptr(s2), ptr(rh), _ll(_ld(rh)), _s()), f"rnn_step[{cell}]")


def _dense_bf16(*ts):
    return all(t is None or (t.is_cuda and t.is_contiguous() and _al16(t)) for t in ts)


_RNN_SYNC = {}


def _rnn_sync(device):
    """Two int32 words (arrival counter, error flag) for the resident-weight LSTM kernels' grid
    barrier, from a per-device ring of 32 slots (each launch zeroes its slot on the stream first)."""
    ent = _RNN_SYNC.get(device)
    if ent is None:
        ent = _RNN_SYNC[device] = [torch.zeros(64, dtype=torch.int32, device=device), 0]
    buf, i = ent
    ent[1] = (i + 1) % 32
    return buf[2 * i:2 * i + 2]


_RNN_XG = {}


def _rnn_xg(device):
    """Granule exchange slots of the resident-weight LSTM kernels' barrier-free hand-off
    (BIGDL_RNN_PERSIST=4/5): [2][B ≤ 32][2H ≤ 512] 8-byte granules, one per device (launches on a
    stream are ordered; each zeroes the part it uses first)."""
    buf = _RNN_XG.get(device)
    if buf is None:
        buf = _RNN_XG[device] = torch.zeros(2 * 32 * 512, dtype=torch.int64, device=device)
    return buf


def rnn_sync_errors(device) -> int:
    """Error words raised by the resident-weight LSTM kernels (a tile that gave up waiting) since
    the ring was created: 0 when every hand-off completed (host sync)."""
    ent = _RNN_SYNC.get(torch.device(device))
    return 0 if ent is None else int(ent[0][1::2].ne(0).sum())


def lstm_seq_forward(x2, h0, c0, U, out, cs, acts, tcs, cbuf):
    """Whole-sequence fused LSTM forward (bigdl_lstm_seq_fwd): x2 [B][T][4H], out [B][T][H]; training
    saves cs / tcs [T][B][H], acts [T][B][4H] (fp32), inference ping-pongs c through cbuf [2][B][H]."""
    B, T, G = x2.shape
    H = G // 4
    assert _dense_bf16(x2, h0, c0, U, out, cs, acts, tcs, cbuf) and tuple(out.shape) == (B, T, H), "lstm_seq_forward"
    check(_lib().bigdl_lstm_seq_fwd(ptr(x2), C.c_int(1 if x2.dtype == _f32 else 0), ptr(h0), ptr(c0), ptr(U), ptr(out),
                                    ptr(cs), ptr(acts), ptr(tcs), ptr(cbuf), C.c_int(B), C.c_int(T), C.c_int(H),
                                    ptr(_rnn_sync(x2.device)), ptr(_rnn_xg(x2.device)), _s()), "lstm_seq_fwd")


def lstm_seq_backward(gy, Ut, acts, tcs, cs, c0, DG, gc):
    B, T, H = gy.shape
    assert _dense_bf16(gy, Ut, acts, tcs, cs, c0, DG, gc), "lstm_seq_backward"
    check(_lib().bigdl_lstm_seq_bwd(ptr(gy), ptr(Ut), ptr(acts), ptr(tcs), ptr(cs), ptr(c0), ptr(DG), ptr(gc),
                                    C.c_int(B), C.c_int(T), C.c_int(H), ptr(_rnn_sync(gy.device)),
                                    ptr(_rnn_xg(gy.device)), _s()),
          "lstm_seq_bwd")


def lstm2_seq_forward(x2, h00, c00, U0, out0, cs0, acts0, tcs0, cbuf0, b1, W1, h01, c01, U1, out1, cs1, acts1,
                      tcs1, cbuf1):
    """Two stacked LSTM layers on the layer wavefront (bigdl_lstm2_seq_fwd): layer 1's input
    projection h0·W1ᵀ + b1 is a second reduction segment of its recurrent step, so the pair runs in
    T + 1 launches.  Layouts as :func:`lstm_seq_forward`; W1 [4H1][H0] bf16, b1 fp32 [4H1]."""
    B, T, G0 = x2.shape
    H0, H1 = G0 // 4, U1.shape[1]
    assert _dense_bf16(x2, h00, c00, U0, out0, cs0, acts0, tcs0, cbuf0, b1, W1, h01, c01, U1, out1, cs1, acts1, tcs1,
                       cbuf1) and tuple(out1.shape) == (B, T, H1) and tuple(W1.shape) == (4 * H1, H0), "lstm2_seq_forward"
    check(_lib().bigdl_lstm2_seq_fwd(ptr(x2), C.c_int(1 if x2.dtype == _f32 else 0), ptr(h00), ptr(c00), ptr(U0),
                                     ptr(out0), ptr(cs0), ptr(acts0), ptr(tcs0), ptr(cbuf0), ptr(b1), ptr(W1), ptr(h01),
                                     ptr(c01), ptr(U1), ptr(out1), ptr(cs1), ptr(acts1), ptr(tcs1), ptr(cbuf1),
                                     C.c_int(B), C.c_int(T), C.c_int(H0), C.c_int(H1), _s()), "lstm2_seq_fwd")


def lstm2_seq_backward(gy1, U1t, acts1, tcs1, cs1, c01, DG1, gc1, U0t, W1t, acts0, tcs0, cs0, c00, DG0, gc0):
    """Backward twin of :func:`lstm2_seq_forward` (bigdl_lstm2_seq_bwd): DG1 / DG0 [B][T][4H] gate
    gradients of both layers; layer 0's dh = dg0·U0 + dg1·W1 inside its step (W1ᵀ [H0][4H1])."""
    B, T, H1 = gy1.shape
    H0 = U0t.shape[0]
    assert _dense_bf16(gy1, U1t, acts1, tcs1, cs1, c01, DG1, gc1, U0t, W1t, acts0, tcs0, cs0, c00, DG0, gc0) \
        and tuple(W1t.shape) == (H0, 4 * H1), "lstm2_seq_backward"
    check(_lib().bigdl_lstm2_seq_bwd(ptr(gy1), ptr(U1t), ptr(acts1), ptr(tcs1), ptr(cs1), ptr(c01), ptr(DG1), ptr(gc1),
                                     ptr(U0t), ptr(W1t), ptr(acts0), ptr(tcs0), ptr(cs0), ptr(c00), ptr(DG0), ptr(gc0),
                                     C.c_int(B), C.c_int(T), C.c_int(H0), C.c_int(H1), _s()), "lstm2_seq_bwd")


def gru_seq_forward(x2, h0, Urz, Uh, out, R, Z, Nn, RH, train):
    B, T, G = x2.shape
    H = G // 3
    assert _dense_bf16(x2, h0, Urz, Uh, out, R, Z, Nn, RH), "gru_seq_forward"
    check(_lib().bigdl_gru_seq_fwd(ptr(x2), C.c_int(1 if x2.dtype == _f32 else 0), ptr(h0), ptr(Urz), ptr(Uh), ptr(out),
                                   ptr(R), ptr(Z), ptr(Nn), ptr(RH), C.c_int(1 if train else 0), C.c_int(B), C.c_int(T),
                                   C.c_int(H), _s()), "gru_seq_fwd")


def gru_seq_backward(gy, Urz_t, Uh_t, R, Z, Nn, out, h0, DG, carry):
    B, T, H = gy.shape
    assert _dense_bf16(gy, Urz_t, Uh_t, R, Z, Nn, out, h0, DG, carry), "gru_seq_backward"
    check(_lib().bigdl_gru_seq_bwd(ptr(gy), ptr(Urz_t), ptr(Uh_t), ptr(R), ptr(Z), ptr(Nn), ptr(out), ptr(h0), ptr(DG),
                                   ptr(carry), C.c_int(B), C.c_int(T), C.c_int(H), _s()), "gru_seq_bwd")


def rnn_fast32_ok(H, *ts):
    """The fp32 recurrence (bf16x3 rnn_step variant) covers dense fp32 device rows with H % 8 == 0."""
    if H % 8 or not N.has("lstm_cell_forward") or not hasattr(_lib(), "bigdl_lstm_seq_fwd32"):
        return False
    return all(t is None or (t.is_cuda and t.dtype == _f32) for t in ts)


def lstm_seq_forward32(x2, h0, c0, U, out, cs, acts, tcs, cbuf):
    """All-fp32 fused LSTM forward (bigdl_lstm_seq_fwd32: bf16x3 recurrent products on MFMA)."""
    B, T, G = x2.shape
    H = G // 4
    assert _dense_bf16(x2, h0, c0, U, out, cs, acts, tcs, cbuf) and x2.dtype == _f32, "lstm_seq_forward32"
    check(_lib().bigdl_lstm_seq_fwd32(ptr(x2), ptr(h0), ptr(c0), ptr(U), ptr(out), ptr(cs), ptr(acts), ptr(tcs),
                                      ptr(cbuf), C.c_int(B), C.c_int(T), C.c_int(H), _s()), "lstm_seq_fwd32")


def lstm_seq_backward32(gy, Ut, acts, tcs, cs, c0, DG, gc):
    B, T, H = gy.shape
    assert _dense_bf16(gy, Ut, acts, tcs, cs, c0, DG, gc) and gy.dtype == _f32, "lstm_seq_backward32"
    check(_lib().bigdl_lstm_seq_bwd32(ptr(gy), ptr(Ut), ptr(acts), ptr(tcs), ptr(cs), ptr(c0), ptr(DG), ptr(gc),
                                      C.c_int(B), C.c_int(T), C.c_int(H), _s()), "lstm_seq_bwd32")


def gru_seq_forward32(x2, h0, Urz, Uh, out, R, Z, Nn, RH, train):
    B, T, G = x2.shape
    H = G // 3
    assert _dense_bf16(x2, h0, Urz, Uh, out, R, Z, Nn, RH) and x2.dtype == _f32, "gru_seq_forward32"
    check(_lib().bigdl_gru_seq_fwd32(ptr(x2), ptr(h0), ptr(Urz), ptr(Uh), ptr(out), ptr(R), ptr(Z), ptr(Nn), ptr(RH),
                                     C.c_int(1 if train else 0), C.c_int(B), C.c_int(T), C.c_int(H), _s()),
          "gru_seq_fwd32")


def gru_seq_backward32(gy, Urz_t, Uh_t, R, Z, Nn, out, h0, DG, carry):
    B, T, H = gy.shape
    assert _dense_bf16(gy, Urz_t, Uh_t, R, Z, Nn, out, h0, DG, carry) and gy.dtype == _f32, "gru_seq_backward32"
    check(_lib().bigdl_gru_seq_bwd32(ptr(gy), ptr(Urz_t), ptr(Uh_t), ptr(R), ptr(Z), ptr(Nn), ptr(out), ptr(h0), ptr(DG),
                                     ptr(carry), C.c_int(B), C.c_int(T), C.c_int(H), _s()), "gru_seq_bwd32")


def rnn_fast_ok(H, *ts):
    """The fused step covers bf16 rows with H % 8 == 0 on a device with the library loaded."""
    if H % 8 or not N.has("lstm_cell_forward"):
        return False
    return all(t is None or (t.is_cuda and t.dtype == _bf16) for t in ts)


# ---------------------------------------------------------------------------------- K13 ClassNLL
def _nll_args(logp, target_1b, weights):
    lp = logp.unsqueeze(0) if logp.dim() == 1 else logp
    if lp.dim() != 2 or lp.dtype not in (_bf16, _f32) or not lp.is_contiguous():
        return None
    B, K = lp.shape
    t = _targets_i32(target_1b.to(lp.device), B)
    if t is None:
        return None
    w = None
    if weights is not None:
        w = weights.to(lp.device, _f32).contiguous()
        if w.numel() != K:
            return None
    return lp, t, w, B, K


@register("class_nll_forward")
def class_nll_forward(logp, target_1b, weights=None, size_average=True, padding_value=-1):
    a = _nll_args(logp, target_1b, weights)
    if a is None:
        return NotImplemented
    lp, t, w, B, K = a
    out = torch.empty(2, dtype=_f32, device=lp.device)
    check(_lib().bigdl_class_nll(ptr(lp), ptr(t), ptr(w), ptr(None), _ll(B), C.c_int(K), C.c_int(int(padding_value)),
                                 C.c_int(1 if size_average else 0), C.c_int(1 if lp.dtype == _bf16 else 0), ptr(out),
                                 _s()), "class_nll")
    return out[0]


@register("class_nll_backward")
def class_nll_backward(logp, target_1b, weights=None, size_average=True, padding_value=-1):
    a = _nll_args(logp, target_1b, weights)
    if a is None:
        return NotImplemented
    lp, t, w, B, K = a
    out = torch.empty(2, dtype=_f32, device=lp.device)
    gx = torch.empty_like(lp)
    check(_lib().bigdl_class_nll(ptr(lp), ptr(t), ptr(w), ptr(gx), _ll(B), C.c_int(K), C.c_int(int(padding_value)),
                                 C.c_int(1 if size_average else 0), C.c_int(1 if lp.dtype == _bf16 else 0), ptr(out),
                                 _s()), "class_nll_bwd")
    return gx.squeeze(0) if logp.dim() == 1 else gx


# ------------------------------------------------------------------------------------------------ sparse
@register("spmm")
def spmm(a, b, alpha=1.0):
    """fp32 ``alpha · a @ b`` for a sparse COO ``a`` [M, K] and a dense ``b`` [K, N] (fp32 or bf16)
    on the device: CSR SpMM kernel (sparse.hip), one wave per output row, no atomics."""
    if not (a.is_sparse and a.is_cuda and b.is_cuda and a.dim() == 2 and b.dim() == 2):
        return NotImplemented
    M, K = a.shape
    N = b.shape[1]
    if b.shape[0] != K or N % 4 or b.dtype not in (_f32, _bf16):
        return NotImplemented
    a = a.coalesce()  # row-major sorted (row, col) → CSR order
    b = b.contiguous()
    idx = a.indices()
    nnz = idx.shape[1]
    it = torch.int32 if nnz < 2 ** 31 - 1 else torch.int64
    rowptr = torch.zeros(M + 1, dtype=it, device=b.device)
    if nnz:
        rowptr[1:] = torch.bincount(idx[0], minlength=M).cumsum(0).to(it)
    col = idx[1].to(it).contiguous()
    val = a.values().float().contiguous()
    out = torch.empty((M, N), dtype=_f32, device=b.device)
    check(_lib().bigdl_spmm_csr(ptr(rowptr), ptr(col), ptr(val), C.c_int(0 if it == torch.int32 else 1), ptr(b),
                                C.c_int(0 if b.dtype == _f32 else 1), ptr(out), C.c_int(M), C.c_int(N),
                                _ll(b.stride(0)), _ll(out.stride(0)), _f(alpha), _f(0.0), _s()), "spmm_csr")
    return out


# ------------------------------------------------------------------------------------------------ layout / wire
@register("trunc_bf16")
def trunc_bf16(src, dst):
    """dst (bf16) ← the top 16 bits of src (fp32): the reference's truncating wire format."""
    if not (src.is_cuda and src.dtype == _f32 and dst.dtype == _bf16 and src.is_contiguous() and dst.is_contiguous()
            and src.numel() == dst.numel() and _al16(src) and dst.data_ptr() % 8 == 0):
        return NotImplemented
    if src.numel():
        check(_lib().bigdl_trunc_bf16(ptr(src), ptr(dst), _ll(src.numel()), _s()), "trunc_bf16")
    return dst


def nchw_to_nhwc_padded(x, slot, cp=4):
    """A contiguous NCHW image batch with C < ``cp`` (the RGB model input) → the stem conv's
    channel-padded bf16 NHWC operand in ONE pass (csrc/elementwise.hip k_nchw_to_nhwc_pad).  Returns
    the C-channel view of it (logical NCHW, the layer's input for every other purpose) and parks
    (view, version, cp, padded) in the conv's pad ``slot`` — :func:`_pad_channels` and the conv
    launch take the padded tensor from there instead of padding again."""
    if not (x.is_cuda and x.dim() == 4 and x.is_contiguous() and x.dtype in (_f32, _bf16) and slot is not None):
        return NotImplemented
    N_, C_, H, W = x.shape
    if C_ >= cp or N_ * H * W == 0:
        return NotImplemented
    padded = torch.empty((N_, cp, H, W), dtype=_bf16, device=x.device, memory_format=torch.channels_last)
    check(_lib().bigdl_nchw_to_nhwc_pad_bf16(ptr(x), C.c_int(0 if x.dtype == _f32 else 1), ptr(padded), C.c_int(N_),
                                             C.c_int(C_), _ll(H * W), C.c_int(cp), _s()), "nchw_to_nhwc_pad_bf16")
    view = padded[:, :C_]
    slot[0] = (view, view._version, cp, padded)
    return view


def _prepadded(x, slot):
    """The channel-padded copy of ``x`` a layout conversion already parked in ``slot`` (or None)."""
    if slot is not None and isinstance(slot[0], tuple) and len(slot[0]) == 4:
        src, ver, ct, padded = slot[0]
        if src is x and ver == x._version:
            return padded
    return None


@register("nchw_to_nhwc_bf16")
def nchw_to_nhwc_bf16(x):
    """Contiguous NCHW (fp32 / bf16) → channels-last bf16 in one pass (tiled LDS transpose)."""
    if not (x.is_cuda and x.dim() == 4 and x.is_contiguous() and x.dtype in (_f32, _bf16)):
        return NotImplemented
    N_, C_, H, W = x.shape
    if N_ > 65535 or N_ * C_ * H * W == 0:
        return NotImplemented
    y = torch.empty((N_, C_, H, W), dtype=_bf16, device=x.device, memory_format=torch.channels_last)
    check(_lib().bigdl_nchw_to_nhwc_bf16(ptr(x), C.c_int(0 if x.dtype == _f32 else 1), ptr(y), C.c_int(N_),
                                         C.c_int(C_), _ll(H * W), _s()), "nchw_to_nhwc_bf16")
    return y


# ------------------------------------------------------------------------------------------------ detection
_NMS_MAX = 32768


@register("nms")
def nms(boxes_sorted, thresh, plus_one=1.0, max_keep=-1):
    """Greedy NMS of score-sorted ``boxes_sorted [n, 4]`` on the device (pairwise IoU bitmask +
    one-wave scan, detection.hip); returns the kept positions (int64, score order)."""
    if not (boxes_sorted.is_cuda and boxes_sorted.dim() == 2 and boxes_sorted.shape[1] == 4):
        return NotImplemented
    n = boxes_sorted.shape[0]
    if n == 0 or n > _NMS_MAX:
        return NotImplemented
    b = boxes_sorted.float().contiguous()
    words = (n + 63) // 64
    mask = torch.empty(n * words, dtype=torch.int64, device=b.device)
    keep = torch.empty(n, dtype=torch.int64, device=b.device)
    count = torch.empty(1, dtype=torch.int32, device=b.device)
    check(_lib().bigdl_nms(ptr(b), C.c_int(n), _f(thresh), _f(plus_one), C.c_int(int(max_keep)), ptr(mask), ptr(keep),
                           ptr(count), _s()), "nms")
    return keep[:int(count.item())]


def _roi_strides(x, y):
    return (C.c_longlong * 8)(*[int(s) for s in x.stride()], *[int(s) for s in y.stride()])


class _RoiAlignFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, data, rois, scale, oh, ow, sr, aligned):
        K = rois.shape[0]
        N_, C_, H, W = data.shape
        y = torch.empty((K, C_, oh, ow), dtype=_f32, device=data.device)
        st = _roi_strides(data, y)
        check(_lib().bigdl_roi_align_fwd(ptr(data), C.c_int(0 if data.dtype == _f32 else 1), ptr(rois), ptr(y),
                                         C.c_int(K), C.c_int(C_), C.c_int(H), C.c_int(W), C.c_int(oh), C.c_int(ow),
                                         _f(scale), C.c_int(sr), C.c_int(1 if aligned else 0), st, _s()),
              "roi_align_fwd")
        ctx.save_for_backward(rois)
        ctx.meta = (data.shape, data.dtype, data.stride(), scale, oh, ow, sr, aligned)
        return y

    @staticmethod
    def backward(ctx, gy):
        (rois,) = ctx.saved_tensors
        shape, dtype, stride, scale, oh, ow, sr, aligned = ctx.meta
        N_, C_, H, W = shape
        cl = stride[1] == 1 and C_ > 1
        gx = torch.empty(shape, dtype=_f32, device=gy.device,
                         memory_format=torch.channels_last if cl else torch.contiguous_format).zero_()
        gy = gy.float()
        st = _roi_strides(gx, gy)
        check(_lib().bigdl_roi_align_bwd(ptr(gy), ptr(rois), ptr(gx), C.c_int(rois.shape[0]), C.c_int(C_), C.c_int(H),
                                         C.c_int(W), C.c_int(oh), C.c_int(ow), _f(scale), C.c_int(sr),
                                         C.c_int(1 if aligned else 0), st, _s()), "roi_align_bwd")
        return gx.to(dtype), None, None, None, None, None, None


@register("roi_align")
def roi_align(data, rois, spatial_scale, out_h, out_w, sampling_ratio=2, aligned=True):
    """Bilinear ROI align on the device (detection.hip); fp32 output cast to ``data.dtype``,
    differentiable w.r.t. ``data``."""
    if not (data.is_cuda and data.dim() == 4 and data.dtype in (_f32, _bf16) and rois.dim() == 2
            and rois.shape[1] == 5 and rois.shape[0] > 0 and min(data.shape) > 0):
        return NotImplemented
    r = rois.detach().float().contiguous().to(data.device)
    y = _RoiAlignFn.apply(data, r, float(spatial_scale), int(out_h), int(out_w), int(sampling_ratio), bool(aligned))
    return y.to(data.dtype)


# ------------------------------------------------------------------------------------------------ vector math
# op codes of ops/csrc/vml.hip
VML_UNARY = {"abs": 0, "exp": 1, "log": 2, "log1p": 3, "sqrt": 4, "tanh": 5, "sigmoid": 6, "pow": 7,
             "square": 8, "inv": 9, "neg": 10, "affine": 11}
VML_BINARY = {"add": 0, "sub": 1, "mul": 2, "div": 3, "tanh_bwd": 4, "sigmoid_bwd": 5, "sqrt_bwd": 6,
              "log_bwd": 7, "exp_bwd": 8, "square_bwd": 9, "abs_bwd": 10, "pow_bwd": 11}
REDUCE = {"sum": 0, "mean": 1, "max": 2, "min": 3}


def _dense(t):
    return t.is_contiguous() or (t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last))


def _vml_ok(*ts):
    """Elementwise kernels walk the storage linearly: every operand dense (row-major or NHWC) with
    the same strides, same dtype and element count."""
    t0 = ts[0]
    return all(t is not None and t.is_cuda and t.dtype == t0.dtype and t.dtype in (_f32, _bf16) and _dense(t)
               and t.shape == t0.shape and t.stride() == t0.stride() and _al16(t) for t in ts) and t0.numel() > 0


@register("vml_unary")
def vml_unary(x, op, p=0.0, q=0.0, out=None):
    """Elementwise ``op`` (a VML_UNARY name) of a contiguous fp32/bf16 device tensor; ``out`` may
    alias ``x`` (in place).  pow: x**p; affine: x·p + q."""
    y = torch.empty_like(x) if out is None else out
    if not _vml_ok(x, y):
        return NotImplemented
    check(_lib().bigdl_vml_unary(C.c_int(VML_UNARY[op]), C.c_int(0 if x.dtype == _f32 else 1), ptr(x), ptr(y),
                                 _ll(x.numel()), _f(p), _f(q), _s()), "vml_unary")
    return y


@register("vml_binary")
def vml_binary(a, b, op, p=1.0, out=None):
    """Elementwise ``op`` (a VML_BINARY name) of two same-shape contiguous device tensors
    (add/sub: a ± p·b; *_bwd: a = upstream gradient, b = saved forward value; pow_bwd uses p)."""
    z = torch.empty_like(a) if out is None else out
    if not _vml_ok(a, b, z):
        return NotImplemented
    check(_lib().bigdl_vml_binary(C.c_int(VML_BINARY[op]), C.c_int(0 if a.dtype == _f32 else 1), ptr(a), ptr(b),
                                  ptr(z), _ll(a.numel()), _f(p), _s()), "vml_binary")
    return z


@register("reduce")
def reduce(x, op, dim=None, keepdim=False):
    """sum / mean / max / min of a contiguous fp32/bf16 device tensor over ``dim`` (None: all
    elements), fp32 result (deterministic two-level order)."""
    if not (x.is_cuda and x.dtype in (_f32, _bf16) and x.is_contiguous() and x.numel() > 0):
        return NotImplemented
    shape = list(x.shape)
    if dim is None:
        outer, n, inner = 1, x.numel(), 1
        oshape = [1] * len(shape) if keepdim else []
    else:
        d = dim % max(1, x.dim())
        outer = 1
        for s_ in shape[:d]:
            outer *= s_
        inner = 1
        for s_ in shape[d + 1:]:
            inner *= s_
        n = shape[d]
        oshape = shape[:d] + ([1] if keepdim else []) + shape[d + 1:]
    out = torch.empty(outer * inner, dtype=_f32, device=x.device)
    scratch = torch.empty(max(outer * 64, 8192), dtype=_f32, device=x.device)
    check(_lib().bigdl_reduce(C.c_int(REDUCE[op]), C.c_int(0 if x.dtype == _f32 else 1), ptr(x), _ll(outer), _ll(n),
                              _ll(inner), ptr(out), ptr(scratch), _ll(scratch.numel()), _s()), "reduce")
    return out.view(oshape)


# ------------------------------------------------------------------------------------------------ autograd conv
class _ConvFn(torch.autograd.Function):
    """The native conv as an autograd op, for layers defined by their forward (AutogradModule):
    forward = conv2d_forward, backward = conv2d_backward (data, weight and bias gradients)."""

    @staticmethod
    def forward(ctx, x, w, b, stride, pad, dilation, groups):
        y = conv2d_forward(x, w.to(_bf16), b, stride, pad, dilation, groups)
        if y is NotImplemented:
            raise RuntimeError("native conv refused its geometry after the eligibility check")
        ctx.save_for_backward(x, w, b)
        ctx.geom = (stride, pad, dilation, groups)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, b = ctx.saved_tensors
        stride, pad, dilation, groups = ctx.geom
        gw = torch.zeros(w.shape, dtype=_f32, device=w.device)
        gb = torch.zeros(b.shape, dtype=_f32, device=w.device) if b is not None else None
        gy = gy.to(_bf16).contiguous(memory_format=torch.channels_last)
        gi = conv2d_backward(gy, x, w.to(_bf16), stride, pad, dilation, groups, ctx.needs_input_grad[0], gw, gb, 1.0)
        if gi is NotImplemented:
            raise RuntimeError("native conv backward refused its geometry")
        return gi, gw.to(w.dtype), (gb.to(b.dtype) if gb is not None else None), None, None, None, None


def conv2d_autograd(x, w, b, stride, pad, dilation=(1, 1), groups=1):
    """Differentiable native conv (NotImplemented when the geometry is not native-eligible)."""
    if not (x.is_cuda and x.dim() == 4 and x.dtype == _bf16 and x.is_contiguous(memory_format=torch.channels_last)
            and _al16(x)):
        return NotImplemented
    wb = w.detach().to(_bf16)
    ok = _depthwise_ok(x, wb, groups) or (groups == 1 and x.shape[1] % 8 == 0 and w.shape[0] % 8 == 0) or \
        (groups > 1 and _grouped_ok(x, wb, groups))
    if not ok:
        return NotImplemented
    return _ConvFn.apply(x, w, b, tuple(stride), tuple(pad), tuple(dilation), groups)


# ------------------------------------------------------------------------------------------------ 3-D conv
_cl3 = torch.channels_last_3d


def _conv3d_launch(x, w, b, out_dims, stride, pad, dilation):
    """y [N][To][P][Q][K] = conv3d(x [N][T][H][W][C], w [K][KT][R][S][C]) (+ fp32 bias) on the
    implicit-GEMM kernel (conv_igemm.hip D3 instantiations); x, w bf16 channels_last_3d, C % 8 == 0."""
    N_, C_, T, H, W = x.shape
    K, _, KT, R, S = w.shape
    To, P, Q = out_dims
    y = torch.empty((N_, K, To, P, Q), dtype=_bf16, device=x.device, memory_format=_cl3)
    check(_lib().bigdl_conv3d_fwd(ptr(x), ptr(w), ptr(b), ptr(y), N_, T, H, W, C_, K, KT, R, S, To, P, Q,
                                  stride[0], stride[1], stride[2], pad[0], pad[1], pad[2],
                                  dilation[0], dilation[1], dilation[2], 0, _s()), "conv3d_fwd")
    return y


def _pad_c8(t):
    """Zero-pad dim 1 (channels) to a multiple of 8, channels_last_3d bf16."""
    c = t.shape[1]
    cp = -(-c // 8) * 8
    if cp != c:
        t = torch.nn.functional.pad(t, (0, 0, 0, 0, 0, 0, 0, cp - c))
    return t.to(_bf16).contiguous(memory_format=_cl3)


class _Conv3dFn(torch.autograd.Function):
    """VolumetricConvolution on the implicit-GEMM kernels: forward and the stride-1 data gradient
    (a forward conv of dY with the flipped, transposed filter; strided convs first scatter dY onto
    the stride lattice) on k_conv_fwd<…, D3>, the weight gradient on k_conv_wgrad<…, D3>
    (VolumetricConvolution.scala updateOutput / updateGradInput / accGradParameters)."""

    @staticmethod
    def forward(ctx, x, w, b, stride, pad, dilation, out_dims):
        C_ = x.shape[1]
        xp, wp = _pad_c8(x), _pad_c8(w.detach())
        bias = b.detach().float().contiguous() if b is not None else None
        y = _conv3d_launch(xp, wp, bias, out_dims, stride, pad, dilation)
        ctx.save_for_backward(xp, wp)
        ctx.geom = (stride, pad, dilation, tuple(x.shape[2:]), C_, b is not None, w.dtype)
        return y

    @staticmethod
    def backward(ctx, gy):
        xp, wp = ctx.saved_tensors
        stride, pad, dilation, in_dims, C_, has_b, wdt = ctx.geom
        gb = gy.float().sum((0, 2, 3, 4)).to(wdt) if has_b else None
        gy = gy.to(_bf16).contiguous(memory_format=_cl3)
        N_, K, To, P, Q = gy.shape
        KT, R, S = wp.shape[2:]
        Cp = xp.shape[1]
        gx = None
        if ctx.needs_input_grad[0]:
            src = gy
            if any(s_ != 1 for s_ in stride):  # dY on the stride lattice, zeros between
                src = torch.empty((N_, K, (To - 1) * stride[0] + 1, (P - 1) * stride[1] + 1, (Q - 1) * stride[2] + 1),
                                  dtype=_bf16, device=gy.device, memory_format=_cl3).zero_()
                src[:, :, ::stride[0], ::stride[1], ::stride[2]] = gy
            wt = wp.flip(2, 3, 4).transpose(0, 1).contiguous(memory_format=_cl3)  # [Cp][KT][R][S][K]
            pd = tuple(d * (k - 1) - p_ for d, k, p_ in zip(dilation, (KT, R, S), pad))
            gx = _conv3d_launch(src, wt, None, in_dims, (1, 1, 1), pd, dilation)[:, :C_]
        gw = torch.zeros(wp.shape, dtype=_f32, device=gy.device).contiguous(memory_format=_cl3)
        T, H, W = in_dims
        check(_lib().bigdl_conv3d_wgrad(ptr(xp), ptr(gy), ptr(gw), _f(1.0), N_, T, H, W, Cp, K, KT, R, S, To, P, Q,
                                        stride[0], stride[1], stride[2], pad[0], pad[1], pad[2],
                                        dilation[0], dilation[1], dilation[2], _s()), "conv3d_wgrad")
        return gx, gw[:, :C_].to(wdt), gb, None, None, None, None


def conv3d_autograd(x, w, b, stride, pad, dilation=(1, 1, 1), out_dims=None):
    """Differentiable native 3-D conv (NotImplemented when not eligible).  ``pad`` is the leading
    pad per dim; ``out_dims`` (To, P, Q) defaults to the symmetric-padding output size."""
    if not (x.is_cuda and x.dim() == 5 and w.dim() == 5 and w.shape[1] == x.shape[1]):
        return NotImplemented
    K, C_, KT, R, S = w.shape
    if K % 8:
        return NotImplemented
    if out_dims is None:
        out_dims = tuple((i + 2 * p_ - d * (k - 1) - 1) // s_ + 1
                         for i, p_, d, k, s_ in zip(x.shape[2:], pad, dilation, (KT, R, S), stride))
    if min(out_dims) <= 0:
        return NotImplemented
    N_ = x.shape[0]
    Cp = -(-C_ // 8) * 8
    T, H, W = x.shape[2:]
    To, P, Q = out_dims
    lim = 0x7fffffff
    if N_ * T * H * W * max(Cp, K) * 2 >= lim or N_ * To * P * Q * K * 2 >= lim or \
            N_ * (To * stride[0]) * (P * stride[1]) * (Q * stride[2]) * K * 2 >= lim:
        return NotImplemented
    return _Conv3dFn.apply(x, w, b, tuple(stride), tuple(pad), tuple(dilation), tuple(out_dims))


# ------------------------------------------------------------------------------------------------ transposed conv
class _DeconvFn(torch.autograd.Function):
    """Transposed convolution (SpatialFullConvolution) on the conv kernels: its forward is the
    backward-data of the conv whose weight is [K = C_in][C = C_out][R][S]; its backward-data is that
    conv's forward; its weight gradient is that conv's weight gradient with the roles of input and
    output gradient exchanged (conv input = dY, conv output gradient = X)."""

    @staticmethod
    def forward(ctx, x, w, b, stride, pad, out_hw):
        N_, Cin, H, W = x.shape
        Cout = w.shape[1]
        wb = w.detach().to(_bf16)
        shape = (N_, Cout, out_hw[0], out_hw[1])
        if tuple(stride) == (1, 1):
            y = _dgrad_s1(x, wb, shape, pad, (1, 1))
        else:
            y = _dgrad_strided(x, wb, shape, tuple(stride), tuple(pad), (1, 1))
        if y is None:
            raise RuntimeError("native transposed conv refused its geometry after the eligibility check")
        if b is not None:
            y = y + b.to(y.dtype).view(1, -1, 1, 1)
        ctx.save_for_backward(x, w, b)
        ctx.geom = (tuple(stride), tuple(pad))
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, b = ctx.saved_tensors
        stride, pad = ctx.geom
        gb = gy.float().sum((0, 2, 3)).to(b.dtype) if b is not None else None  # before the bf16 cast
        gy = gy.to(_bf16).contiguous(memory_format=torch.channels_last)
        wb = w.detach().to(_bf16)
        gx = None
        if ctx.needs_input_grad[0]:
            gx = conv2d_forward(gy, wb, None, stride, pad)
            if gx is NotImplemented:
                raise RuntimeError("native transposed-conv backward-data refused its geometry")
        gw = torch.zeros(w.shape, dtype=_f32, device=w.device)
        _wgrad_launch(gy, x, wb, gw, 1.0, stride, pad, (1, 1), None)
        return gx, gw.to(w.dtype), gb, None, None, None


class _GroupedDeconvFn(torch.autograd.Function):
    """Grouped transposed convolution (SpatialFullConvolution nGroup > 1) on the single-launch
    grouped conv kernels: with W [C_in][C_out/G][R][S] the weight of the grouped conv whose
    backward-data this is, the forward is that conv's data gradient (x on the stride lattice, each
    group's flipped, transposed filter), the input gradient is that conv's forward of dY, and the
    weight gradient is its grouped weight gradient with input = dY and output gradient = x."""

    @staticmethod
    def forward(ctx, x, w, b, stride, pad, out_hw, groups):
        N_, Cin, H, W = x.shape
        _, Cog, R, S = w.shape
        src = x
        if tuple(stride) != (1, 1):
            src = torch.empty((N_, Cin, (H - 1) * stride[0] + 1, (W - 1) * stride[1] + 1), dtype=_bf16,
                              device=x.device, memory_format=torch.channels_last).zero_()
            src[:, :, ::stride[0], ::stride[1]] = x
        Cig = Cin // groups
        wt = w.detach().reshape(groups, Cig, Cog, R, S).flip(3, 4).transpose(1, 2).reshape(groups * Cog, Cig, R, S)
        y = _conv_fwd_grouped_1(src, wt, b, (1, 1), (R - 1 - pad[0], S - 1 - pad[1]), (1, 1), groups, out_hw=out_hw)
        if y is NotImplemented:
            raise RuntimeError("native grouped transposed conv refused its geometry after the eligibility check")
        ctx.save_for_backward(x, w)
        ctx.geom = (tuple(stride), tuple(pad), groups, b is not None, None if b is None else b.dtype)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        stride, pad, groups, has_b, bdt = ctx.geom
        gb = gy.float().sum((0, 2, 3)).to(bdt) if has_b else None
        gy = gy.to(_bf16).contiguous(memory_format=torch.channels_last)
        gx = None
        if ctx.needs_input_grad[0]:
            gx = _conv_fwd_grouped_1(gy, w.detach().to(_bf16), None, stride, pad, (1, 1), groups,
                                     out_hw=(x.shape[2], x.shape[3]))
            if gx is NotImplemented:
                raise RuntimeError("native grouped transposed-conv backward-data refused its geometry")
        gw = torch.zeros(w.shape, dtype=_f32, device=w.device)
        r = _conv_bwd_grouped_1(x, gy, w.detach().to(_bf16), stride, pad, (1, 1), groups, False, gw, None, 1.0)
        if r is NotImplemented:
            raise RuntimeError("native grouped transposed-conv weight gradient refused its geometry")
        return gx, gw.to(w.dtype), gb, None, None, None, None


def conv_transpose2d(x, w, b, stride, pad, adj=(0, 0), groups=1):
    """Differentiable native transposed conv; NotImplemented when not eligible.
    ``w``: [C_in][C_out / groups][R][S]."""
    if not (x.is_cuda and x.dim() == 4 and x.dtype == _bf16 and x.is_contiguous(memory_format=torch.channels_last)
            and _al16(x) and w.dim() == 4 and w.shape[0] == x.shape[1]):
        return NotImplemented
    if groups > 1:
        Cin, Cog, R, S = w.shape
        H, W = x.shape[2], x.shape[3]
        oh = (H - 1) * stride[0] - 2 * pad[0] + R + adj[0]
        ow = (W - 1) * stride[1] - 2 * pad[1] + S + adj[1]
        if Cin % groups or oh <= 0 or ow <= 0 or adj[0] >= max(stride[0], 1) or adj[1] >= max(stride[1], 1):
            return NotImplemented
        Cig = Cin // groups
        if _group_pack(groups, Cig, Cog) is None or _group_pack(groups, Cog, Cig) is None:
            return NotImplemented
        return _GroupedDeconvFn.apply(x, w, b, tuple(stride), tuple(pad), (oh, ow), groups)
    Cin, Cout, R, S = w.shape
    if Cin % 8 or Cout % 8:
        return NotImplemented
    H, W = x.shape[2], x.shape[3]
    oh = (H - 1) * stride[0] - 2 * pad[0] + R + adj[0]
    ow = (W - 1) * stride[1] - 2 * pad[1] + S + adj[1]
    if oh <= 0 or ow <= 0 or adj[0] >= max(stride[0], 1) or adj[1] >= max(stride[1], 1):
        return NotImplemented
    if stride[0] == 1 and stride[1] == 1 and (R - 1 - pad[0] < 0 or S - 1 - pad[1] < 0):
        return NotImplemented
    return _DeconvFn.apply(x, w, b, tuple(stride), tuple(pad), (oh, ow))


# ------------------------------------------------------------------------------------------------ bilinear resize
class _ResizeFn(torch.autograd.Function):
    """Bilinear resize (reference sampling) on resize.hip: NHWC bf16 forward, fp32-atomic backward."""

    @staticmethod
    def forward(ctx, x, oh, ow, align):
        N_, C_, H, W = x.shape
        y = torch.empty((N_, C_, oh, ow), dtype=_bf16, device=x.device, memory_format=torch.channels_last)
        check(_lib().bigdl_resize_bilinear_fwd(ptr(x), ptr(y), N_, H, W, C_, oh, ow, int(bool(align)), _s()),
              "resize_bilinear_fwd")
        ctx.geom = (N_, C_, H, W, oh, ow, int(bool(align)))
        return y

    @staticmethod
    def backward(ctx, gy):
        N_, C_, H, W, oh, ow, align = ctx.geom
        gy = gy.to(_bf16).contiguous(memory_format=torch.channels_last)
        gx = torch.zeros((N_, H, W, C_), dtype=_f32, device=gy.device)
        check(_lib().bigdl_resize_bilinear_bwd(ptr(gy), ptr(gx), N_, H, W, C_, oh, ow, align, _s()),
              "resize_bilinear_bwd")
        return gx.permute(0, 3, 1, 2).to(_bf16), None, None, None


@register("resize_bilinear")
def resize_bilinear(x, oh, ow, align=False):
    """Differentiable native bilinear resize of an NCHW-logical bf16 channels-last tensor
    (NotImplemented when not eligible; deterministic mode keeps the atomic-free reference)."""
    if not (x.is_cuda and x.dim() == 4 and x.dtype == _bf16 and x.shape[1] % 8 == 0 and _al16(x)
            and x.is_contiguous(memory_format=torch.channels_last)):
        return NotImplemented
    if config.get_property("bigdl.deterministic"):
        return NotImplemented
    return _ResizeFn.apply(x, int(oh), int(ow), bool(align))


# ------------------------------------------------------------------------------------------------ 3-D pooling
def _pool_out(n, k, s_, p_, ceil):
    o = (n + 2 * p_ - k + ((s_ - 1) if ceil else 0)) // s_ + 1
    if ceil and (o - 1) * s_ >= n + p_:
        o -= 1
    return o


class _Pool3dFn(torch.autograd.Function):
    """VolumetricMax/AveragePooling on pool3d.hip (NDHWC bf16; max keeps a uint8 window argmax)."""

    @staticmethod
    def forward(ctx, x, mode, k, st, pd, out, cip):
        N_, C_, T, H, W = x.shape
        OT, OH, OW = out
        y = torch.empty((N_, C_, OT, OH, OW), dtype=_bf16, device=x.device, memory_format=_cl3)
        idx = torch.empty((N_, OT, OH, OW, C_), dtype=torch.uint8, device=x.device) if mode == 0 else None
        check(_lib().bigdl_pool3d_fwd(mode, ptr(x), ptr(y), ptr(idx), N_, T, H, W, C_, OT, OH, OW, k[0], k[1], k[2],
                                      st[0], st[1], st[2], pd[0], pd[1], pd[2], int(bool(cip)), _s()), "pool3d_fwd")
        if idx is not None:
            ctx.save_for_backward(idx)
        ctx.geom = (mode, k, st, pd, (N_, C_, T, H, W), out, int(bool(cip)))
        return y

    @staticmethod
    def backward(ctx, gy):
        mode, k, st, pd, (N_, C_, T, H, W), (OT, OH, OW), cip = ctx.geom
        idx = ctx.saved_tensors[0] if mode == 0 else None
        gy = gy.to(_bf16).contiguous(memory_format=_cl3)
        gx = torch.zeros((N_, T, H, W, C_), dtype=_f32, device=gy.device)
        check(_lib().bigdl_pool3d_bwd(mode, ptr(gy), ptr(idx), ptr(gx), N_, T, H, W, C_, OT, OH, OW, k[0], k[1], k[2],
                                      st[0], st[1], st[2], pd[0], pd[1], pd[2], cip, _s()), "pool3d_bwd")
        return gx.permute(0, 4, 1, 2, 3).to(_bf16), None, None, None, None, None, None


@register("pool3d")
def pool3d(x, mode, k, st, pd, ceil=False, count_include_pad=True):
    """Differentiable native 3-D pooling (mode 0 max, 1 average) of an NCDHW-logical bf16 tensor;
    NotImplemented when not eligible (deterministic mode keeps the atomic-free reference)."""
    if not (x.is_cuda and x.dim() == 5 and x.dtype == _bf16 and x.shape[1] % 8 == 0 and _al16(x)
            and x.is_contiguous(memory_format=_cl3)):
        return NotImplemented
    if config.get_property("bigdl.deterministic") or k[0] * k[1] * k[2] > 255:
        return NotImplemented
    if any(p_ * 2 > kk for p_, kk in zip(pd, k)):
        return NotImplemented  # torch's rule: pad ≤ kernel / 2 (windows always touch the input)
    out = tuple(_pool_out(n, kk, s_, p_, ceil) for n, kk, s_, p_ in zip(x.shape[2:], k, st, pd))
    if min(out) <= 0:
        return NotImplemented
    return _Pool3dFn.apply(x, mode, tuple(k), tuple(st), tuple(pd), out, count_include_pad)


# ------------------------------------------------------------------------------------------------ layer norm
_LN_MAX_H = 4096


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, eps):
        H = x.shape[-1]
        rows = x.numel() // H
        y = torch.empty_like(x)
        mean = torch.empty(rows, dtype=_f32, device=x.device)
        rstd = torch.empty(rows, dtype=_f32, device=x.device)
        wf = None if w is None else w.detach().float().contiguous()
        bf = None if b is None else b.detach().float().contiguous()
        check(_lib().bigdl_ln_fwd(ptr(x), C.c_int(0 if x.dtype == _f32 else 1), ptr(wf), ptr(bf), ptr(y), ptr(mean),
                                  ptr(rstd), _ll(rows), C.c_int(H), _f(eps), _s()), "ln_fwd")
        ctx.save_for_backward(x, wf, mean, rstd)
        ctx.meta = (w is not None and w.requires_grad, b is not None and b.requires_grad,
                    None if w is None else w.dtype, None if b is None else b.dtype)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, wf, mean, rstd = ctx.saved_tensors
        need_w, need_b, wdt, bdt = ctx.meta
        H = x.shape[-1]
        rows = x.numel() // H
        gy = gy.to(x.dtype).contiguous()
        gx = torch.empty_like(x)
        # one buffer: [gw | gb | block partials (≤ 512 rows of 2H)] — a single allocation and memset
        G = min(512, max(1, (rows + 3) // 4))
        buf = torch.empty(2 * H + G * 2 * H, dtype=_f32, device=x.device)
        buf[:2 * H].zero_()
        gw = buf[:H] if need_w else None
        gb = buf[H:2 * H] if need_b else None
        check(_lib().bigdl_ln_bwd(ptr(gy), ptr(x), C.c_int(0 if x.dtype == _f32 else 1), ptr(wf), ptr(mean), ptr(rstd),
                                  ptr(gx), ptr(gw), ptr(gb), _ll(rows), C.c_int(H), ptr(buf[2 * H:]), _ll(G * 2 * H),
                                  _s()), "ln_bwd")
        return gx, None if gw is None else gw.to(wdt), None if gb is None else gb.to(bdt), None


@register("layer_norm")
def layer_norm(x, weight=None, bias=None, eps=1e-5):
    """Layer normalisation over the last dimension (layernorm.hip): one wave per row, fp32
    statistics, fp32/bf16 I/O; differentiable w.r.t. x, weight and bias (fp32 [H] each)."""
    if not (x.is_cuda and x.dtype in (_f32, _bf16) and x.dim() >= 1 and 0 < x.shape[-1] <= _LN_MAX_H
            and x.numel() > 0):
        return NotImplemented
    H = x.shape[-1]
    if any(p is not None and (p.numel() != H or not p.is_cuda) for p in (weight, bias)):
        return NotImplemented
    return _LayerNormFn.apply(x.contiguous(), weight, bias, float(eps))


# ---------------------------------------------------------------------------------- K30 attention
def _attn_rows_ok(t, rows, cols):
    """[rows][≥cols] bf16 device rows, unit column stride, 16-B aligned, row stride % 8 == 0."""
    return (isinstance(t, torch.Tensor) and t.dim() == 2 and t.dtype == _bf16 and t.is_cuda
            and t.shape[0] == rows and t.shape[1] >= cols and t.stride(1) == 1 and t.stride(0) % 8 == 0
            and t.stride(0) >= cols and _al16(t))


def _attn_bias(bias, B, Hh, Lq, Lk, device):
    """fp32 bias broadcast to (B, Hh, Lq, Lk) → (tensor, element strides); broadcast dims get
    stride 0, so a (1, 1, L, L) or (B, 1, 1, L) mask is read in place."""
    if bias is None:
        return None, (0, 0, 0, 0)
    b = bias.to(device=device, dtype=_f32)
    while b.dim() < 4:
        b = b.unsqueeze(0)
    try:
        b = torch.broadcast_to(b, (B, Hh, Lq, Lk))
    except RuntimeError:
        return NotImplemented, None
    return b, tuple(b.stride())


def attention_seed(device, rng=None):
    """The dropout seed of one attention call, shared by its forward and backward: a host int, or
    under HIP-graph capture a snapshot of the per-device seed counter (a fresh mask per replay)."""
    if torch.cuda.is_current_stream_capturing():
        snap = _device_seed(device).clone()
        _device_seed(device).add_(1)
        return snap
    return int(torch.randint(0, 2 ** 31, (1,), generator=rng))


def _seed_args(seed):
    if isinstance(seed, torch.Tensor):
        return C.c_uint(0), ptr(seed)
    return C.c_uint(int(seed) & 0xFFFFFFFF), ptr(None)


@register("attention_forward")
def attention_forward(q, k, v, B, Hh, Lq, Lk, D, scale, bias=None, causal=False, keep=1.0, seed=0):
    """Fused multi-head attention (attention.hip) on projection rows; see the reference op."""
    HD = Hh * D
    if D not in (32, 64, 96, 128) or not (_attn_rows_ok(q, B * Lq, HD) and _attn_rows_ok(k, B * Lk, HD)
                                  and _attn_rows_ok(v, B * Lk, HD)):
        return NotImplemented
    if (causal and Lq != Lk) or not (0.0 < keep <= 1.0):
        return NotImplemented
    bt, bs = _attn_bias(bias, B, Hh, Lq, Lk, q.device)
    if bt is NotImplemented:
        return NotImplemented
    out = torch.empty((B * Lq, HD), dtype=_bf16, device=q.device)
    lse = torch.empty((B, Hh, Lq), dtype=_f32, device=q.device)
    hs, ds = _seed_args(seed)
    check(_lib().bigdl_attn_fwd(ptr(q), _ll(q.stride(0)), ptr(k), _ll(k.stride(0)), ptr(v), _ll(v.stride(0)),
                                ptr(out), _ll(HD), ptr(lse), ptr(bt), *[_ll(x) for x in bs], C.c_int(B), C.c_int(Hh),
                                C.c_int(Lq), C.c_int(Lk), C.c_int(D), _f(scale), C.c_int(1 if causal else 0),
                                _f(keep), hs, ds, _s()), "attn_fwd")
    return out, lse


@register("attention_decode")
def attention_decode(q, kc, vc, L, Hh, D, scale, bias=None, bias_rev=True):
    """Cached incremental-decoding attention (attn_decode.hip): ``q`` [rows, Lq, H] attends over the
    first ``L`` positions of the preallocated caches ``kc`` / ``vc`` [rows, Lmax, H]; ``bias``
    broadcastable to (rows, Hh, Lq, L), indexed newest-key-first when ``bias_rev`` (the reference's
    [new; cache] concatenation order).  Returns o [rows, Lq, H] bf16."""
    if not (q.dim() == 3 and kc.dim() == 3 and vc.dim() == 3 and q.dtype == _bf16 and kc.dtype == _bf16
            and vc.dtype == _bf16 and q.is_cuda):
        return NotImplemented
    rows, Lq, H = q.shape
    if H != Hh * D or D % 8 or D > 256 or kc.shape[0] != rows or vc.shape[0] != rows or kc.shape[1] < L \
            or vc.shape[1] < L or L <= 0:
        return NotImplemented
    if q.stride(2) != 1 or kc.stride(2) != 1 or vc.stride(2) != 1 or q.stride(0) != Lq * q.stride(1):
        return NotImplemented
    if not (_al16(q) and _al16(kc) and q.stride(1) % 8 == 0 and kc.stride(1) % 8 == 0 and kc.stride(0) % 8 == 0):
        return NotImplemented
    bt, bs = _attn_bias(bias, rows, Hh, Lq, L, q.device)
    if bt is NotImplemented:
        return NotImplemented
    out = torch.empty((rows, Lq, H), dtype=_bf16, device=q.device)
    check(_lib().bigdl_attn_decode(ptr(q), _ll(q.stride(1)), ptr(kc), _ll(kc.stride(1)), _ll(kc.stride(0)), ptr(vc),
                                   _ll(vc.stride(1)), _ll(vc.stride(0)), ptr(out), _ll(H), ptr(bt),
                                   *[_ll(x) for x in bs], C.c_int(1 if bias_rev else 0), C.c_int(rows), C.c_int(Hh),
                                   C.c_int(Lq), C.c_int(L), C.c_int(D), _f(scale), _s()), "attn_decode")
    return out


@register("attention_backward")
def attention_backward(dout, q, k, v, o, lse, B, Hh, Lq, Lk, D, scale, bias=None, causal=False, keep=1.0, seed=0,
                       dq=None, dk=None, dv=None):
    """dQ, dK, dV of :func:`attention_forward` (two kernels, no atomics); ``dq``/``dk``/``dv`` may be
    column slices of one fused [B·L][3·H] buffer (the QKV projection's backward reads it whole)."""
    HD = Hh * D
    if D not in (32, 64, 96, 128) or not (_attn_rows_ok(q, B * Lq, HD) and _attn_rows_ok(k, B * Lk, HD)
                                  and _attn_rows_ok(v, B * Lk, HD) and _attn_rows_ok(o, B * Lq, HD)
                                  and _attn_rows_ok(dout, B * Lq, HD)):
        return NotImplemented
    if (causal and Lq != Lk) or not (0.0 < keep <= 1.0):
        return NotImplemented
    if not (lse.dtype == _f32 and lse.is_contiguous() and lse.numel() == B * Hh * Lq):
        return NotImplemented
    bt, bs = _attn_bias(bias, B, Hh, Lq, Lk, q.device)
    if bt is NotImplemented:
        return NotImplemented
    outs = []
    for t, L in ((dq, Lq), (dk, Lk), (dv, Lk)):
        if t is None:
            t = torch.empty((B * L, HD), dtype=_bf16, device=q.device)
        elif not _attn_rows_ok(t, B * L, HD):
            return NotImplemented
        outs.append(t)
    dq, dk, dv = outs
    delta = torch.empty((B, Hh, Lq), dtype=_f32, device=q.device)
    hs, ds = _seed_args(seed)
    check(_lib().bigdl_attn_bwd(ptr(q), _ll(q.stride(0)), ptr(k), _ll(k.stride(0)), ptr(v), _ll(v.stride(0)),
                                ptr(o), _ll(o.stride(0)), ptr(dout), _ll(dout.stride(0)), ptr(lse), ptr(delta),
                                ptr(bt), *[_ll(x) for x in bs], ptr(dq), _ll(dq.stride(0)), ptr(dk),
                                _ll(dk.stride(0)), ptr(dv), _ll(dv.stride(0)), C.c_int(B), C.c_int(Hh), C.c_int(Lq),
                                C.c_int(Lk), C.c_int(D), _f(scale), C.c_int(1 if causal else 0), _f(keep), hs, ds,
                                _s()), "attn_bwd")
    return dq, dk, dv
