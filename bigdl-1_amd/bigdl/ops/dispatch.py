"""Device dispatch for the hot ops: native HIP kernels for GPU tensors, reference otherwise."""
from __future__ import annotations

import torch

from . import reference as R
from . import native as N

__all__ = [
    "cast_copy", "zero_fill", "relu_forward", "relu_backward",
    "conv2d_forward", "conv2d_backward", "conv_transpose2d_forward",
    "batchnorm_forward_train", "batchnorm_forward_infer", "batchnorm_backward",
    "maxpool2d_forward", "maxpool2d_backward", "avgpool2d_forward", "avgpool2d_backward",
    "linear_forward", "linear_backward",
    "log_softmax_forward", "log_softmax_backward", "softmax_forward", "softmax_backward",
    "class_nll_forward", "class_nll_backward", "cross_entropy_fused",
    "sgd_step", "adam_step", "lstm_cell_forward", "lstm_cell_backward",
    "embedding_forward", "embedding_backward", "dropout_forward", "dropout_backward", "lrn_forward", "lrn_backward",
    "quant_rows", "gemm_i8", "image_crop_flip_norm", "attention_forward", "attention_backward",
    "attention_decode",
]


def fallback_counts() -> dict:
    """{(op, reason, signature): count} of device-tensor calls that ran the torch reference op
    instead of a HIP kernel since the last :func:`reset_fallbacks`."""
    return N.fallback_counts()


def reset_fallbacks() -> None:
    N.reset_fallbacks()


def native_status() -> dict:
    return N.status()


def native_has(opname: str) -> bool:
    """True when device tensors of ``opname`` go to the HIP kernel (library loaded and enabled)."""
    return N.has(opname)


def _nat(t: torch.Tensor, opname: str) -> bool:
    """True → use the native kernel for this op on this tensor."""
    if not (isinstance(t, torch.Tensor) and t.is_cuda):
        return False
    return N.has(opname)


def _g(opname):
    nat = getattr(N, opname, None)
    ref = getattr(R, opname)

    def f(*args, **kwargs):
        t = None
        for a in args:
            if isinstance(a, torch.Tensor):
                t = a
                break
        if t is not None and t.is_cuda:
            if nat is not None and N.has(opname):
                r = nat(*args, **kwargs)
                if r is not NotImplemented:
                    return r
                N.note_fallback(opname, "unsupported", args)
            else:
                N.note_fallback(opname, "no-kernel" if nat is None else "disabled", args)
        # the reference ops take plain tensors: build any deferred BN input gradient first
        args = tuple(a.dense() if isinstance(a, R.BNGrad) else a for a in args)
        return ref(*args, **kwargs)

    f.__name__ = opname
    f.__doc__ = ref.__doc__
    return f


for _name in __all__:
    globals()[_name] = _g(_name)
