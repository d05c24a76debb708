"""Vector-math entry points (the reference's MKL VML role, ``tensor/TensorNumeric.scala:600-700``):
device tensors go to the HIP kernels of ``ops/csrc/vml.hip``; everything else (host tensors,
fp64, mixed dtypes, strided views) returns ``None`` and the caller runs its torch formulation.
A device tensor that could have used a kernel but did not is counted by ``note_fallback``."""
from __future__ import annotations

from typing import Optional

import torch

from . import native


def _eligible(*ts) -> bool:
    return all(t.is_cuda for t in ts)


def unary(x: torch.Tensor, op: str, p: float = 0.0, q: float = 0.0,
          out: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    if not (x.is_cuda and native.has("vml_unary")):
        return None
    r = native.native_ops.vml_unary(x, op, p, q, out)
    if r is NotImplemented:
        if x.dtype in (torch.float32, torch.bfloat16):
            native.note_fallback("vml_unary." + op, "layout", (x,))
        return None
    return r


def binary(a: torch.Tensor, b: torch.Tensor, op: str, p: float = 1.0,
           out: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    if not (_eligible(a, b) and native.has("vml_binary")):
        return None
    r = native.native_ops.vml_binary(a, b, op, p, out)
    if r is NotImplemented:
        if a.dtype == b.dtype and a.dtype in (torch.float32, torch.bfloat16) and a.shape == b.shape:
            native.note_fallback("vml_binary." + op, "layout", (a, b))
        return None
    return r


def reduce(x: torch.Tensor, op: str, dim: Optional[int] = None, keepdim: bool = False) -> Optional[torch.Tensor]:
    if not (x.is_cuda and native.has("reduce")):
        return None
    r = native.native_ops.reduce(x, op, dim, keepdim)
    return None if r is NotImplemented else r


__all__ = ["unary", "binary", "reduce"]
