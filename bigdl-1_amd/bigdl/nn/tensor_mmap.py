"""``TensorMMap`` (``DL/nn/mkldnn/TensorMMap.scala``): a parameter's dense fp32 tensor paired with
its native (kernel-layout) copy.

The reference pairs a heap ``dense`` tensor (what optimizers and serialization see) with a
``DnnTensor`` in the MKL-DNN primitive's blocked layout and a reorder between them.  Here the dense
side is an fp32 tensor (usually a view of the flat master-parameter arena) and the native side is
what a HIP kernel consumes: a device tensor in the compute dtype (bf16) with an optional axis
permutation (e.g. OIHW → OHWI = KRSC for the implicit-GEMM conv).  ``sync()`` reorders dense →
native (the reference's ``_reorder.forward``), ``sync_back()`` native → dense.
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch


class TensorMMap:
    def __init__(self, size: Sequence[int], dense: Optional[torch.Tensor] = None):
        self.dense = dense if dense is not None else torch.zeros(*size, dtype=torch.float32)
        if tuple(self.dense.shape) != tuple(size):
            raise ValueError(f"dense tensor shape {tuple(self.dense.shape)} != {tuple(size)}")
        self._native: Optional[torch.Tensor] = None
        self._perm: Optional[Sequence[int]] = None
        self._dtype = None
        self._device = None

    @property
    def native(self) -> Optional[torch.Tensor]:
        return self._native

    def set_memory_data(self, device=None, dtype=torch.bfloat16, permute: Optional[Sequence[int]] = None):
        """Fix the native format once (``setMemoryData``); allocates the native tensor (zeros) —
        call :meth:`sync` to fill it."""
        if self._native is not None:
            raise RuntimeError("you only can set once the memory data")
        self._device = torch.device(device) if device is not None else self.dense.device
        self._dtype, self._perm = dtype, (tuple(permute) if permute is not None else None)
        shape = [self.dense.shape[i] for i in self._perm] if self._perm else list(self.dense.shape)
        self._native = torch.zeros(shape, dtype=dtype, device=self._device)
        return self

    setMemoryData = set_memory_data

    def sync(self):
        if self._native is None:
            raise RuntimeError("you should initialize the native relevant resources first")
        src = self.dense.permute(*self._perm) if self._perm else self.dense
        self._native.copy_(src, non_blocking=True)

    def sync_back(self):
        if self._native is None:
            raise RuntimeError("you should initialize the native relevant resources first")
        src = self._native
        if self._perm:
            inv = [0] * len(self._perm)
            for i, p in enumerate(self._perm):
                inv[p] = i
            src = src.permute(*inv)
        self.dense.copy_(src)

    def zero(self):
        self.dense.zero_()
        if self._native is not None:
            self._native.zero_()

    def copy(self, t: torch.Tensor):
        self.dense.copy_(t)

    def size(self, index: Optional[int] = None):
        return list(self.dense.shape) if index is None else int(self.dense.shape[index - 1])

    def release(self):
        self._native = None

    def set_native(self, other: "TensorMMap"):
        if self._native is not None and other._native is not None:
            self._native = other._native

    setNative = set_native
