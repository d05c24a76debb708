"""Flat element storage behind a :class:`~bigdl.tensor.Tensor` (``DL/tensor/Storage.scala``,
``ArrayStorage.scala:28-80``).  Wraps a 1-D torch view over the tensor's whole storage (host or
HBM) — never a copy — so writes through it are seen by every tensor sharing that storage.  Element
indices are 0-based like the reference's ``ArrayStorage.apply``; ``fill`` / ``copy`` offsets are
1-based like theirs."""
from __future__ import annotations

import torch


class Storage:
    __slots__ = ("data",)

    def __init__(self, data):
        if isinstance(data, Storage):
            data = data.data
        if not isinstance(data, torch.Tensor):
            data = torch.as_tensor(data)
        self.data = data.reshape(-1) if data.dim() != 1 else data

    @staticmethod
    def of(t: torch.Tensor) -> "Storage":
        """The whole storage under ``t`` as a flat typed view."""
        flat = torch.empty(0, dtype=t.dtype, device=t.device)
        flat.set_(t.untyped_storage(), 0, (t.untyped_storage().nbytes() // t.element_size(),), (1,))
        return Storage(flat)

    def length(self) -> int:
        return self.data.numel()

    size = length
    __len__ = length

    def apply(self, index: int):
        return self.data[index].item()

    __getitem__ = apply

    def update(self, index: int, value):
        self.data[index] = value

    __setitem__ = update

    def array(self) -> torch.Tensor:
        return self.data

    def __iter__(self):
        return iter(self.data.tolist())

    def copy(self, source, offset: int = 1, source_offset: int = 1, length: int | None = None) -> "Storage":
        src = source.data if isinstance(source, Storage) else torch.as_tensor(source).reshape(-1)
        n = src.numel() - (source_offset - 1) if length is None else length
        self.data[offset - 1:offset - 1 + n].copy_(src[source_offset - 1:source_offset - 1 + n])
        return self

    def fill(self, value, offset: int = 1, length: int | None = None) -> "Storage":
        n = self.length() - (offset - 1) if length is None else length
        self.data[offset - 1:offset - 1 + n].fill_(value)
        return self

    def resize(self, size: int) -> "Storage":
        new = torch.zeros(int(size), dtype=self.data.dtype, device=self.data.device)
        n = min(int(size), self.length())
        new[:n].copy_(self.data[:n])
        self.data = new
        return self

    def set(self, other: "Storage") -> "Storage":
        self.data = other.data
        return self

    def __repr__(self):
        return f"Storage({self.data.tolist()!r})"
