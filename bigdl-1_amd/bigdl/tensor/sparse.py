"""COO sparse tensor (``DL/tensor/SparseTensor.scala:55``, ``SparseTensorBLAS.scala``): 1-based
indices at the API; device storage is a torch sparse COO tensor so ``coomm``-style products run
on the GPU through the native CSR SpMM kernel (``ops/csrc/sparse.hip``)."""
from __future__ import annotations

import torch


class SparseTensor:
    def __init__(self, indices, values, shape):
        idx = torch.as_tensor(indices).long()
        if idx.dim() == 2 and idx.shape[0] != len(shape):
            idx = idx.t()
        self.data = torch.sparse_coo_tensor(idx - 1, torch.as_tensor(values, dtype=torch.float32), tuple(shape)).coalesce()

    @staticmethod
    def from_dense(t: torch.Tensor) -> "SparseTensor":
        s = SparseTensor.__new__(SparseTensor)
        s.data = t.to_sparse().coalesce()
        return s

    def size(self):
        return list(self.data.shape)

    def nElement(self):
        return self.data._nnz()

    def to_dense(self) -> torch.Tensor:
        return self.data.to_dense()

    def mm(self, dense: torch.Tensor) -> torch.Tensor:
        """sparse × dense (``SparseTensorBLAS.coomm``): the native CSR SpMM kernel on a GPU
        (``ops/csrc/sparse.hip``; N % 4 == 0), ``torch.sparse.mm`` otherwise."""
        a = self.data.to(dense.device)
        if dense.is_cuda and dense.dim() == 2 and dense.shape[1] % 4 == 0:
            from ..ops import native as N
            if N.has("spmm"):
                r = N.native_ops.spmm(a, dense)
                if r is not NotImplemented:
                    return r
        return torch.sparse.mm(a, dense.float() if dense.dtype != torch.float64 else dense)

    def mv(self, vec: torch.Tensor) -> torch.Tensor:
        return torch.sparse.mm(self.data.to(vec.device), vec.unsqueeze(1)).squeeze(1)

    def __repr__(self):
        return f"SparseTensor(shape={tuple(self.data.shape)}, nnz={self.data._nnz()})"
