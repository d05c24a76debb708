"""Sparse-activation layers: ``DenseToSparse`` (``DL/nn/DenseToSparse.scala``) and
``SparseJoinTable`` (``DL/nn/SparseJoinTable.scala``).  Sparse activations are torch COO tensors
(device-resident; ``SparseLinear`` consumes them through hipSPARSE SpMM)."""
from __future__ import annotations

import torch

from ..abstractnn import AbstractModule, TensorModule
from ...utils.table import Table


class DenseToSparse(TensorModule):
    """Dense → COO sparse; backward densifies the gradient when ``propagate_back``."""

    def __init__(self, propagate_back: bool = True, bigdl_type="float"):
        super().__init__()
        self.propagateBack = propagate_back

    def updateOutput(self, input):
        if input.is_sparse:
            raise ValueError("DenseToSparse: input should be a dense tensor")
        return input.to_sparse().coalesce()

    def updateGradInput(self, input, gradOutput):
        if not self.propagateBack:
            return None
        g = gradOutput.to_dense() if gradOutput.is_sparse else gradOutput
        return g.reshape(input.shape).to(input.dtype)

    def __repr__(self):
        return "DenseToSparse()"


class SparseJoinTable(AbstractModule):
    """Concatenate COO sparse tensors along ``dimension`` (1-based).  The gradient of input ``i``
    is its slice of ``gradOutput`` (the reference hands every input the whole gradOutput, which is
    only well-formed for a single input)."""

    def __init__(self, dimension: int, bigdl_type="float"):
        super().__init__()
        self.dimension = dimension

    def updateOutput(self, input: Table):
        parts = [t if t.is_sparse else t.to_sparse() for t in input.values()]
        d = self.dimension - 1
        idx, vals, off = [], [], 0
        shape = list(parts[0].shape)
        for p in parts:
            p = p.coalesce()
            i = p.indices().clone()
            i[d] += off
            idx.append(i)
            vals.append(p.values())
            off += p.shape[d]
        shape[d] = off
        self._sizes = [p.shape[d] for p in parts]
        return torch.sparse_coo_tensor(torch.cat(idx, 1), torch.cat(vals), shape).coalesce()

    def updateGradInput(self, input, gradOutput):
        g = gradOutput.to_dense() if gradOutput.is_sparse else gradOutput
        out, off = Table(), 0
        for i, n in enumerate(self._sizes, start=1):
            out[i] = g.narrow(self.dimension - 1, off, n)
            off += n
        return out

    def __repr__(self):
        return f"nn.SparseJoinTable({self.dimension})"
