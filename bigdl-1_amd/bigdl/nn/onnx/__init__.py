"""ONNX-semantics layers (``DL/nn/onnx/{Gemm,Reshape,Shape}.scala``)."""
from __future__ import annotations

import torch

from ...utils.table import Table
from ..abstractnn import AutogradModule, TensorModule


class Gemm(AutogradModule):
    """``Y = alpha·op(A)·op(B) + beta·C`` (``nn/onnx/Gemm.scala``).  With ``matrix_b``/``matrix_c``
    given the layer takes A only; otherwise a Table(A, B, C)."""

    def __init__(self, alpha=1.0, beta=1.0, trans_a=False, trans_b=False, matrix_b=None, matrix_c=None):
        super().__init__()
        self.alpha, self.beta, self.transA, self.transB = float(alpha), float(beta), bool(trans_a), bool(trans_b)
        self.matrixB = None if matrix_b is None else torch.as_tensor(matrix_b, dtype=torch.float32)
        self.matrixC = None if matrix_c is None else torch.as_tensor(matrix_c, dtype=torch.float32)

    def _forward(self, x):
        if isinstance(x, Table):
            a, b, c = x[1], x[2], x[3] if len(x) > 2 else None
        else:
            a, b, c = x, self.matrixB.to(x.device, x.dtype), (None if self.matrixC is None else
                                                               self.matrixC.to(x.device, x.dtype))
        a = a.t() if self.transA else a
        b = b.t() if self.transB else b
        y = self.alpha * (a @ b)
        return y if c is None else y + self.beta * c


class Reshape(TensorModule):
    """ONNX Reshape: ``0`` copies the input dim, ``-1`` is inferred (``nn/onnx/Reshape.scala``)."""

    def __init__(self, shape=None):
        super().__init__()
        self.shape = None if shape is None else [int(s) for s in shape]

    def _target(self, x, shape):
        return [x.shape[i] if s == 0 else s for i, s in enumerate(shape)]

    def updateOutput(self, input):
        if isinstance(input, Table):
            x, shape = input[1], [int(v) for v in input[2].flatten().tolist()]
        else:
            x, shape = input, self.shape
        return x.reshape(self._target(x, shape))

    def updateGradInput(self, input, gradOutput):
        x = input[1] if isinstance(input, Table) else input
        g = gradOutput.reshape(x.shape)
        return Table(g, torch.zeros(0)) if isinstance(input, Table) else g


class Shape(TensorModule):
    def updateOutput(self, x):
        return torch.tensor(list(x.shape), dtype=torch.int64)

    def updateGradInput(self, input, gradOutput):
        return torch.zeros_like(input)
