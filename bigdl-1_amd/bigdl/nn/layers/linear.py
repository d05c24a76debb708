"""Linear / matmul family.

``Linear`` — ``DL/nn/Linear.scala`` (weight (out, in), y = x·Wᵀ + b at :108-109, backward at
:128-158, default init U(±1/√in) at :68-71).  On device the three products run on MFMA GEMM
kernels with the bias add / bias-gradient reduction fused.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from ... import ops
from ..abstractnn import TensorModule, AutogradModule
from ..initialization_method import RandomUniform, Zeros, VariableFormats
from ...utils.table import Table
from ...utils import acc_float


class Linear(TensorModule):
    def __init__(self, input_size, output_size, with_bias=True, wRegularizer=None, bRegularizer=None,
                 init_weight=None, init_bias=None, init_grad_weight=None, init_grad_bias=None, bigdl_type="float"):
        super().__init__()
        self.inputSize, self.outputSize, self.withBias = input_size, output_size, with_bias
        self.wRegularizer, self.bRegularizer = wRegularizer, bRegularizer
        self.register_parameter("weight", torch.zeros(output_size, input_size) if init_weight is None else
                                torch.as_tensor(init_weight, dtype=torch.float32).reshape(output_size, input_size))
        if with_bias:
            self.register_parameter("bias", torch.zeros(output_size) if init_bias is None else
                                    torch.as_tensor(init_bias, dtype=torch.float32).reshape(output_size))
        else:
            self.bias = self.gradBias = None
        self._has_init_w, self._has_init_b = init_weight is not None, init_bias is not None
        stdv = 1.0 / math.sqrt(input_size)
        self._init_weight_method = RandomUniform(-stdv, stdv)
        self._init_bias_method = RandomUniform(-stdv, stdv)
        self.reset()

    def reset(self):
        if not self._has_init_w:
            self._init_weight_method.init(self.weight, VariableFormats.OUT_IN)
        if self.withBias and not self._has_init_b:
            self._init_bias_method.init(self.bias, VariableFormats.ONE_D)
        self.zeroGradParameters()
        return self

    def _x2(self, input):
        if input.dim() == 1:
            return input.unsqueeze(0)
        if input.dim() > 2:
            return input.reshape(-1, input.shape[-1])
        return input

    def updateOutput(self, input):
        if input.shape[-1] != self.inputSize:
            raise ValueError(f"Linear: input size {input.shape[-1]} != {self.inputSize}")
        x = self._x2(input)
        if x.is_cuda:
            from ...utils.engine import Engine
            dt = Engine.compute_dtype()
            if x.dtype != dt and x.is_floating_point():
                x = x.to(dt)
            x = x.contiguous()
        # device: the fp32 master bias goes straight into the GEMM epilogue (no per-call cast)
        b = (self.bias if x.is_cuda else self.cw("bias")) if self.withBias else None
        y = ops.linear_forward(x, self.cw("weight"), b)
        if input.dim() == 1:
            return y.squeeze(0)
        if input.dim() > 2:
            return y.reshape(*input.shape[:-1], self.outputSize)
        return y

    def _bwd(self, input, gradOutput, need_input, acc):
        x = self._x2(input)
        gy = self._x2(gradOutput)
        if x.is_cuda:
            from ...utils.engine import Engine
            dt = Engine.compute_dtype()
            x = x.to(dt).contiguous()
            gy = gy.to(dt).contiguous()
        same = self.scale_w == self.scale_b
        gi = ops.linear_backward(gy, x, self.cw("weight"), need_input,
                                 self.gradWeight if acc else None,
                                 self.gradBias if (acc and self.withBias and same) else None,
                                 self.scale_w if acc else 0.0)
        if acc and self.withBias and not same and self.scale_b != 0:
            self.gradBias.add_(acc_float(gy).sum(0), alpha=self.scale_b)
        if acc and self.wRegularizer is not None and self.scale_w != 0:
            self.wRegularizer.accRegularization(self.weight, self.gradWeight, self.scale_w)
        if acc and self.withBias and self.bRegularizer is not None and self.scale_b != 0:
            self.bRegularizer.accRegularization(self.bias, self.gradBias, self.scale_b)
        if gi is not None:
            gi = gi.reshape(input.shape)
        return gi

    def updateGradInput(self, input, gradOutput):
        gi = self._bwd(input, gradOutput, True, True)
        self._gi_done = True
        return gi

    def accGradParameters(self, input, gradOutput):
        if not getattr(self, "_gi_done", False):
            self._bwd(input, gradOutput, False, True)
        self._gi_done = False

    def __repr__(self):
        return f"Linear[{self.get_name()}]({self.inputSize} -> {self.outputSize})"


class SparseLinear(Linear):
    """Linear over a sparse (COO) input (``SparseLinear.scala``); accepts dense too."""

    def __init__(self, input_size, output_size, with_bias=True, backwardStart=-1, backwardLength=-1,
                 wRegularizer=None, bRegularizer=None, init_weight=None, init_bias=None, init_grad_weight=None,
                 init_grad_bias=None, bigdl_type="float"):
        super().__init__(input_size, output_size, with_bias, wRegularizer, bRegularizer, init_weight, init_bias)
        self.backwardStart, self.backwardLength = backwardStart, backwardLength

    @staticmethod
    def _spmm(a, b):
        """sparse × dense: the native CSR SpMM kernel on a GPU (ops/csrc/sparse.hip), torch.sparse
        on the host."""
        if a.is_cuda:
            from ...ops import native as N
            if N.has("spmm"):
                r = N.native_ops.spmm(a, b.contiguous())
                if r is not NotImplemented:
                    return r
                N.note_fallback("spmm", "shape", (b,))
        return torch.sparse.mm(acc_float(a), b)

    def updateOutput(self, input):
        if input.is_sparse:
            y = self._spmm(input, acc_float(self.weight).t())
            if self.withBias:
                y = y + self.bias
            return y
        return super().updateOutput(input)

    def _bwd(self, input, gradOutput, need_input, acc):
        if input.is_sparse:
            if acc:
                # dW = Gᵀ·X, formed as (Xᵀ·G)ᵀ so the sparse operand stays on the left
                self.gradWeight.add_(self._spmm(input.t().coalesce(), acc_float(gradOutput)).t(), alpha=self.scale_w)
                if self.withBias:
                    self.gradBias.add_(acc_float(gradOutput).sum(0), alpha=self.scale_b)
            if need_input and self.backwardStart > 0:
                g = acc_float(gradOutput) @ self.weight
                return g[:, self.backwardStart - 1:self.backwardStart - 1 + self.backwardLength]
            return None
        return super()._bwd(input, gradOutput, need_input, acc)


class Bilinear(AutogradModule):
    """y_k = x1ᵀ W_k x2 + b_k (``Bilinear.scala``); input Table(x1, x2)."""

    def __init__(self, input_size1, input_size2, output_size, bias_res=True, wRegularizer=None, bRegularizer=None,
                 bigdl_type="float"):
        super().__init__()
        self.register_parameter("weight", torch.zeros(output_size, input_size1, input_size2))
        self.biasRes = bias_res
        if bias_res:
            self.register_parameter("bias", torch.zeros(output_size))
        stdv = 1.0 / math.sqrt(input_size1)
        RandomUniform(-stdv, stdv).init(self.weight)
        if bias_res:
            RandomUniform(-stdv, stdv).init(self.bias)

    def _forward(self, x):
        return F.bilinear(x[1], x[2], self.P("weight").to(x[1].dtype),
                          self.P("bias").to(x[1].dtype) if self.biasRes else None)


class MM(AutogradModule):
    """Batched/unbatched matrix product of a Table(A, B) with optional transposes (``MM.scala``)."""

    def __init__(self, trans_a=False, trans_b=False, bigdl_type="float"):
        super().__init__()
        self.transA, self.transB = trans_a, trans_b

    def _forward(self, x):
        a, b = x[1], x[2]
        if self.transA:
            a = a.transpose(-1, -2)
        if self.transB:
            b = b.transpose(-1, -2)
        return torch.matmul(a, b)


class MV(AutogradModule):
    def __init__(self, trans=False, bigdl_type="float"):
        super().__init__()
        self.trans = trans

    def _forward(self, x):
        m, v = x[1], x[2]
        if self.trans:
            m = m.transpose(-1, -2)
        return torch.matmul(m, v.unsqueeze(-1)).squeeze(-1)


class Cosine(AutogradModule):
    """Cosine similarity of the input with each of outputSize weight rows (``Cosine.scala``)."""

    def __init__(self, input_size, output_size, bigdl_type="float"):
        super().__init__()
        self.register_parameter("weight", torch.zeros(output_size, input_size))
        stdv = 1.0 / math.sqrt(input_size)
        RandomUniform(-stdv, stdv).init(self.weight)

    def _forward(self, x):
        w = self.P("weight").to(x.dtype)
        xn = x / (x.norm(dim=-1, keepdim=True) + 1e-12)
        wn = w / (w.norm(dim=-1, keepdim=True) + 1e-12)
        return xn @ wn.t()


class Euclidean(AutogradModule):
    """‖x − w_j‖ for each weight column j (``Euclidean.scala``); weight (in, out)."""

    def __init__(self, input_size, output_size, fast_backward=True, bigdl_type="float"):
        super().__init__()
        self.register_parameter("weight", torch.zeros(input_size, output_size))
        stdv = 1.0 / math.sqrt(input_size)
        RandomUniform(-stdv, stdv).init(self.weight)

    def _forward(self, x):
        w = self.P("weight").to(x.dtype)
        batched = x.dim() == 2
        xx = x if batched else x.unsqueeze(0)
        d = torch.sqrt(((xx.unsqueeze(2) - w.unsqueeze(0)) ** 2).sum(1) + 1e-12)
        return d if batched else d.squeeze(0)


class DotProduct(AutogradModule):
    def _forward(self, x):
        return (x[1] * x[2]).sum(-1)


class CosineDistance(AutogradModule):
    def _forward(self, x):
        return F.cosine_similarity(x[1], x[2], dim=-1, eps=1e-12)


class PairwiseDistance(AutogradModule):
    def __init__(self, norm=2, bigdl_type="float"):
        super().__init__()
        self.norm = norm

    def _forward(self, x):
        return torch.norm(x[1] - x[2], p=self.norm, dim=-1)


class CrossProduct(AutogradModule):
    """Pairwise dot products between all entries of the input Table (``CrossProduct.scala``)."""

    def __init__(self, num_tensor=0, embedding_size=0, bigdl_type="float"):
        super().__init__()

    def _forward(self, x):
        ts = list(x)
        outs = []
        for i in range(len(ts)):
            for j in range(i + 1, len(ts)):
                outs.append((ts[i] * ts[j]).sum(-1, keepdim=True))
        return torch.cat(outs, dim=-1)


class Gemm(AutogradModule):
    """ONNX Gemm: α·op(A)·op(B) + β·C (``DL/nn/onnx/Gemm.scala``)."""

    def __init__(self, alpha=1.0, beta=1.0, trans_a=False, trans_b=False, bigdl_type="float"):
        super().__init__()
        self.alpha, self.beta, self.transA, self.transB = alpha, beta, trans_a, trans_b

    def _forward(self, x):
        a, b, c = x[1], x[2], x[3]
        if self.transA:
            a = a.t()
        if self.transB:
            b = b.t()
        return self.alpha * (a @ b) + self.beta * c
