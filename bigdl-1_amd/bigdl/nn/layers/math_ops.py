"""Element / reduction math layers (``DL/nn/{Add,AddConstant,CAdd,CMul,Mul,MulConstant,Power,Sqrt,
Square,Exp,Log,Abs,Negative,Sum,Mean,Max,Min,Scale,Maxout,Highway,GradientReversal,L1Penalty,
ActivityRegularization,NegativeEntropyPenalty}.scala``)."""
from __future__ import annotations

import math

import torch

from ..abstractnn import TensorModule, AutogradModule
from ..initialization_method import RandomUniform
from ...ops import vml
from .shape import _bdim


class Add(AutogradModule):
    """Learnable bias vector (``Add.scala``), init U(±1/√n)."""

    def __init__(self, input_size, bigdl_type="float"):
        super().__init__()
        self.inputSize = input_size
        self.register_parameter("bias", torch.zeros(input_size))
        stdv = 1.0 / math.sqrt(input_size)
        RandomUniform(-stdv, stdv).init(self.bias)

    def _forward(self, x):
        b = self.P("bias").to(x.dtype)
        if x.dim() > 1 and x.shape[-1] != b.numel():
            return x + b.view(x.shape[1:])
        return x + b


class AddConstant(TensorModule):
    def __init__(self, constant_scalar, inplace=False, bigdl_type="float"):
        super().__init__()
        self.constant = constant_scalar
        self.inplace = inplace

    def updateOutput(self, input):
        return input + self.constant

    def updateGradInput(self, input, gradOutput):
        return gradOutput


class CAdd(AutogradModule):
    """Learnable broadcast bias of ``size`` (``CAdd.scala``)."""

    def __init__(self, size, bRegularizer=None, bigdl_type="float"):
        super().__init__()
        self.size = list(size)
        self.register_parameter("bias", torch.zeros(self.size))
        stdv = 1.0 / math.sqrt(int(torch.tensor(self.size).prod()))
        RandomUniform(-stdv, stdv).init(self.bias)
        self.bRegularizer = bRegularizer

    def _forward(self, x):
        b = self.P("bias").to(x.dtype)
        if b.dim() == x.dim() - 1 or (b.numel() == x[0].numel() and x.dim() > b.dim()):
            return x + b.view(x.shape[1:]) if b.numel() == x[0].numel() else x + b
        return x + b


class CMul(AutogradModule):
    def __init__(self, size, wRegularizer=None, bigdl_type="float"):
        super().__init__()
        self.size = list(size)
        self.register_parameter("weight", torch.zeros(self.size))
        stdv = 1.0 / math.sqrt(int(torch.tensor(self.size).prod()))
        RandomUniform(-stdv, stdv).init(self.weight)
        self.wRegularizer = wRegularizer

    def _forward(self, x):
        w = self.P("weight").to(x.dtype)
        if w.numel() == x[0].numel() and x.dim() > w.dim():
            return x * w.view(x.shape[1:])
        return x * w


class Mul(AutogradModule):
    """Single learnable scalar gain."""

    def __init__(self, bigdl_type="float"):
        super().__init__()
        self.register_parameter("weight", torch.zeros(1))
        RandomUniform(-1.0, 1.0).init(self.weight)

    def _forward(self, x):
        return x * self.P("weight").to(x.dtype)


class MulConstant(TensorModule):
    def __init__(self, scalar, inplace=False, bigdl_type="float"):
        super().__init__()
        self.scalar, self.inplace = scalar, inplace

    def updateOutput(self, input):
        return input * self.scalar

    def updateGradInput(self, input, gradOutput):
        return gradOutput * self.scalar


class Power(AutogradModule):
    """(shift + scale·x)^power (``Power.scala``)."""

    def __init__(self, power, scale=1.0, shift=0.0, bigdl_type="float"):
        super().__init__()
        self.power, self.scale, self.shift = power, scale, shift

    def _forward(self, x):
        return torch.pow(self.shift + self.scale * x, self.power)


class _Elementwise(TensorModule):
    """y = f(x) with an explicit gradient: device tensors run the ``ops/csrc/vml.hip`` kernels
    (the reference's VML calls), host tensors the torch formulas.  ``_saved`` names the forward
    value the gradient needs ("output" or "input")."""
    _op = _bwd = None
    _saved = "output"

    def _f(self, x):
        raise NotImplementedError

    def _df(self, x, y, g):
        raise NotImplementedError

    def updateOutput(self, input):
        r = vml.unary(input, self._op)
        return r if r is not None else self._f(input)

    def updateGradInput(self, input, gradOutput):
        r = vml.binary(gradOutput, self.output if self._saved == "output" else input, self._bwd)
        return r if r is not None else self._df(input, self.output, gradOutput)


class Sqrt(_Elementwise):
    _op, _bwd = "sqrt", "sqrt_bwd"

    def _f(self, x):
        return torch.sqrt(x)

    def _df(self, x, y, g):
        return 0.5 * g / y


class Square(_Elementwise):
    _op, _bwd, _saved = "square", "square_bwd", "input"

    def _f(self, x):
        return x * x

    def _df(self, x, y, g):
        return 2.0 * g * x


class Exp(_Elementwise):
    _op, _bwd = "exp", "exp_bwd"

    def _f(self, x):
        return torch.exp(x)

    def _df(self, x, y, g):
        return g * y


class Log(_Elementwise):
    _op, _bwd, _saved = "log", "log_bwd", "input"

    def _f(self, x):
        return torch.log(x)

    def _df(self, x, y, g):
        return g / x


class Abs(_Elementwise):
    _op, _bwd, _saved = "abs", "abs_bwd", "input"

    def _f(self, x):
        return torch.abs(x)

    def _df(self, x, y, g):
        return g * torch.sign(x)


class Negative(AutogradModule):
    def __init__(self, inplace=False, bigdl_type="float"):
        super().__init__()

    def _forward(self, x):
        return -x


class Sum(AutogradModule):
    def __init__(self, dimension=1, n_input_dims=-1, size_average=False, squeeze=True, bigdl_type="float"):
        super().__init__()
        self.dimension, self.nInputDims, self.sizeAverage, self.squeeze = dimension, n_input_dims, size_average, squeeze

    def _forward(self, x):
        d = _bdim(self.dimension, x, self.nInputDims if self.nInputDims > 0 else None)
        y = x.sum(d, keepdim=not self.squeeze)
        if self.sizeAverage:
            y = y / x.shape[d]
        # Sum.scala:82-90: a 1-D input sums to a 1-element tensor, not a 0-d scalar
        return y.reshape(1) if y.dim() == 0 else y


class Mean(Sum):
    def __init__(self, dimension=1, n_input_dims=-1, squeeze=True, bigdl_type="float"):
        super().__init__(dimension, n_input_dims, True, squeeze)


class Max(AutogradModule):
    def __init__(self, dim=1, num_input_dims=-2147483648, bigdl_type="float"):
        super().__init__()
        self.dim, self.numInputDims = dim, (None if num_input_dims == -2147483648 else num_input_dims)

    def _forward(self, x):
        return x.max(_bdim(self.dim, x, self.numInputDims))[0]


class Min(Max):
    def _forward(self, x):
        return x.min(_bdim(self.dim, x, self.numInputDims))[0]


class Scale(AutogradModule):
    """CMul followed by CAdd with the same shape (``Scale.scala``)."""

    def __init__(self, size, bigdl_type="float"):
        super().__init__()
        self.size = list(size)
        self.register_parameter("weight", torch.ones(self.size))
        self.register_parameter("bias", torch.zeros(self.size))

    def _forward(self, x):
        w, b = self.P("weight").to(x.dtype), self.P("bias").to(x.dtype)
        if w.dim() < x.dim():
            shape = [1] * x.dim()
            for i, s in enumerate(self.size):
                shape[i + (1 if x.dim() > len(self.size) else 0)] = s
            w, b = w.view(shape), b.view(shape)
        return x * w + b


class Maxout(AutogradModule):
    """Linear(in, out·k) then max over k pieces (``Maxout.scala``)."""

    def __init__(self, input_size, output_size, maxout_number, with_bias=True, w_regularizer=None,
                 b_regularizer=None, init_weight=None, init_bias=None, bigdl_type="float"):
        super().__init__()
        self.outputSize, self.k = output_size, maxout_number
        self.withBias = with_bias
        self.register_parameter("weight", torch.zeros(output_size * maxout_number, input_size))
        if with_bias:
            self.register_parameter("bias", torch.zeros(output_size * maxout_number))
        stdv = 1.0 / math.sqrt(input_size)
        RandomUniform(-stdv, stdv).init(self.weight)
        if with_bias:
            RandomUniform(-stdv, stdv).init(self.bias)

    def _forward(self, x):
        y = x @ self.P("weight").to(x.dtype).t()
        if self.withBias:
            y = y + self.P("bias").to(x.dtype)
        return y.view(x.shape[0], self.outputSize, self.k).max(-1)[0]


class Highway(AutogradModule):
    """y = t·H(x) + (1−t)·x, t = σ(W_t x + b_t) (``Highway.scala``)."""

    def __init__(self, size, with_bias=True, activation=None, wRegularizer=None, bRegularizer=None,
                 bigdl_type="float"):
        super().__init__()
        self.size, self.withBias, self.activation = size, with_bias, activation
        self.register_parameter("weight", torch.zeros(2 * size, size))
        if with_bias:
            self.register_parameter("bias", torch.zeros(2 * size))
        stdv = 1.0 / math.sqrt(size)
        RandomUniform(-stdv, stdv).init(self.weight)
        if with_bias:
            with torch.no_grad():
                self.bias[:size].fill_(-1.0)  # carry bias (transform gate starts closed)
                self.bias[size:].zero_()

    def _forward(self, x):
        w = self.P("weight").to(x.dtype)
        y = x @ w.t()
        if self.withBias:
            y = y + self.P("bias").to(x.dtype)
        t = torch.sigmoid(y[:, :self.size])
        h = y[:, self.size:]
        if self.activation is not None:
            name = self.activation if isinstance(self.activation, str) else type(self.activation).__name__
            h = {"tanh": torch.tanh, "Tanh": torch.tanh, "relu": torch.relu, "ReLU": torch.relu,
                 "sigmoid": torch.sigmoid, "Sigmoid": torch.sigmoid}.get(name, lambda v: v)(h)
        return t * h + (1 - t) * x


class GradientReversal(TensorModule):
    def __init__(self, the_lambda=1.0, bigdl_type="float"):
        super().__init__()
        self.lam = the_lambda

    def setLambda(self, lam):
        self.lam = lam
        return self

    def updateOutput(self, input):
        return input

    def updateGradInput(self, input, gradOutput):
        return -self.lam * gradOutput


class L1Penalty(TensorModule):
    """Adds an L1 sparsity penalty on activations to the gradient (``L1Penalty.scala``)."""

    def __init__(self, l1weight, size_average=False, provide_output=True, bigdl_type="float"):
        super().__init__()
        self.l1weight, self.sizeAverage, self.provideOutput = l1weight, size_average, provide_output
        self.loss = 0.0

    def updateOutput(self, input):
        m = self.l1weight / input.numel() if self.sizeAverage else self.l1weight
        self.loss = m * float(input.abs().sum())
        return input

    def updateGradInput(self, input, gradOutput):
        m = self.l1weight / input.numel() if self.sizeAverage else self.l1weight
        gi = torch.sign(input) * m
        if self.provideOutput:
            gi = gi + gradOutput
        return gi


class ActivityRegularization(TensorModule):
    def __init__(self, l1, l2, bigdl_type="float"):
        super().__init__()
        self.l1, self.l2 = l1, l2
        self.loss = 0.0

    def updateOutput(self, input):
        self.loss = self.l1 * float(input.abs().sum()) + self.l2 * float((input * input).sum())
        return input

    def updateGradInput(self, input, gradOutput):
        return gradOutput + self.l1 * torch.sign(input) + 2 * self.l2 * input


class NegativeEntropyPenalty(TensorModule):
    """Penalise low entropy of a probability input: loss = β·Σ p log p."""

    def __init__(self, beta=0.01, bigdl_type="float"):
        super().__init__()
        self.beta = beta
        self.loss = 0.0

    def updateOutput(self, input):
        self.loss = self.beta * float((input * torch.log(input.clamp_min(1e-12))).sum())
        return input

    def updateGradInput(self, input, gradOutput):
        return gradOutput + self.beta * (torch.log(input.clamp_min(1e-12)) + 1)
