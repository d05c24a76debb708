"""Activation and softmax layers.

Hot: ``ReLU`` (= ``Threshold(0, 0, ip)``, ``DL/nn/ReLU.scala:33-35``), ``Threshold``
(``Threshold.scala:46-421``), ``Tanh``, ``Sigmoid``, ``LogSoftMax`` (``LogSoftMax.scala:49-130``),
``SoftMax``.  When a fusion pass folds a ReLU into the preceding BN/conv epilogue the layer is
marked pass-through (forward/backward become identities), like ``bigdl.mkldnn.fusion.bnrelu``.
The remaining activations are defined by their forward (gradient by AD).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ... import ops
from ...ops import vml
from ..abstractnn import TensorModule, AutogradModule
from ...utils import acc_float


class Threshold(TensorModule):
    def __init__(self, th=1e-6, v=0.0, ip=False, bigdl_type="float"):
        super().__init__()
        self.threshold, self.value, self.inPlace = th, v, ip
        self._passthrough = False

    def updateOutput(self, input):
        if self._passthrough:
            return input
        if input.dtype == torch.int8 and getattr(input, "_qscale", None) is not None:
            # an int8 activation of a quantised chain (its producer usually applied this ReLU already)
            if self.threshold == 0.0 and self.value == 0.0:
                # the unsigned (offset) code is non-negative by construction; the signed one clamps
                fused = getattr(self, "_i8_fused", False) or getattr(input, "_qzero", 0)
                y = input if fused else input.clamp_min(0)
                y._qscale = input._qscale
                y._qzero = getattr(input, "_qzero", 0)
                return y
            from ..quantized.layers import dequant
            input = dequant(input)
        # ``ip`` is a memory hint in the reference; out-of-place costs the same HBM traffic and
        # never aliases an activation a predecessor's backward still needs
        return ops.relu_forward(input, self.threshold, self.value, inplace=False)

    def updateGradInput(self, input, gradOutput):
        if self._passthrough == "mask":
            # the producer applied this ReLU in its epilogue: input is already ReLU(x), and
            # ReLU(x) > 0 ⇔ x > 0, so the mask comes from it
            return ops.relu_backward(gradOutput, input, 0.0)
        if self._passthrough:
            return gradOutput
        ref = self.output if self.value <= self.threshold else input
        return ops.relu_backward(gradOutput, ref, self.threshold)


class ReLU(Threshold):
    def __init__(self, ip=False, bigdl_type="float"):
        super().__init__(0.0, 0.0, ip)


class Tanh(TensorModule):
    """``Tanh.scala`` (VML vsTanh); device tensors run the vml.hip kernels forward and backward."""

    def updateOutput(self, input):
        r = vml.unary(input, "tanh")
        return r if r is not None else torch.tanh(input)

    def updateGradInput(self, input, gradOutput):
        y = self.output
        r = vml.binary(gradOutput, y, "tanh_bwd")
        return r if r is not None else gradOutput * (1 - y * y)


class Sigmoid(TensorModule):
    def updateOutput(self, input):
        r = vml.unary(input, "sigmoid")
        return r if r is not None else torch.sigmoid(input)

    def updateGradInput(self, input, gradOutput):
        y = self.output
        r = vml.binary(gradOutput, y, "sigmoid_bwd")
        return r if r is not None else gradOutput * y * (1 - y)


class LogSoftMax(TensorModule):
    def updateOutput(self, input):
        return ops.log_softmax_forward(input)

    def updateGradInput(self, input, gradOutput):
        return ops.log_softmax_backward(gradOutput, self.output)


class SoftMax(TensorModule):
    def __init__(self, pos=1, bigdl_type="float"):
        super().__init__()
        self.pos = pos

    def _dim(self, x):
        # reference: 1-D/2-D over the last dim, 3-D/4-D over the channel dim (dim 1 batched)
        if x.dim() <= 2:
            return -1
        return 1 if x.dim() == 4 else 0 if x.dim() == 3 and self.pos == 1 else -1

    def updateOutput(self, input):
        d = self._dim(input)
        if d == -1:
            return ops.softmax_forward(input)
        if d == 1 and input.is_cuda and ops.native_has("softmax_forward"):
            # NHWC device layout: the channel softmax is a row softmax over contiguous channels
            r = ops.native_ops.softmax_channels_nhwc(input)
            if r is not NotImplemented:
                return r
            ops.native.note_fallback("softmax_forward.channels", "layout", (input,))
        return torch.softmax(acc_float(input), dim=d).to(input.dtype)

    def updateGradInput(self, input, gradOutput):
        d = self._dim(input)
        y = self.output
        if d == -1:
            return ops.softmax_backward(gradOutput, y)
        if d == 1 and y.is_cuda and ops.native_has("softmax_backward"):
            r = ops.native_ops.softmax_channels_nhwc(y, backward_gy=gradOutput)
            if r is not NotImplemented:
                return r
            ops.native.note_fallback("softmax_backward.channels", "layout", (y,))
        return (y * (gradOutput - (gradOutput * y).sum(d, keepdim=True))).to(y.dtype)


class SoftMin(AutogradModule):
    def _forward(self, x):
        return torch.softmax(-x, dim=-1 if x.dim() <= 2 else 1)


class ReLU6(AutogradModule):
    def __init__(self, inplace=False, bigdl_type="float"):
        super().__init__()
        self.inplace = inplace

    def _forward(self, x):
        return torch.clamp(x, 0, 6)


class HardTanh(AutogradModule):
    def __init__(self, min_value=-1.0, max_value=1.0, inplace=False, bigdl_type="float"):
        super().__init__()
        self.minValue, self.maxValue = min_value, max_value

    def _forward(self, x):
        return torch.clamp(x, self.minValue, self.maxValue)


class Clamp(HardTanh):
    def __init__(self, min, max, bigdl_type="float"):  # noqa: A002
        super().__init__(min, max)


class HardSigmoid(AutogradModule):
    """max(0, min(1, 0.2x + 0.5)) (``HardSigmoid.scala``)."""

    def _forward(self, x):
        return torch.clamp(0.2 * x + 0.5, 0, 1)


class LeakyReLU(AutogradModule):
    def __init__(self, negval=0.01, inplace=False, bigdl_type="float"):
        super().__init__()
        self.negval = negval

    def _forward(self, x):
        return F.leaky_relu(x, self.negval)


class ELU(AutogradModule):
    def __init__(self, alpha=1.0, inplace=False, bigdl_type="float"):
        super().__init__()
        self.alpha = alpha

    def _forward(self, x):
        return F.elu(x, self.alpha)


class PReLU(AutogradModule):
    """Learnable leak per channel (``PReLU.scala``); nOutputPlane = 0 → single shared weight, init 0.25."""

    def __init__(self, n_output_plane=0, bigdl_type="float"):
        super().__init__()
        self.nOutputPlane = n_output_plane
        self.register_parameter("weight", torch.full((max(1, n_output_plane),), 0.25))

    def _forward(self, x):
        w = self.P("weight").to(x.dtype)
        if self.nOutputPlane == 0:
            return torch.where(x > 0, x, x * w[0])
        shape = [1] * x.dim()
        cdim = 1 if x.dim() in (2, 4) else 0
        shape[cdim] = self.nOutputPlane
        return torch.where(x > 0, x, x * w.view(shape))


class RReLU(AutogradModule):
    """Randomised leaky ReLU (``RReLU.scala``): slope ~ U(lower, upper) in training, mean in eval."""

    def __init__(self, lower=1.0 / 8, upper=1.0 / 3, inplace=False, bigdl_type="float"):
        super().__init__()
        self.lower, self.upper = lower, upper

    def _forward(self, x):
        if self.train:
            a = torch.empty_like(x).uniform_(self.lower, self.upper)
        else:
            a = torch.full_like(x, (self.lower + self.upper) / 2)
        return torch.where(x >= 0, x, x * a)


class SReLU(AutogradModule):
    """S-shaped ReLU with learnable (tl, al, tr, ar) per feature (``SReLU.scala``)."""

    def __init__(self, shape, share_axes=None, bigdl_type="float"):
        super().__init__()
        shape = list(shape)
        if share_axes:
            for a in share_axes:
                shape[a - 1] = 1
        self.register_parameter("tLeft", torch.zeros(shape), "gradTLeft")
        self.register_parameter("aLeft", torch.zeros(shape), "gradALeft")
        self.register_parameter("tRight", torch.zeros(shape), "gradTRight")
        self.register_parameter("aRight", torch.ones(shape), "gradARight")
        with torch.no_grad():
            self.tRight.uniform_(0, 1)

    def _forward(self, x):
        tl, al, tr, ar = (self.P(n).to(x.dtype) for n in ("tLeft", "aLeft", "tRight", "aRight"))
        y = torch.where(x >= tr, tr + ar * (x - tr), x)
        return torch.where(x <= tl, tl + al * (x - tl), y)


class SoftPlus(AutogradModule):
    def __init__(self, beta=1.0, bigdl_type="float"):
        super().__init__()
        self.beta = beta

    def _forward(self, x):
        return F.softplus(x, self.beta)


class SoftSign(AutogradModule):
    def _forward(self, x):
        return x / (1 + x.abs())


class SoftShrink(AutogradModule):
    def __init__(self, the_lambda=0.5, bigdl_type="float"):
        super().__init__()
        self.lam = the_lambda

    def _forward(self, x):
        return F.softshrink(x, self.lam)


class HardShrink(AutogradModule):
    def __init__(self, the_lambda=0.5, bigdl_type="float"):
        super().__init__()
        self.lam = the_lambda

    def _forward(self, x):
        return torch.where(x.abs() > self.lam, x, torch.zeros_like(x))


class TanhShrink(AutogradModule):
    def _forward(self, x):
        return x - torch.tanh(x)


class LogSigmoid(AutogradModule):
    def _forward(self, x):
        return F.logsigmoid(x)


class BinaryThreshold(TensorModule):
    """y = x > th ? 1 : 0; zero gradient (``BinaryThreshold.scala``)."""

    def __init__(self, th=1e-6, ip=False, bigdl_type="float"):
        super().__init__()
        self.th = th

    def updateOutput(self, input):
        return (input > self.th).to(input.dtype)

    def updateGradInput(self, input, gradOutput):
        return torch.zeros_like(input)


class GaussianSampler(AutogradModule):
    """VAE reparameterisation: input Table(mean, logvar) → mean + exp(logvar/2)·ε."""

    def _forward(self, x):
        mean, logvar = x[1], x[2]
        eps = torch.randn_like(mean)
        return mean + torch.exp(0.5 * logvar) * eps
