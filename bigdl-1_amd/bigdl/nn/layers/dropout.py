"""Dropout family (``DL/nn/Dropout.scala:64-150``, ``SpatialDropout{1,2,3}D``, ``GaussianDropout``,
``GaussianNoise``).  ``Dropout(initP)`` takes the DROP probability p and scales kept units by
1/(1−p) when ``scale`` is true (SURVEY §2.5 warns that ``Attention`` passes 1−dropout)."""
from __future__ import annotations

import math

import torch

from ... import ops
from ..abstractnn import TensorModule


class Dropout(TensorModule):
    def __init__(self, init_p=0.5, inplace=False, scale=True, bigdl_type="float"):
        super().__init__()
        self.p = init_p
        self.inplace = inplace
        self.scale = scale
        self._mask = None

    def setP(self, p):
        self.p = p
        return self

    def getP(self):
        return self.p

    def updateOutput(self, input):
        if not self.train or self.p <= 0:
            if not self.scale and self.p > 0:
                return input * (1 - self.p)
            return input
        y, mask = ops.dropout_forward(input, self.p)
        if not self.scale:
            y = y * (1 - self.p)
        self._mask = mask
        return y

    def updateGradInput(self, input, gradOutput):
        if not self.train or self.p <= 0:
            return gradOutput * ((1 - self.p) if (not self.scale and self.p > 0) else 1.0)
        g = ops.dropout_backward(gradOutput, self._mask, self.p)
        if not self.scale:
            g = g * (1 - self.p)
        return g


class _SpatialDropout(TensorModule):
    _keep_dims = 2  # mask shape (N, C, 1, 1, ...)

    def __init__(self, init_p=0.5, format="NCHW", bigdl_type="float"):
        super().__init__()
        self.p, self.format = init_p, format
        self._mask = None

    def _mask_shape(self, x):
        raise NotImplementedError

    def updateOutput(self, input):
        if not self.train or self.p <= 0:
            return input
        mshape = self._mask_shape(input)
        self._mask = (torch.rand(mshape, device=input.device) >= self.p).to(input.dtype) / (1 - self.p)
        return input * self._mask

    def updateGradInput(self, input, gradOutput):
        if not self.train or self.p <= 0:
            return gradOutput
        return gradOutput * self._mask


class SpatialDropout1D(_SpatialDropout):
    """Drops whole feature channels of (N, T, C) input."""

    def __init__(self, init_p=0.5, bigdl_type="float"):
        super().__init__(init_p)

    def _mask_shape(self, x):
        return (x.shape[0], 1, x.shape[2]) if x.dim() == 3 else (1, x.shape[1])


class SpatialDropout2D(_SpatialDropout):
    def _mask_shape(self, x):
        if self.format == "NCHW":
            return (x.shape[0], x.shape[1], 1, 1) if x.dim() == 4 else (x.shape[0], 1, 1)
        return (x.shape[0], 1, 1, x.shape[3]) if x.dim() == 4 else (1, 1, x.shape[2])


class SpatialDropout3D(_SpatialDropout):
    def _mask_shape(self, x):
        if self.format == "NCHW":
            return (x.shape[0], x.shape[1], 1, 1, 1) if x.dim() == 5 else (x.shape[0], 1, 1, 1)
        return (x.shape[0], 1, 1, 1, x.shape[4]) if x.dim() == 5 else (1, 1, 1, x.shape[3])


class GaussianDropout(TensorModule):
    """Multiplicative N(1, p/(1−p)) noise in training (``GaussianDropout.scala``)."""

    def __init__(self, rate, bigdl_type="float"):
        super().__init__()
        self.rate = rate
        self._noise = None

    def updateOutput(self, input):
        if not self.train:
            return input
        std = math.sqrt(self.rate / (1 - self.rate))
        self._noise = torch.randn_like(input) * std + 1
        return input * self._noise

    def updateGradInput(self, input, gradOutput):
        return gradOutput * self._noise if self.train else gradOutput


class GaussianNoise(TensorModule):
    def __init__(self, stddev, bigdl_type="float"):
        super().__init__()
        self.stddev = stddev

    def updateOutput(self, input):
        if not self.train:
            return input
        return input + torch.randn_like(input) * self.stddev

    def updateGradInput(self, input, gradOutput):
        return gradOutput
