"""Weight initialisers and fan-in/fan-out formats (``DL/nn/InitializationMethod.scala:38-362``)."""
from __future__ import annotations

import math

import numpy as np
import torch

from ..utils.random import RNG


class VariableFormat:
    def fan_in(self, shape):
        raise ValueError("FanIn is not defined in this format")

    def fan_out(self, shape):
        raise ValueError("FanOut is not defined in this format")


class _Default(VariableFormat):
    def fan_in(self, s):
        return int(np.prod(s))

    def fan_out(self, s):
        return int(np.prod(s))


class _OneD(VariableFormat):
    def fan_in(self, s):
        return s[0]

    def fan_out(self, s):
        return 1


class _InOut(VariableFormat):
    def fan_in(self, s):
        return s[0]

    def fan_out(self, s):
        return s[1]


class _OutIn(VariableFormat):
    def fan_in(self, s):
        return s[1]

    def fan_out(self, s):
        return s[0]


class _InOutKwKh(VariableFormat):
    def fan_in(self, s):
        return s[0] * s[2] * s[3]

    def fan_out(self, s):
        return s[1] * s[2] * s[3]


class _OutInKwKh(VariableFormat):
    def fan_in(self, s):
        return s[1] * s[2] * s[3]

    def fan_out(self, s):
        return s[0] * s[2] * s[3]


class _GpOutInKwKh(VariableFormat):
    def fan_in(self, s):
        return s[2] * s[0] * s[3] * s[4]

    def fan_out(self, s):
        return s[1] * s[0] * s[3] * s[4]


class _GpInOutKwKh(VariableFormat):
    def fan_in(self, s):
        return s[1] * s[0] * s[3] * s[4]

    def fan_out(self, s):
        return s[2] * s[0] * s[3] * s[4]


class _OutInKtKhKw(VariableFormat):
    def fan_in(self, s):
        return s[1] * s[2] * s[3] * s[4]

    def fan_out(self, s):
        return s[0] * s[2] * s[3] * s[4]


class _GpKhKwInOut(VariableFormat):
    def fan_in(self, s):
        return s[2] * s[0] * s[1] * s[2]

    def fan_out(self, s):
        return s[3] * s[0] * s[1] * s[2]


class VariableFormats:
    Default = _Default()
    ONE_D = _OneD()
    IN_OUT = _InOut()
    OUT_IN = _OutIn()
    IN_OUT_KW_KH = _InOutKwKh()
    OUT_IN_KW_KH = _OutInKwKh()
    GP_OUT_IN_KW_KH = _GpOutInKwKh()
    GP_IN_OUT_KW_KH = _GpInOutKwKh()
    OUT_IN_KT_KH_KW = _OutInKtKhKw()
    GP_KH_KW_IN_OUT = _GpKhKwInOut()


def _fill(variable: torch.Tensor, host: torch.Tensor):
    with torch.no_grad():
        variable.copy_(host.to(variable.device, variable.dtype).reshape(variable.shape))


class InitializationMethod:
    SCALA_PACKAGE = "com.intel.analytics.bigdl.nn"

    def init(self, variable: torch.Tensor, fmt: VariableFormat = VariableFormats.Default):
        raise NotImplementedError

    def __repr__(self):
        return type(self).__name__


class RandomUniform(InitializationMethod):
    """No args: U(-1/√fanIn, 1/√fanIn); with (lower, upper): U(lower, upper)."""

    def __init__(self, lower=None, upper=None):
        self.lower = lower
        self.upper = upper

    def init(self, variable, fmt=VariableFormats.Default):
        if self.lower is None:
            stdv = 1.0 / math.sqrt(fmt.fan_in(list(variable.shape)))
            lo, hi = -stdv, stdv
        else:
            lo, hi = self.lower, self.upper
        _fill(variable, RNG.uniform_tensor(tuple(variable.shape), lo, hi))


class RandomNormal(InitializationMethod):
    def __init__(self, mean=0.0, stdv=1.0):
        self.mean = mean
        self.stdv = stdv

    def init(self, variable, fmt=VariableFormats.Default):
        _fill(variable, RNG.normal_tensor(tuple(variable.shape), self.mean, self.stdv))


class Zeros(InitializationMethod):
    def init(self, variable, fmt=VariableFormats.Default):
        with torch.no_grad():
            variable.zero_()


class Ones(InitializationMethod):
    def init(self, variable, fmt=VariableFormats.Default):
        with torch.no_grad():
            variable.fill_(1.0)


class ConstInitMethod(InitializationMethod):
    def __init__(self, value: float):
        self.value = value

    def init(self, variable, fmt=VariableFormats.Default):
        with torch.no_grad():
            variable.fill_(self.value)


class Xavier(InitializationMethod):
    def __init__(self, variance_norm_average: bool = True):
        self.varianceNormAverage = variance_norm_average

    def init(self, variable, fmt=VariableFormats.Default):
        s = list(variable.shape)
        fi, fo = fmt.fan_in(s), fmt.fan_out(s)
        stdv = math.sqrt(3.0 / fi) if not self.varianceNormAverage else math.sqrt(6.0 / (fi + fo))
        _fill(variable, RNG.uniform_tensor(tuple(variable.shape), -stdv, stdv))


class MsraFiller(InitializationMethod):
    def __init__(self, variance_norm_average: bool = True):
        self.varianceNormAverage = variance_norm_average

    def init(self, variable, fmt=VariableFormats.Default):
        s = list(variable.shape)
        fi, fo = fmt.fan_in(s), fmt.fan_out(s)
        n = (fi + fo) / 2 if self.varianceNormAverage else fo
        _fill(variable, RNG.normal_tensor(tuple(variable.shape), 0.0, math.sqrt(2.0 / n)))


class BilinearFiller(InitializationMethod):
    def init(self, variable, fmt=VariableFormats.Default):
        s = list(variable.shape)
        if len(s) != 5:
            raise ValueError(f"weight must be 5 dim, but got {len(s)}")
        kH, kW = s[3], s[4]
        if kH != kW:
            raise ValueError(f"Kernel {kH} * {kW} must be square")
        f = math.ceil(kW / 2.0)
        c = (2 * f - 1 - f % 2) / (2.0 * f)
        n = variable.numel()
        i = np.arange(n)
        x = (i % kW).astype(np.float32)
        y = ((i // kW) % kH).astype(np.float32)
        vals = (1 - np.abs(x / f - c)) * (1 - np.abs(y / f - c))
        _fill(variable, torch.from_numpy(vals.astype(np.float32)))


# pyspark-style aliases (bigdl/nn/initialization_method.py)
Default = VariableFormats.Default
