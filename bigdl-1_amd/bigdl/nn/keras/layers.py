"""Keras-1.2.2 layers (``DL/nn/keras/*.scala``, ``pyspark/bigdl/nn/keras/layer.py``): each builds the
matching ``bigdl.nn`` module once its input shape is known and infers its output shape.

Conventions: shapes exclude the batch dimension; ``dim_ordering="th"`` = channels first (NCHW),
``"tf"`` = channels last; ``border_mode`` "valid" / "same"; activations and initialisers by their
Keras names."""
from __future__ import annotations

import math
from typing import List, Optional, Sequence

from .. import layers as L
from ..containers import Sequential as _Seq, ConcatTable as _ConcatTable
from ..initialization_method import Xavier, MsraFiller, RandomUniform, RandomNormal, Zeros, Ones
from .topology import KerasLayer, _as_shape


# ------------------------------------------------------------------------------------------------ helpers
def activation_module(name):
    if name is None or name == "linear":
        return None
    if not isinstance(name, str):
        return name
    n = name.lower()
    table = {"relu": lambda: L.ReLU(), "tanh": lambda: L.Tanh(), "sigmoid": lambda: L.Sigmoid(),
             "hard_sigmoid": lambda: L.HardSigmoid(), "softmax": lambda: L.SoftMax(),
             "softplus": lambda: L.SoftPlus(), "softsign": lambda: L.SoftSign(), "relu6": lambda: L.ReLU6(),
             "elu": lambda: L.ELU(), "log_softmax": lambda: L.LogSoftMax()}
    if n not in table:
        raise ValueError(f"Unsupported activation: {name}")
    return table[n]()


def init_method(name):
    if not isinstance(name, str):
        return name
    n = name.lower()
    if n == "glorot_uniform":
        return Xavier()
    if n in ("one", "ones"):
        return Ones()
    if n in ("zero", "zeros"):
        return Zeros()
    if n == "uniform":
        return RandomUniform(-0.05, 0.05)
    if n == "normal":
        return RandomNormal(0.0, 0.05)
    if n in ("he_normal", "msra"):
        return MsraFiller(False)
    raise ValueError(f"Unsupported init: {name}")


def _with_activation(core, activation):
    act = activation_module(activation)
    if act is None:
        return core
    return _Seq().add(core).add(act)


def _conv_out(size, k, s, mode, dil=1):
    if size < 0:
        return -1
    ke = dil * (k - 1) + 1
    if mode == "same":
        return int(math.ceil(size / s))
    return (size - ke) // s + 1


def _pad_for(mode):
    return -1 if mode == "same" else 0


# ------------------------------------------------------------------------------------------------ core
class Dense(KerasLayer):
    def __init__(self, output_dim, init="glorot_uniform", activation=None, W_regularizer=None, b_regularizer=None,
                 bias=True, input_dim=None, input_shape=None, name=None):
        super().__init__((input_dim,) if input_dim else input_shape, name)
        self.output_dim, self.init, self.activation = output_dim, init, activation
        self.W_regularizer, self.b_regularizer, self.bias = W_regularizer, b_regularizer, bias

    def build_labor(self, s):
        lin = L.Linear(s[-1], self.output_dim, self.bias, self.W_regularizer, self.b_regularizer)
        lin.setInitMethod(init_method(self.init), Zeros())
        core = lin if len(s) == 1 else L.TimeDistributed(lin)
        return _with_activation(core, self.activation)

    def compute_output_shape(self, s):
        return tuple(s[:-1]) + (self.output_dim,)


class MaxoutDense(KerasLayer):
    def __init__(self, output_dim, nb_feature=4, W_regularizer=None, b_regularizer=None, bias=True, input_dim=None,
                 input_shape=None, name=None):
        super().__init__((input_dim,) if input_dim else input_shape, name)
        self.output_dim, self.nb_feature, self.bias = output_dim, nb_feature, bias
        self.W_regularizer, self.b_regularizer = W_regularizer, b_regularizer

    def build_labor(self, s):
        return L.Maxout(s[-1], self.output_dim, self.nb_feature, self.bias, self.W_regularizer, self.b_regularizer)

    def compute_output_shape(self, s):
        return (self.output_dim,)


class Activation(KerasLayer):
    def __init__(self, activation, input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.activation = activation

    def build_labor(self, s):
        a = activation_module(self.activation)
        return a if a is not None else L.Identity()


class Dropout(KerasLayer):
    def __init__(self, p, input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.p = p

    def build_labor(self, s):
        return L.Dropout(self.p)


class Flatten(KerasLayer):
    def build_labor(self, s):
        return L.Reshape([int(math.prod(s))], batch_mode=True)

    def compute_output_shape(self, s):
        return (int(math.prod(s)),)


class Reshape(KerasLayer):
    def __init__(self, target_shape, input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.target_shape = tuple(target_shape)

    def _resolved(self, s):
        tgt = list(self.target_shape)
        if -1 in tgt:
            known = int(math.prod(v for v in tgt if v != -1))
            tgt[tgt.index(-1)] = int(math.prod(s)) // known
        return tuple(tgt)

    def build_labor(self, s):
        return L.Reshape(list(self._resolved(s)), batch_mode=True)

    def compute_output_shape(self, s):
        return self._resolved(s)


class Permute(KerasLayer):
    def __init__(self, dims, input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.dims = tuple(dims)  # 1-based over non-batch dims

    def build_labor(self, s):
        # express the permutation as a sequence of swaps on 1-based dims (batch = dim 1)
        cur = list(range(1, len(s) + 1))
        swaps = []
        for i, d in enumerate(self.dims):
            j = cur.index(d)
            if j != i:
                swaps.append((i + 2, j + 2))
                cur[i], cur[j] = cur[j], cur[i]
        return L.Transpose(swaps) if swaps else L.Identity()

    def compute_output_shape(self, s):
        return tuple(s[d - 1] for d in self.dims)


class RepeatVector(KerasLayer):
    def __init__(self, n, input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.n = n

    def build_labor(self, s):
        return L.Replicate(self.n, dim=1, n_dim=1)

    def compute_output_shape(self, s):
        return (self.n,) + tuple(s)


class Highway(KerasLayer):
    def __init__(self, activation=None, W_regularizer=None, b_regularizer=None, bias=True, input_shape=None,
                 name=None):
        super().__init__(input_shape, name)
        self.activation, self.W_regularizer, self.b_regularizer, self.bias = activation, W_regularizer, \
            b_regularizer, bias

    def build_labor(self, s):
        return L.Highway(s[-1], self.bias, activation_module(self.activation), self.W_regularizer,
                         self.b_regularizer)


class Masking(KerasLayer):
    def __init__(self, mask_value=0.0, input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.mask_value = mask_value

    def build_labor(self, s):
        return L.Masking(self.mask_value)


class Embedding(KerasLayer):
    def __init__(self, input_dim, output_dim, init="uniform", W_regularizer=None, input_shape=None,
                 input_length=None, name=None):
        super().__init__((input_length,) if input_length else input_shape, name)
        self.input_dim, self.output_dim, self.init, self.W_regularizer = input_dim, output_dim, init, W_regularizer

    def build_labor(self, s):
        # Keras indices are 0-based; LookupTable is 1-based
        lt = L.LookupTable(self.input_dim, self.output_dim, wRegularizer=self.W_regularizer)
        lt.setInitMethod(init_method(self.init))
        return _Seq().add(L.AddConstant(1.0)).add(lt)

    def compute_output_shape(self, s):
        return tuple(s) + (self.output_dim,)


class BatchNormalization(KerasLayer):
    def __init__(self, epsilon=1e-3, mode=0, axis=1, momentum=0.99, beta_init="zero", gamma_init="one",
                 dim_ordering="th", input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.epsilon, self.momentum, self.dim_ordering = epsilon, momentum, dim_ordering
        self.beta_init, self.gamma_init = beta_init, gamma_init

    def build_labor(self, s):
        # Keras momentum m keeps m of the running value; BigDL's momentum is the new-sample weight
        mom = 1.0 - self.momentum
        if len(s) == 3:
            fmt = "NCHW" if self.dim_ordering == "th" else "NHWC"
            bn = L.SpatialBatchNormalization(s[0] if fmt == "NCHW" else s[-1], self.epsilon, mom, data_format=fmt)
        else:
            bn = L.BatchNormalization(s[-1], self.epsilon, mom)
        bn.setInitMethod(init_method(self.gamma_init), init_method(self.beta_init))
        return bn


class Merge(KerasLayer):
    """Merge a list of inputs: ``mode`` in sum / mul / concat / ave / max / dot / cos."""

    def __init__(self, layers=None, mode="sum", concat_axis=-1, input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.mode, self.concat_axis = mode, concat_axis
        self.layers = layers

    def build_labor(self, shapes):
        m = self.mode
        if m == "sum":
            return L.CAddTable()
        if m == "mul":
            return L.CMulTable()
        if m == "ave":
            return L.CAveTable()
        if m == "max":
            return L.CMaxTable()
        if m == "concat":
            nd = len(shapes[0])
            ax = self.concat_axis if self.concat_axis >= 0 else nd + 1 + self.concat_axis
            return L.JoinTable(ax, nd)
        if m == "dot":
            return L.DotProduct()
        if m == "cos":
            return L.CosineDistance()
        raise ValueError(f"Unsupported merge mode: {m}")

    def compute_output_shape(self, shapes):
        m = self.mode
        if m == "concat":
            nd = len(shapes[0])
            ax = (self.concat_axis if self.concat_axis >= 0 else nd + 1 + self.concat_axis) - 1
            out = list(shapes[0])
            out[ax] = sum(s[ax] for s in shapes)
            return tuple(out)
        if m in ("dot", "cos"):
            return (1,)
        return tuple(shapes[0])


# ------------------------------------------------------------------------------------------------ conv
class Convolution1D(KerasLayer):
    def __init__(self, nb_filter, filter_length, init="glorot_uniform", activation=None, border_mode="valid",
                 subsample_length=1, W_regularizer=None, b_regularizer=None, bias=True, input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.nb_filter, self.k, self.init, self.activation = nb_filter, filter_length, init, activation
        self.border_mode, self.stride, self.bias = border_mode, subsample_length, bias
        self.W_regularizer, self.b_regularizer = W_regularizer, b_regularizer

    def build_labor(self, s):
        core = L.TemporalConvolution(s[-1], self.nb_filter, self.k, self.stride,
                                     weight_regularizer=self.W_regularizer,
                                     bias_regularizer=self.b_regularizer) if self.border_mode == "valid" else None
        if core is None:  # same padding along time
            tot = max((self.k - 1), 0)
            core = _Seq().add(L.Padding(1, -(tot // 2), 2)).add(L.Padding(1, tot - tot // 2, 2)).add(
                L.TemporalConvolution(s[-1], self.nb_filter, self.k, self.stride,
                                      weight_regularizer=self.W_regularizer, bias_regularizer=self.b_regularizer))
        return _with_activation(core, self.activation)

    def compute_output_shape(self, s):
        return (_conv_out(s[0], self.k, self.stride, self.border_mode), self.nb_filter)


class Convolution2D(KerasLayer):
    def __init__(self, nb_filter, nb_row, nb_col, init="glorot_uniform", activation=None, border_mode="valid",
                 subsample=(1, 1), dim_ordering="th", W_regularizer=None, b_regularizer=None, bias=True,
                 input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.nb_filter, self.nb_row, self.nb_col = nb_filter, nb_row, nb_col
        self.init, self.activation, self.border_mode = init, activation, border_mode
        self.subsample, self.dim_ordering, self.bias = tuple(subsample), dim_ordering, bias
        self.W_regularizer, self.b_regularizer = W_regularizer, b_regularizer

    def _cin(self, s):
        return s[0] if self.dim_ordering == "th" else s[-1]

    def build_labor(self, s):
        p = _pad_for(self.border_mode)
        conv = L.SpatialConvolution(self._cin(s), self.nb_filter, self.nb_col, self.nb_row, self.subsample[1],
                                    self.subsample[0], p, p, 1, True, self.W_regularizer, self.b_regularizer,
                                    with_bias=self.bias, data_format="NCHW" if self.dim_ordering == "th" else "NHWC")
        conv.setInitMethod(init_method(self.init), Zeros())
        return _with_activation(conv, self.activation)

    def compute_output_shape(self, s):
        if self.dim_ordering == "th":
            return (self.nb_filter, _conv_out(s[1], self.nb_row, self.subsample[0], self.border_mode),
                    _conv_out(s[2], self.nb_col, self.subsample[1], self.border_mode))
        return (_conv_out(s[0], self.nb_row, self.subsample[0], self.border_mode),
                _conv_out(s[1], self.nb_col, self.subsample[1], self.border_mode), self.nb_filter)


class AtrousConvolution2D(Convolution2D):
    def __init__(self, nb_filter, nb_row, nb_col, init="glorot_uniform", activation=None, border_mode="valid",
                 subsample=(1, 1), atrous_rate=(1, 1), dim_ordering="th", W_regularizer=None, b_regularizer=None,
                 bias=True, input_shape=None, name=None):
        super().__init__(nb_filter, nb_row, nb_col, init, activation, border_mode, subsample, dim_ordering,
                         W_regularizer, b_regularizer, bias, input_shape, name)
        self.atrous_rate = tuple(atrous_rate)

    def build_labor(self, s):
        conv = L.SpatialDilatedConvolution(self._cin(s), self.nb_filter, self.nb_col, self.nb_row, self.subsample[1],
                                           self.subsample[0], 0, 0, self.atrous_rate[1], self.atrous_rate[0],
                                           self.W_regularizer, self.b_regularizer)
        conv.setInitMethod(init_method(self.init), Zeros())
        return _with_activation(conv, self.activation)

    def compute_output_shape(self, s):
        return (self.nb_filter, _conv_out(s[1], self.nb_row, self.subsample[0], "valid", self.atrous_rate[0]),
                _conv_out(s[2], self.nb_col, self.subsample[1], "valid", self.atrous_rate[1]))


class AtrousConvolution1D(Convolution1D):
    def __init__(self, nb_filter, filter_length, init="glorot_uniform", activation=None, border_mode="valid",
                 subsample_length=1, atrous_rate=1, W_regularizer=None, b_regularizer=None, bias=True,
                 input_shape=None, name=None):
        super().__init__(nb_filter, filter_length, init, activation, border_mode, subsample_length, W_regularizer,
                         b_regularizer, bias, input_shape, name)
        self.atrous_rate = atrous_rate

    def build_labor(self, s):
        # (T, F) → (F, T, 1) dilated 2-D conv → (T', nb_filter)
        conv = L.SpatialDilatedConvolution(s[-1], self.nb_filter, 1, self.k, 1, self.stride, 0, 0, 1,
                                           self.atrous_rate, self.W_regularizer, self.b_regularizer)
        core = _Seq().add(L.Transpose([(2, 3)])).add(L.Unsqueeze(4)).add(conv).add(L.Squeeze(4)).add(
            L.Transpose([(2, 3)]))
        return _with_activation(core, self.activation)

    def compute_output_shape(self, s):
        return (_conv_out(s[0], self.k, self.stride, "valid", self.atrous_rate), self.nb_filter)


class Deconvolution2D(Convolution2D):
    def __init__(self, nb_filter, nb_row, nb_col, output_shape=None, init="glorot_uniform", activation=None,
                 border_mode="valid", subsample=(1, 1), dim_ordering="th", W_regularizer=None, b_regularizer=None,
                 bias=True, input_shape=None, name=None):
        super().__init__(nb_filter, nb_row, nb_col, init, activation, border_mode, subsample, dim_ordering,
                         W_regularizer, b_regularizer, bias, input_shape, name)

    def build_labor(self, s):
        conv = L.SpatialFullConvolution(self._cin(s), self.nb_filter, self.nb_col, self.nb_row, self.subsample[1],
                                        self.subsample[0], 0, 0, 0, 0, 1, not self.bias, self.W_regularizer,
                                        self.b_regularizer)
        return _with_activation(conv, self.activation)

    def compute_output_shape(self, s):
        return (self.nb_filter, (s[1] - 1) * self.subsample[0] + self.nb_row,
                (s[2] - 1) * self.subsample[1] + self.nb_col)


class SeparableConvolution2D(Convolution2D):
    def __init__(self, nb_filter, nb_row, nb_col, init="glorot_uniform", activation=None, border_mode="valid",
                 subsample=(1, 1), depth_multiplier=1, dim_ordering="th", depthwise_regularizer=None,
                 pointwise_regularizer=None, b_regularizer=None, bias=True, input_shape=None, name=None):
        super().__init__(nb_filter, nb_row, nb_col, init, activation, border_mode, subsample, dim_ordering, None,
                         b_regularizer, bias, input_shape, name)
        self.depth_multiplier = depth_multiplier
        self.depthwise_regularizer, self.pointwise_regularizer = depthwise_regularizer, pointwise_regularizer

    def build_labor(self, s):
        p = _pad_for(self.border_mode)
        conv = L.SpatialSeparableConvolution(self._cin(s), self.nb_filter, self.depth_multiplier, self.nb_col,
                                             self.nb_row, self.subsample[1], self.subsample[0], p, p, self.bias,
                                             "NCHW" if self.dim_ordering == "th" else "NHWC",
                                             self.depthwise_regularizer, self.pointwise_regularizer,
                                             self.b_regularizer)
        return _with_activation(conv, self.activation)


class Convolution3D(KerasLayer):
    def __init__(self, nb_filter, kernel_dim1, kernel_dim2, kernel_dim3, init="glorot_uniform", activation=None,
                 border_mode="valid", subsample=(1, 1, 1), dim_ordering="th", W_regularizer=None, b_regularizer=None,
                 bias=True, input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.nb_filter, self.k = nb_filter, (kernel_dim1, kernel_dim2, kernel_dim3)
        self.init, self.activation, self.border_mode, self.subsample = init, activation, border_mode, \
            tuple(subsample)
        self.W_regularizer, self.b_regularizer, self.bias = W_regularizer, b_regularizer, bias

    def build_labor(self, s):
        p = _pad_for(self.border_mode)
        conv = L.VolumetricConvolution(s[0], self.nb_filter, self.k[0], self.k[2], self.k[1], self.subsample[0],
                                       self.subsample[2], self.subsample[1], p, p, p, self.bias, self.W_regularizer,
                                       self.b_regularizer)
        return _with_activation(conv, self.activation)

    def compute_output_shape(self, s):
        return (self.nb_filter,) + tuple(_conv_out(s[i + 1], self.k[i], self.subsample[i], self.border_mode)
                                         for i in range(3))


class LocallyConnected1D(KerasLayer):
    def __init__(self, nb_filter, filter_length, activation=None, border_mode="valid", subsample_length=1,
                 W_regularizer=None, b_regularizer=None, bias=True, input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.nb_filter, self.k, self.activation, self.stride = nb_filter, filter_length, activation, subsample_length
        self.W_regularizer, self.b_regularizer = W_regularizer, b_regularizer

    def build_labor(self, s):
        return _with_activation(L.LocallyConnected1D(s[0], s[1], self.nb_filter, self.k, self.stride, True,
                                                     self.W_regularizer, self.b_regularizer), self.activation)

    def compute_output_shape(self, s):
        return ((s[0] - self.k) // self.stride + 1, self.nb_filter)


class LocallyConnected2D(KerasLayer):
    def __init__(self, nb_filter, nb_row, nb_col, activation=None, border_mode="valid", subsample=(1, 1),
                 dim_ordering="th", W_regularizer=None, b_regularizer=None, bias=True, input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.nb_filter, self.nb_row, self.nb_col = nb_filter, nb_row, nb_col
        self.activation, self.border_mode, self.subsample = activation, border_mode, tuple(subsample)
        self.W_regularizer, self.b_regularizer = W_regularizer, b_regularizer

    def build_labor(self, s):
        p = _pad_for(self.border_mode)
        return _with_activation(L.LocallyConnected2D(s[0], s[2], s[1], self.nb_filter, self.nb_col, self.nb_row,
                                                     self.subsample[1], self.subsample[0], p, p, True,
                                                     self.W_regularizer, self.b_regularizer), self.activation)

    def compute_output_shape(self, s):
        return (self.nb_filter, _conv_out(s[1], self.nb_row, self.subsample[0], self.border_mode),
                _conv_out(s[2], self.nb_col, self.subsample[1], self.border_mode))


# ------------------------------------------------------------------------------------------------ pooling
class _Pool2D(KerasLayer):
    MAX = True

    def __init__(self, pool_size=(2, 2), strides=None, border_mode="valid", dim_ordering="th", input_shape=None,
                 name=None):
        super().__init__(input_shape, name)
        self.pool_size = tuple(pool_size)
        self.strides = tuple(strides) if strides is not None else self.pool_size
        self.border_mode, self.dim_ordering = border_mode, dim_ordering

    def build_labor(self, s):
        p = _pad_for(self.border_mode)
        fmt = "NCHW" if self.dim_ordering == "th" else "NHWC"
        if self.MAX:
            return L.SpatialMaxPooling(self.pool_size[1], self.pool_size[0], self.strides[1], self.strides[0], p, p,
                                       format=fmt)
        return L.SpatialAveragePooling(self.pool_size[1], self.pool_size[0], self.strides[1], self.strides[0], p, p,
                                       count_include_pad=False, format=fmt)

    def compute_output_shape(self, s):
        if self.dim_ordering == "th":
            return (s[0], _conv_out(s[1], self.pool_size[0], self.strides[0], self.border_mode),
                    _conv_out(s[2], self.pool_size[1], self.strides[1], self.border_mode))
        return (_conv_out(s[0], self.pool_size[0], self.strides[0], self.border_mode),
                _conv_out(s[1], self.pool_size[1], self.strides[1], self.border_mode), s[2])


class MaxPooling2D(_Pool2D):
    MAX = True


class AveragePooling2D(_Pool2D):
    MAX = False


class _Pool1D(KerasLayer):
    MAX = True

    def __init__(self, pool_length=2, stride=None, border_mode="valid", input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.pool_length, self.stride, self.border_mode = pool_length, stride or pool_length, border_mode

    def build_labor(self, s):
        if self.MAX:
            return L.TemporalMaxPooling(self.pool_length, self.stride)
        # (T, F) → (F, T, 1) average → back
        return _Seq().add(L.Transpose([(2, 3)])).add(L.Unsqueeze(4)).add(
            L.SpatialAveragePooling(1, self.pool_length, 1, self.stride)).add(L.Squeeze(4)).add(
            L.Transpose([(2, 3)]))

    def compute_output_shape(self, s):
        return (_conv_out(s[0], self.pool_length, self.stride, self.border_mode), s[1])


class MaxPooling1D(_Pool1D):
    MAX = True


class AveragePooling1D(_Pool1D):
    MAX = False


class _Pool3D(KerasLayer):
    MAX = True

    def __init__(self, pool_size=(2, 2, 2), strides=None, border_mode="valid", dim_ordering="th", input_shape=None,
                 name=None):
        super().__init__(input_shape, name)
        self.pool_size = tuple(pool_size)
        self.strides = tuple(strides) if strides is not None else self.pool_size

    def build_labor(self, s):
        k, d = self.pool_size, self.strides
        if self.MAX:
            return L.VolumetricMaxPooling(k[0], k[2], k[1], d[0], d[2], d[1])
        return L.VolumetricAveragePooling(k[0], k[2], k[1], d[0], d[2], d[1])

    def compute_output_shape(self, s):
        return (s[0],) + tuple((s[i + 1] - self.pool_size[i]) // self.strides[i] + 1 for i in range(3))


class MaxPooling3D(_Pool3D):
    MAX = True


class AveragePooling3D(_Pool3D):
    MAX = False


class _GlobalPool(KerasLayer):
    MAX = True
    NDIM = 2

    def __init__(self, dim_ordering="th", input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.dim_ordering = dim_ordering

    def build_labor(self, s):
        red = L.Max if self.MAX else L.Mean
        if self.NDIM == 1:  # (T, F) → reduce T
            return red(1, 2)
        first = 2 if self.dim_ordering == "th" else 1  # 1-based among non-batch dims
        seq = _Seq()
        nd = len(s)
        for i in range(self.NDIM):
            seq.add(red(first, nd - i))
        return seq

    def compute_output_shape(self, s):
        if self.NDIM == 1:
            return (s[1],)
        return (s[0],) if self.dim_ordering == "th" else (s[-1],)


class GlobalMaxPooling1D(_GlobalPool):
    MAX, NDIM = True, 1


class GlobalAveragePooling1D(_GlobalPool):
    MAX, NDIM = False, 1


class GlobalMaxPooling2D(_GlobalPool):
    MAX, NDIM = True, 2


class GlobalAveragePooling2D(_GlobalPool):
    MAX, NDIM = False, 2


class GlobalMaxPooling3D(_GlobalPool):
    MAX, NDIM = True, 3


class GlobalAveragePooling3D(_GlobalPool):
    MAX, NDIM = False, 3


# ------------------------------------------------------------------------------------------------ padding etc.
class ZeroPadding1D(KerasLayer):
    def __init__(self, padding=1, input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.padding = (padding, padding) if isinstance(padding, int) else tuple(padding)

    def build_labor(self, s):
        return _Seq().add(L.Padding(1, -self.padding[0], 2)).add(L.Padding(1, self.padding[1], 2))

    def compute_output_shape(self, s):
        return (s[0] + sum(self.padding), s[1])


class ZeroPadding2D(KerasLayer):
    def __init__(self, padding=(1, 1), dim_ordering="th", input_shape=None, name=None):
        super().__init__(input_shape, name)
        p = tuple(padding)
        self.padding = (p[0], p[0], p[1], p[1]) if len(p) == 2 else p
        self.dim_ordering = dim_ordering

    def build_labor(self, s):
        top, bottom, left, right = self.padding
        return L.SpatialZeroPadding(left, right, top, bottom)

    def compute_output_shape(self, s):
        t, b, l, r = self.padding
        return (s[0], s[1] + t + b, s[2] + l + r)


class ZeroPadding3D(KerasLayer):
    def __init__(self, padding=(1, 1, 1), dim_ordering="th", input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.padding = tuple(padding)

    def build_labor(self, s):
        seq = _Seq()
        for i, p in enumerate(self.padding):
            seq.add(L.Padding(i + 2, -p, 4)).add(L.Padding(i + 2, p, 4))
        return seq

    def compute_output_shape(self, s):
        return (s[0],) + tuple(s[i + 1] + 2 * self.padding[i] for i in range(3))


class Cropping1D(KerasLayer):
    def __init__(self, cropping=(1, 1), input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.cropping = tuple(cropping)

    def build_labor(self, s):
        return L.Narrow(2, self.cropping[0] + 1, s[0] - sum(self.cropping))

    def compute_output_shape(self, s):
        return (s[0] - sum(self.cropping), s[1])


class Cropping2D(KerasLayer):
    def __init__(self, cropping=((0, 0), (0, 0)), dim_ordering="th", input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.cropping = tuple(tuple(c) for c in cropping)
        self.dim_ordering = dim_ordering

    def build_labor(self, s):
        return L.Cropping2D(self.cropping[0], self.cropping[1], "NCHW" if self.dim_ordering == "th" else "NHWC")

    def compute_output_shape(self, s):
        (t, b), (l, r) = self.cropping
        if self.dim_ordering == "th":
            return (s[0], s[1] - t - b, s[2] - l - r)
        return (s[0] - t - b, s[1] - l - r, s[2])


class Cropping3D(KerasLayer):
    def __init__(self, cropping=((1, 1), (1, 1), (1, 1)), dim_ordering="th", input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.cropping = tuple(tuple(c) for c in cropping)

    def build_labor(self, s):
        return L.Cropping3D(*self.cropping)

    def compute_output_shape(self, s):
        return (s[0],) + tuple(s[i + 1] - sum(self.cropping[i]) for i in range(3))


class UpSampling1D(KerasLayer):
    def __init__(self, length=2, input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.length = length

    def build_labor(self, s):
        return L.UpSampling1D(self.length)

    def compute_output_shape(self, s):
        return (s[0] * self.length, s[1])


class UpSampling2D(KerasLayer):
    def __init__(self, size=(2, 2), dim_ordering="th", input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.size, self.dim_ordering = tuple(size), dim_ordering

    def build_labor(self, s):
        return L.UpSampling2D(self.size, "nchw" if self.dim_ordering == "th" else "nhwc")

    def compute_output_shape(self, s):
        if self.dim_ordering == "th":
            return (s[0], s[1] * self.size[0], s[2] * self.size[1])
        return (s[0] * self.size[0], s[1] * self.size[1], s[2])


class UpSampling3D(KerasLayer):
    def __init__(self, size=(2, 2, 2), dim_ordering="th", input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.size = tuple(size)

    def build_labor(self, s):
        return L.UpSampling3D(self.size)

    def compute_output_shape(self, s):
        return (s[0],) + tuple(s[i + 1] * self.size[i] for i in range(3))


# ------------------------------------------------------------------------------------------------ noise / activations
class SpatialDropout1D(KerasLayer):
    def __init__(self, p=0.5, input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.p = p

    def build_labor(self, s):
        return L.SpatialDropout1D(self.p)


class SpatialDropout2D(KerasLayer):
    def __init__(self, p=0.5, dim_ordering="th", input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.p, self.dim_ordering = p, dim_ordering

    def build_labor(self, s):
        return L.SpatialDropout2D(self.p, "NCHW" if self.dim_ordering == "th" else "NHWC")


class SpatialDropout3D(KerasLayer):
    def __init__(self, p=0.5, dim_ordering="th", input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.p, self.dim_ordering = p, dim_ordering

    def build_labor(self, s):
        return L.SpatialDropout3D(self.p, "NCHW" if self.dim_ordering == "th" else "NHWC")


class GaussianDropout(KerasLayer):
    def __init__(self, p, input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.p = p

    def build_labor(self, s):
        return L.GaussianDropout(self.p)


class GaussianNoise(KerasLayer):
    def __init__(self, sigma, input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.sigma = sigma

    def build_labor(self, s):
        return L.GaussianNoise(self.sigma)


class ELU(KerasLayer):
    def __init__(self, alpha=1.0, input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.alpha = alpha

    def build_labor(self, s):
        return L.ELU(self.alpha)


class LeakyReLU(KerasLayer):
    def __init__(self, alpha=0.3, input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.alpha = alpha

    def build_labor(self, s):
        return L.LeakyReLU(self.alpha)


class ThresholdedReLU(KerasLayer):
    def __init__(self, theta=1.0, input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.theta = theta

    def build_labor(self, s):
        return L.Threshold(self.theta, 0.0)


class SReLU(KerasLayer):
    def __init__(self, t_left_init="zero", a_left_init="glorot_uniform", t_right_init="glorot_uniform",
                 a_right_init="one", shared_axes=None, input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.shared_axes = shared_axes

    def build_labor(self, s):
        return L.SReLU(list(s), self.shared_axes)


# ------------------------------------------------------------------------------------------------ recurrent
class _RNN(KerasLayer):
    def __init__(self, output_dim, activation="tanh", return_sequences=False, go_backwards=False,
                 W_regularizer=None, U_regularizer=None, b_regularizer=None, input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.output_dim, self.activation = output_dim, activation
        self.return_sequences, self.go_backwards = return_sequences, go_backwards
        self.W_regularizer, self.U_regularizer, self.b_regularizer = W_regularizer, U_regularizer, b_regularizer

    def cell(self, s):  # pragma: no cover - abstract
        raise NotImplementedError

    def build_labor(self, s):
        seq = _Seq()
        if self.go_backwards:
            seq.add(L.Reverse(2))
        seq.add(L.Recurrent().add(self.cell(s)))
        if not self.return_sequences:
            seq.add(L.Select(2, -1))
        return seq

    def compute_output_shape(self, s):
        return (s[0], self.output_dim) if self.return_sequences else (self.output_dim,)


class SimpleRNN(_RNN):
    def cell(self, s):
        return L.RnnCell(s[-1], self.output_dim, activation_module(self.activation) or L.Tanh())


class LSTM(_RNN):
    def __init__(self, output_dim, activation="tanh", inner_activation="hard_sigmoid", return_sequences=False,
                 go_backwards=False, W_regularizer=None, U_regularizer=None, b_regularizer=None, input_shape=None,
                 name=None):
        super().__init__(output_dim, activation, return_sequences, go_backwards, W_regularizer, U_regularizer,
                         b_regularizer, input_shape, name)
        self.inner_activation = inner_activation

    def cell(self, s):
        return L.LSTM(s[-1], self.output_dim, 0.0, activation_module(self.activation),
                      activation_module(self.inner_activation), self.W_regularizer, self.U_regularizer,
                      self.b_regularizer)


class GRU(LSTM):
    def cell(self, s):
        return L.GRU(s[-1], self.output_dim, 0.0, activation_module(self.activation),
                     activation_module(self.inner_activation), self.W_regularizer, self.U_regularizer,
                     self.b_regularizer)


class ConvLSTM2D(KerasLayer):
    def __init__(self, nb_filter, nb_kernel, activation="tanh", inner_activation="hard_sigmoid",
                 dim_ordering="th", border_mode="same", subsample=(1, 1), W_regularizer=None, U_regularizer=None,
                 b_regularizer=None, return_sequences=False, go_backwards=False, input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.nb_filter, self.nb_kernel, self.return_sequences = nb_filter, nb_kernel, return_sequences
        self.go_backwards, self.subsample = go_backwards, subsample
        self.activation, self.inner_activation = activation, inner_activation

    def build_labor(self, s):
        seq = _Seq()
        if self.go_backwards:
            seq.add(L.Reverse(2))
        seq.add(L.Recurrent().add(L.ConvLSTMPeephole(s[1], self.nb_filter, self.nb_kernel, self.nb_kernel,
                                                     self.subsample[0] if isinstance(self.subsample, tuple)
                                                     else self.subsample)))
        if not self.return_sequences:
            seq.add(L.Select(2, -1))
        return seq

    def compute_output_shape(self, s):
        st = self.subsample[0] if isinstance(self.subsample, tuple) else self.subsample
        o = (self.nb_filter, int(math.ceil(s[2] / st)), int(math.ceil(s[3] / st)))
        return (s[0],) + o if self.return_sequences else o


class TimeDistributed(KerasLayer):
    def __init__(self, layer: KerasLayer, input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.layer = layer

    def build_labor(self, s):
        self.layer.build(tuple(s[1:]))
        return L.TimeDistributed(self.layer)

    def compute_output_shape(self, s):
        return (s[0],) + tuple(self.layer.output_shape)


class Bidirectional(KerasLayer):
    def __init__(self, layer: _RNN, merge_mode="concat", input_shape=None, name=None):
        super().__init__(input_shape, name)
        self.layer, self.merge_mode = layer, merge_mode

    def build_labor(self, s):
        merge = {"concat": L.JoinTable(3, 3), "sum": L.CAddTable(), "mul": L.CMulTable(),
                 "ave": L.CAveTable()}[self.merge_mode]
        bi = L.BiRecurrent(merge)
        bi.add(self.layer.cell(s))
        seq = _Seq().add(bi)
        if not self.layer.return_sequences:
            seq.add(L.Select(2, -1))
        return seq

    def compute_output_shape(self, s):
        d = self.layer.output_dim * (2 if self.merge_mode == "concat" else 1)
        return (s[0], d) if self.layer.return_sequences else (d,)
