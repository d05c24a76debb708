"""LeNet-5 (``DL/models/lenet/LeNet5.scala:25-43``): conv(1→6,5)·tanh·maxpool·conv(6→12,5)·tanh·
maxpool·reshape(192)·linear(192→100)·tanh·linear(100→10)·logsoftmax; 22,278 parameters."""
from __future__ import annotations

from ..nn import (Sequential, Reshape, SpatialConvolution, Tanh, SpatialMaxPooling, Linear, LogSoftMax, Input, Graph)


def LeNet5(class_num: int = 10):
    model = Sequential()
    model.add(Reshape([1, 28, 28]))
    model.add(SpatialConvolution(1, 6, 5, 5).set_name("conv1_5x5"))
    model.add(Tanh())
    model.add(SpatialMaxPooling(2, 2, 2, 2))
    model.add(SpatialConvolution(6, 12, 5, 5).set_name("conv2_5x5"))
    model.add(Tanh())
    model.add(SpatialMaxPooling(2, 2, 2, 2))
    model.add(Reshape([12 * 4 * 4]))
    model.add(Linear(12 * 4 * 4, 100).set_name("fc1"))
    model.add(Tanh())
    model.add(Linear(100, class_num).set_name("fc2"))
    model.add(LogSoftMax())
    return model


def LeNet5Graph(class_num: int = 10):
    inp = Input()
    x = Reshape([1, 28, 28])(inp)
    x = SpatialConvolution(1, 6, 5, 5).set_name("conv1_5x5")(x)
    x = Tanh()(x)
    x = SpatialMaxPooling(2, 2, 2, 2)(x)
    x = SpatialConvolution(6, 12, 5, 5).set_name("conv2_5x5")(x)
    x = Tanh()(x)
    x = SpatialMaxPooling(2, 2, 2, 2)(x)
    x = Reshape([12 * 4 * 4])(x)
    x = Linear(12 * 4 * 4, 100).set_name("fc1")(x)
    x = Tanh()(x)
    x = Linear(100, class_num).set_name("fc2")(x)
    out = LogSoftMax()(x)
    return Graph(inp, out)
