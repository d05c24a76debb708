"""ResNet builders (``DL/models/resnet/ResNet.scala:75-449``).

Same topology and initialisation as the reference: ``Convolution`` = SpatialShareConvolution with
bias, L2Regularizer(1e-4) on weight and bias, MsraFiller(false)/Zeros init; ``Sbn`` =
SpatialBatchNormalization(eps=1e-3) with Ones/Zeros init; bottleneck with the stride on the 3×3
conv and the last BN of each block zero-initialised (:208); shortcut types A/B/C; ImageNet depths
18/34/50/101/152/200 and CIFAR-10 depths 6n+2.  ``modelInit`` (ResNet.scala:118-143) re-draws
conv weights N(0, √(2/(k²·nOut))).
"""
from __future__ import annotations

import math

from ..nn import (Sequential, ConcatTable, CAddTable, ReLU, Identity, Concat, MulConstant, View, Linear,
                  SpatialShareConvolution, SpatialConvolution, SpatialBatchNormalization, SpatialMaxPooling,
                  SpatialAveragePooling)
from ..nn.initialization_method import MsraFiller, Zeros, Ones, RandomNormal
from ..optim.regularizer import L2Regularizer
from ..utils.random import RNG


class ShortcutType:
    A = "A"
    B = "B"
    C = "C"


class DatasetType:
    CIFAR10 = "CIFAR10"
    ImageNet = "ImageNet"


def Convolution(n_in, n_out, kw, kh, sw=1, sh=1, pw=0, ph=0, n_group=1, propagate_back=True, optnet=True,
                weight_decay=1e-4):
    cls = SpatialShareConvolution if optnet else SpatialConvolution
    conv = cls(n_in, n_out, kw, kh, sw, sh, pw, ph, n_group, propagate_back, L2Regularizer(weight_decay),
               L2Regularizer(weight_decay))
    conv.setInitMethod(MsraFiller(False), Zeros())
    return conv


def Sbn(n, eps=1e-3, momentum=0.1, affine=True):
    return SpatialBatchNormalization(n, eps, momentum, affine).setInitMethod(Ones(), Zeros())


def ResNet(class_num: int, depth: int = 18, shortcut_type: str = ShortcutType.B, dataset: str = DatasetType.CIFAR10,
           optnet: bool = True, image_size: int = 224):
    """``image_size`` (ImageNet only) sizes the final average pool (7 at the reference's 224²), so
    the same topology runs on smaller synthetic images (CPU launch tests)."""
    state = {"iChannels": 64}

    def shortcut(n_in, n_out, stride):
        use_conv = shortcut_type == ShortcutType.C or (shortcut_type == ShortcutType.B and n_in != n_out)
        if use_conv:
            return Sequential().add(Convolution(n_in, n_out, 1, 1, stride, stride, optnet=optnet)).add(Sbn(n_out))
        if n_in != n_out:
            return Sequential().add(SpatialAveragePooling(1, 1, stride, stride)).add(
                Concat(2).add(Identity()).add(MulConstant(0.0)))
        return Identity()

    def basic_block(n, stride):
        n_in = state["iChannels"]
        state["iChannels"] = n
        s = Sequential()
        s.add(Convolution(n_in, n, 3, 3, stride, stride, 1, 1, optnet=optnet))
        s.add(Sbn(n))
        s.add(ReLU(True))
        s.add(Convolution(n, n, 3, 3, 1, 1, 1, 1, optnet=optnet))
        s.add(Sbn(n))
        return Sequential().add(ConcatTable().add(s).add(shortcut(n_in, n, stride))).add(CAddTable(True)).add(ReLU(True))

    def bottleneck(n, stride):
        n_in = state["iChannels"]
        state["iChannels"] = n * 4
        s = Sequential()
        s.add(Convolution(n_in, n, 1, 1, 1, 1, 0, 0, optnet=optnet)).add(Sbn(n)).add(ReLU(True))
        s.add(Convolution(n, n, 3, 3, stride, stride, 1, 1, optnet=optnet)).add(Sbn(n)).add(ReLU(True))
        s.add(Convolution(n, n * 4, 1, 1, 1, 1, 0, 0, optnet=optnet)).add(Sbn(n * 4).setInitMethod(Zeros(), Zeros()))
        return Sequential().add(ConcatTable().add(s).add(shortcut(n_in, n * 4, stride))).add(CAddTable(True)).add(ReLU(True))

    def layer(block, features, count, stride=1):
        s = Sequential()
        for i in range(count):
            s.add(block(features, stride if i == 0 else 1))
        return s

    model = Sequential()
    if dataset == DatasetType.ImageNet:
        cfg = {18: ((2, 2, 2, 2), 512, basic_block), 34: ((3, 4, 6, 3), 512, basic_block),
               50: ((3, 4, 6, 3), 2048, bottleneck), 101: ((3, 4, 23, 3), 2048, bottleneck),
               152: ((3, 8, 36, 3), 2048, bottleneck), 200: ((3, 24, 36, 3), 2048, bottleneck)}
        if depth not in cfg:
            raise ValueError(f"Invalid depth {depth}")
        loop, n_features, block = cfg[depth]
        state["iChannels"] = 64
        model.add(Convolution(3, 64, 7, 7, 2, 2, 3, 3, optnet=optnet, propagate_back=False)).add(Sbn(64)).add(ReLU(True))
        model.add(SpatialMaxPooling(3, 3, 2, 2, 1, 1))
        model.add(layer(block, 64, loop[0]))
        model.add(layer(block, 128, loop[1], 2))
        model.add(layer(block, 256, loop[2], 2))
        model.add(layer(block, 512, loop[3], 2))
        pool = max(1, -(-int(image_size) // 32))
        model.add(SpatialAveragePooling(pool, pool, 1, 1))
        model.add(View(n_features).setNumInputDims(3))
        model.add(Linear(n_features, class_num, True, L2Regularizer(1e-4), L2Regularizer(1e-4))
                  .setInitMethod(RandomNormal(0.0, 0.01), Zeros()))
    else:
        if (depth - 2) % 6 != 0:
            raise ValueError("depth should be one of 20, 32, 44, 56, 110, 1202")
        n = (depth - 2) // 6
        state["iChannels"] = 16
        model.add(Convolution(3, 16, 3, 3, 1, 1, 1, 1, optnet=optnet)).add(Sbn(16)).add(ReLU(True))
        model.add(layer(basic_block, 16, n))
        model.add(layer(basic_block, 32, n, 2))
        model.add(layer(basic_block, 64, n, 2))
        model.add(SpatialAveragePooling(8, 8, 1, 1))
        model.add(View(64).setNumInputDims(3))
        model.add(Linear(64, class_num))
    return model


def model_init(model):
    """``ResNet.modelInit``: conv N(0, √(2/(kW²·nOut))) with zero bias, BN γ=1 β=0, Linear bias 0."""
    import torch
    for m in model.flattened_modules():
        if isinstance(m, SpatialConvolution):
            n = m.kernelW * m.kernelW * m.nOutputPlane
            m.weight.copy_(RNG.normal_tensor(tuple(m.weight.shape), 0.0, math.sqrt(2.0 / n)).to(m.weight.device))
            if m.bias is not None:
                m.bias.zero_()
        elif isinstance(m, SpatialBatchNormalization):
            m.weight.fill_(1.0)
            m.bias.zero_()
        elif isinstance(m, Linear) and m.bias is not None:
            m.bias.zero_()
    return model
