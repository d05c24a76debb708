"""VGG builders (``DL/models/vgg/VggForCifar10.scala:23-75``, ``Vgg_16``/``Vgg_19`` :131/:235).

VggForCifar10: 13 conv3×3 + SpatialBatchNormalization(eps=1e-3) + ReLU blocks with dropout
(0.3/0.4), ceil max-pools, classifier Dropout(0.5)·Linear(512,512)·BN·ReLU·Dropout(0.5)·Linear(512,10)
·LogSoftMax; ≈14.99 M parameters.
"""
from __future__ import annotations

from ..nn import (Sequential, SpatialConvolution, SpatialBatchNormalization, ReLU, Dropout, SpatialMaxPooling, View,
                  Linear, BatchNormalization, LogSoftMax, Threshold)


def VggForCifar10(class_num: int = 10, has_dropout: bool = True):
    m = Sequential()

    def conv_bn_relu(n_in, n_out):
        m.add(SpatialConvolution(n_in, n_out, 3, 3, 1, 1, 1, 1))
        m.add(SpatialBatchNormalization(n_out, 1e-3))
        m.add(ReLU(True))

    conv_bn_relu(3, 64)
    if has_dropout:
        m.add(Dropout(0.3))
    conv_bn_relu(64, 64)
    m.add(SpatialMaxPooling(2, 2, 2, 2).ceil())
    conv_bn_relu(64, 128)
    if has_dropout:
        m.add(Dropout(0.4))
    conv_bn_relu(128, 128)
    m.add(SpatialMaxPooling(2, 2, 2, 2).ceil())
    conv_bn_relu(128, 256)
    if has_dropout:
        m.add(Dropout(0.4))
    conv_bn_relu(256, 256)
    if has_dropout:
        m.add(Dropout(0.4))
    conv_bn_relu(256, 256)
    m.add(SpatialMaxPooling(2, 2, 2, 2).ceil())
    conv_bn_relu(256, 512)
    if has_dropout:
        m.add(Dropout(0.4))
    conv_bn_relu(512, 512)
    if has_dropout:
        m.add(Dropout(0.4))
    conv_bn_relu(512, 512)
    m.add(SpatialMaxPooling(2, 2, 2, 2).ceil())
    conv_bn_relu(512, 512)
    if has_dropout:
        m.add(Dropout(0.4))
    conv_bn_relu(512, 512)
    if has_dropout:
        m.add(Dropout(0.4))
    conv_bn_relu(512, 512)
    m.add(SpatialMaxPooling(2, 2, 2, 2).ceil())
    m.add(View(512))
    classifier = Sequential()
    if has_dropout:
        classifier.add(Dropout(0.5))
    classifier.add(Linear(512, 512))
    classifier.add(BatchNormalization(512))
    classifier.add(ReLU(True))
    if has_dropout:
        classifier.add(Dropout(0.5))
    classifier.add(Linear(512, class_num))
    classifier.add(LogSoftMax())
    m.add(classifier)
    return m


def _vgg(cfg, class_num, has_dropout=True):
    m = Sequential()
    n_in = 3
    for v in cfg:
        if v == "M":
            m.add(SpatialMaxPooling(2, 2, 2, 2))
        else:
            m.add(SpatialConvolution(n_in, v, 3, 3, 1, 1, 1, 1))
            m.add(ReLU(True))
            n_in = v
    m.add(View(512 * 7 * 7))
    m.add(Linear(512 * 7 * 7, 4096))
    m.add(Threshold(0, 1e-6))
    if has_dropout:
        m.add(Dropout(0.5))
    m.add(Linear(4096, 4096))
    m.add(Threshold(0, 1e-6))
    if has_dropout:
        m.add(Dropout(0.5))
    m.add(Linear(4096, class_num))
    m.add(LogSoftMax())
    return m


def Vgg_16(class_num: int = 1000, has_dropout: bool = True):
    return _vgg([64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"],
                class_num, has_dropout)


def Vgg_19(class_num: int = 1000, has_dropout: bool = True):
    return _vgg([64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512,
                 "M"], class_num, has_dropout)
