"""Load a pre-trained ImageNet model and validate it (``DL/example/loadmodel/{ModelValidator,
AlexNet,DatasetUtil}.scala``).

``--modelType caffe|torch|bigdl`` with ``--modelName``: caffe ``alexnet`` (mean-file preprocessing,
227 crop) or ``inception`` (224 crop, BGR minus (123, 117, 104)); torch ``resnet`` (ImageNet mean /
std); bigdl ``resnet`` (minus (104, 117, 123), ×1/128) or ``vgg16``.  The validation set is
``<folder>/val`` (or ``<folder>``) Hadoop sequence files of BGR records (``SeqFileFolder``); the
result is Top-1 / Top-5 accuracy.  This module also holds the example's two AlexNet definitions:
``AlexNet_OWT`` (one-weird-trick, 64-192-384-256-256) as a Sequential or a Graph, and the Caffe
``AlexNet`` (LRN, grouped conv2/4/5).

    python -m bigdl.example.loadmodel -t caffe -m alexnet -f <seq folder> --caffeDefPath
        deploy.prototxt --modelPath bvlc_alexnet.caffemodel --meanFile mean.txt [-b 32]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch


# ------------------------------------------------------------------------------------------ models
def AlexNet_OWT(class_num: int, has_dropout: bool = True, first_layer_propagate_back: bool = False):
    """``AlexNet_OWT.apply``: the one-weird-trick AlexNet as a Sequential."""
    from ..nn import Dropout, Linear, LogSoftMax, ReLU, Sequential, SpatialConvolution, SpatialMaxPooling, View
    m = Sequential()
    m.add(SpatialConvolution(3, 64, 11, 11, 4, 4, 2, 2, 1, first_layer_propagate_back).setName("conv1"))
    m.add(ReLU(True).setName("relu1")).add(SpatialMaxPooling(3, 3, 2, 2).setName("pool1"))
    m.add(SpatialConvolution(64, 192, 5, 5, 1, 1, 2, 2).setName("conv2"))
    m.add(ReLU(True).setName("relu2")).add(SpatialMaxPooling(3, 3, 2, 2).setName("pool2"))
    m.add(SpatialConvolution(192, 384, 3, 3, 1, 1, 1, 1).setName("conv3")).add(ReLU(True).setName("relu3"))
    m.add(SpatialConvolution(384, 256, 3, 3, 1, 1, 1, 1).setName("conv4")).add(ReLU(True).setName("relu4"))
    m.add(SpatialConvolution(256, 256, 3, 3, 1, 1, 1, 1).setName("conv5")).add(ReLU(True).setName("relu5"))
    m.add(SpatialMaxPooling(3, 3, 2, 2).setName("poo5")).add(View([256 * 6 * 6]).setName("view"))
    m.add(Linear(256 * 6 * 6, 4096).setName("fc6")).add(ReLU(True).setName("relu6"))
    if has_dropout:
        m.add(Dropout(0.5).setName("drop6"))
    m.add(Linear(4096, 4096).setName("fc7")).add(ReLU(True).setName("relu7"))
    if has_dropout:
        m.add(Dropout(0.5).setName("drop7"))
    m.add(Linear(4096, class_num).setName("fc8")).add(LogSoftMax().setName("logsoftmax"))
    return m


def AlexNet_OWT_graph(class_num: int, has_dropout: bool = True, first_layer_propagate_back: bool = False):
    """``AlexNet_OWT.graph``: the same network as a Graph of named nodes."""
    from ..nn import Dropout, Graph, Linear, LogSoftMax, ReLU, SpatialConvolution, SpatialMaxPooling, View
    conv1 = SpatialConvolution(3, 64, 11, 11, 4, 4, 2, 2, 1, first_layer_propagate_back).setName("conv1").inputs()
    x = ReLU(True).setName("relu1").inputs(conv1)
    x = SpatialMaxPooling(3, 3, 2, 2).setName("pool1").inputs(x)
    x = ReLU(True).setName("relu2").inputs(SpatialConvolution(64, 192, 5, 5, 1, 1, 2, 2).setName("conv2").inputs(x))
    x = SpatialMaxPooling(3, 3, 2, 2).setName("pool2").inputs(x)
    for i, (ci, co) in enumerate(((192, 384), (384, 256), (256, 256)), start=3):
        x = ReLU(True).setName(f"relu{i}").inputs(
            SpatialConvolution(ci, co, 3, 3, 1, 1, 1, 1).setName(f"conv{i}").inputs(x))
    x = View([256 * 6 * 6]).inputs(SpatialMaxPooling(3, 3, 2, 2).setName("poo5").inputs(x))
    x = ReLU(True).setName("relu6").inputs(Linear(256 * 6 * 6, 4096).setName("fc6").inputs(x))
    if has_dropout:
        x = Dropout(0.5).setName("drop6").inputs(x)
    x = ReLU(True).setName("relu7").inputs(Linear(4096, 4096).setName("fc7").inputs(x))
    if has_dropout:
        x = Dropout(0.5).setName("drop7").inputs(x)
    out = LogSoftMax().inputs(Linear(4096, class_num).setName("fc8").inputs(x))
    return Graph([conv1], [out])


def AlexNet(class_num: int, has_dropout: bool = True):
    """``AlexNet.apply``: the Caffe BVLC AlexNet (96-256-384-384-256, LRN after conv1/2, conv2/4/5
    in two groups)."""
    from ..nn import (Dropout, Linear, LogSoftMax, ReLU, Sequential, SpatialConvolution, SpatialCrossMapLRN,
                      SpatialMaxPooling, View)
    m = Sequential()
    m.add(SpatialConvolution(3, 96, 11, 11, 4, 4, 0, 0, 1, False).setName("conv1")).add(ReLU(True).setName("relu1"))
    m.add(SpatialCrossMapLRN(5, 0.0001, 0.75).setName("norm1")).add(SpatialMaxPooling(3, 3, 2, 2).setName("pool1"))
    m.add(SpatialConvolution(96, 256, 5, 5, 1, 1, 2, 2, 2).setName("conv2")).add(ReLU(True).setName("relu2"))
    m.add(SpatialCrossMapLRN(5, 0.0001, 0.75).setName("norm2")).add(SpatialMaxPooling(3, 3, 2, 2).setName("pool2"))
    m.add(SpatialConvolution(256, 384, 3, 3, 1, 1, 1, 1).setName("conv3")).add(ReLU(True).setName("relu3"))
    m.add(SpatialConvolution(384, 384, 3, 3, 1, 1, 1, 1, 2).setName("conv4")).add(ReLU(True).setName("relu4"))
    m.add(SpatialConvolution(384, 256, 3, 3, 1, 1, 1, 1, 2).setName("conv5")).add(ReLU(True).setName("relu5"))
    m.add(SpatialMaxPooling(3, 3, 2, 2).setName("pool5")).add(View([256 * 6 * 6]).setName("view"))
    m.add(Linear(256 * 6 * 6, 4096).setName("fc6")).add(ReLU(True).setName("relu6"))
    if has_dropout:
        m.add(Dropout(0.5).setName("drop6"))
    m.add(Linear(4096, 4096).setName("fc7")).add(ReLU(True).setName("relu7"))
    if has_dropout:
        m.add(Dropout(0.5).setName("drop7"))
    m.add(Linear(4096, class_num).setName("fc8")).add(LogSoftMax().setName("loss"))
    return m


# ------------------------------------------------------------------------------------------ data
class _Rescale:
    """BGR image content ×``k`` (the sequence-file reader yields pixels / 255; the Caffe
    preprocessors work on 0-255 values) and optional resize to ``size`` (``BytesToBGRImg(1, w, h)``)."""

    def __init__(self, k: float, size=None):
        self.k, self.size = k, size

    def __call__(self, it):
        from ..transform.vision.image.augmentation import resize_mat
        for img in it:
            c = img.content * self.k
            if self.size is not None and tuple(c.shape[:2]) != tuple(self.size):
                c = resize_mat(c, self.size[0], self.size[1])
            img.content = c
            yield img


def _chain(ds, *stages):
    from ..dataset.core import Transformer

    class _F(Transformer):
        def __init__(self, f):
            self.f = f

        def apply(self, it):
            return self.f(it)
    for s in stages:
        ds = ds >> (s if isinstance(s, Transformer) else _F(s))
    return ds


def create_means(mean_file: str) -> torch.Tensor:
    """Pixel-level mean image, one value per line in H·W·C order (``createMeans``)."""
    with open(mean_file) as f:
        return torch.tensor([float(l) for l in f if l.strip()], dtype=torch.float32)


def _val_path(folder):
    return os.path.join(folder, "val") if os.path.isdir(os.path.join(folder, "val")) else folder


def alexnet_preprocessor(path, batch, mean_file, size=256, crop=227):
    """``AlexNetPreprocessor``: 0-255 BGR 256×256, minus the mean image, centre 227 crop, BGR batch."""
    from ..dataset.core import DataSet
    from ..dataset.image import BGRImgCropper, BGRImgPixelNormalizer, BGRImgToBatch
    return _chain(DataSet.SeqFileFolder.files(_val_path(path), 1000), _Rescale(255.0, (size, size)),
                  BGRImgPixelNormalizer(create_means(mean_file)), BGRImgCropper(crop, crop, "center"),
                  BGRImgToBatch(batch, False))


def inception_preprocessor(path, batch, crop=224):
    """``InceptionPreprocessor``: 0-255 BGR, centre 224 crop, minus (R 123, G 117, B 104)."""
    from ..dataset.core import DataSet
    from ..dataset.image import BGRImgCropper, BGRImgNormalizer, BGRImgToBatch
    return _chain(DataSet.SeqFileFolder.files(_val_path(path), 1000), _Rescale(255.0),
                  BGRImgCropper(crop, crop, "center"), BGRImgNormalizer(123, 117, 104, 1, 1, 1),
                  BGRImgToBatch(batch, False))


def resnet_preprocessor(path, batch, bigdl_model=False, crop=224):
    """``ResNetPreprocessor``: Torch models take [0, 1] RGB with the ImageNet mean / std; BigDL
    models take 0-255 BGR values minus ``ChannelScaledNormalizer(104, 117, 123, 1/128)``."""
    from ..dataset.core import DataSet
    from ..dataset.image import BGRImgCropper, BGRImgNormalizer, BGRImgToBatch
    if bigdl_model:
        s = 0.0078125
        return _chain(DataSet.SeqFileFolder.files(_val_path(path), 1000), _Rescale(255.0, (256, 256)),
                      BGRImgCropper(crop, crop, "center"),
                      BGRImgNormalizer(104, 117, 123, 1 / s, 1 / s, 1 / s), BGRImgToBatch(batch, False))
    return _chain(DataSet.SeqFileFolder.files(_val_path(path), 1000), BGRImgCropper(crop, crop, "center"),
                  BGRImgNormalizer(0.485, 0.456, 0.406, 0.229, 0.224, 0.225), BGRImgToBatch(batch, True))


def vgg_preprocessor(path, batch, crop=224):
    """``VGGPreprocessor``: 0-255 BGR 256×256, centre 224 crop, minus (123, 117, 104)."""
    from ..dataset.core import DataSet
    from ..dataset.image import BGRImgCropper, BGRImgNormalizer, BGRImgToBatch
    return _chain(DataSet.SeqFileFolder.files(_val_path(path), 1000), _Rescale(255.0, (256, 256)),
                  BGRImgCropper(crop, crop, "center"), BGRImgNormalizer(123, 117, 104, 1, 1, 1),
                  BGRImgToBatch(batch, False))


# ------------------------------------------------------------------------------------------ main
def _parser():
    ap = argparse.ArgumentParser(description="BigDL Load Model Example")
    ap.add_argument("-t", "--modelType", required=True, choices=["torch", "caffe", "bigdl"])
    ap.add_argument("-m", "--modelName", required=True, type=str.lower)
    ap.add_argument("-f", "--folder", default="./", help="sequence files of the validation images")
    ap.add_argument("--caffeDefPath")
    ap.add_argument("--modelPath", required=True)
    ap.add_argument("-b", "--batchSize", type=int, default=32)
    ap.add_argument("--meanFile")
    return ap


def _load(a):
    from ..nn.module import Module
    if a.modelType == "caffe":
        if not a.caffeDefPath:
            raise ValueError("caffe models need --caffeDefPath")
        return Module.loadCaffeModel(a.caffeDefPath, a.modelPath)
    if a.modelType == "torch":
        return Module.loadTorch(a.modelPath)
    return Module.loadModule(a.modelPath)


def main(argv=None):
    a = _parser().parse_args(argv)
    from ..optim.validation import Top1Accuracy, Top5Accuracy
    from ..utils.engine import Engine
    Engine.init()
    key = (a.modelType, a.modelName)
    if key == ("caffe", "alexnet"):
        if not a.meanFile:
            raise ValueError("alexnet needs --meanFile")
        data = alexnet_preprocessor(a.folder, a.batchSize, a.meanFile)
    elif key == ("caffe", "inception"):
        data = inception_preprocessor(a.folder, a.batchSize)
    elif key == ("torch", "resnet"):
        data = resnet_preprocessor(a.folder, a.batchSize)
    elif key == ("bigdl", "resnet"):
        data = resnet_preprocessor(a.folder, a.batchSize, bigdl_model=True)
    elif key == ("bigdl", "vgg16"):
        data = vgg_preprocessor(a.folder, a.batchSize)
    else:
        raise ValueError(f"{a.modelType} {a.modelName} is not supported in this example")
    model = _load(a)
    model.evaluate()
    batches = list(data.data(train=False))
    res = model.evaluate(batches, [Top1Accuracy(), Top5Accuracy()])
    for r, m in res:
        print(f"{m} is {r}")
    return res


if __name__ == "__main__":
    main(sys.argv[1:])
