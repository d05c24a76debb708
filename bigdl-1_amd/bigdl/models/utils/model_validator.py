"""Pretrained-model validator (``DL/example/loadmodel/ModelValidator.scala:60-150`` and its
preprocessors ``DatasetUtil.scala``): load a Caffe / Torch7 / BigDL ImageNet model and report
Top-1 / Top-5 accuracy over a class-per-subfolder image folder.

    python -m bigdl.models.utils.model_validator -f /data/val -m inception -t caffe \\
        --caffeDefPath deploy.prototxt --modelPath bvlc_googlenet.caffemodel -b 64

Preprocessing per model (the reference's AlexNet / Inception / ResNet / VGG preprocessors):
shorter side → 256, center crop (227 AlexNet, 224 otherwise), then
  * alexnet  : BGR, minus the mean image (``--meanFile``, .npy [3,H,W] BGR or per-channel [3])
  * inception: BGR 0-255 minus (104, 117, 123)
  * vgg16    : BGR 0-255 minus (104, 117, 123)
  * resnet   : RGB / 255, ImageNet mean / std normalisation
Labels are the 1-based sorted subfolder indices (``DataSet.ImageFolder``).
"""
from __future__ import annotations

import argparse
import sys
from typing import List, Optional

import numpy as np
import torch

_BGR_MEAN = (104.0, 117.0, 123.0)
_RGB_MEAN, _RGB_STD = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)


def preprocess(img_bgr01: torch.Tensor, model_name: str, mean: Optional[np.ndarray] = None) -> torch.Tensor:
    """[H, W, 3] BGR in [0, 1] (``LocalImgReader`` output) → [3, crop, crop] network input."""
    from ...transform.vision.image.augmentation import resize_mat
    m = img_bgr01.float()
    h, w = m.shape[0], m.shape[1]
    s = 256.0 / min(h, w)
    m = resize_mat(m, int(round(h * s)), int(round(w * s)))
    crop = 227 if model_name == "alexnet" else 224
    y0, x0 = (m.shape[0] - crop) // 2, (m.shape[1] - crop) // 2
    m = m[y0:y0 + crop, x0:x0 + crop].permute(2, 0, 1).contiguous()  # [3, crop, crop] BGR
    if model_name == "resnet":
        rgb = m.flip(0)
        return (rgb - torch.tensor(_RGB_MEAN).view(3, 1, 1)) / torch.tensor(_RGB_STD).view(3, 1, 1)
    m = m * 255.0
    if model_name == "alexnet":
        if mean is None:
            raise ValueError("alexnet needs --meanFile")
        mt = torch.from_numpy(np.asarray(mean, dtype=np.float32))
        if mt.dim() == 1:
            return m - mt.view(3, 1, 1)
        my, mx = (mt.shape[1] - crop) // 2, (mt.shape[2] - crop) // 2
        return m - mt[:, my:my + crop, mx:mx + crop]
    return m - torch.tensor(_BGR_MEAN).view(3, 1, 1)


def load_model(model_type: str, model_path: str, caffe_def: Optional[str] = None):
    from ...nn.module import Module
    t = model_type.lower()
    if t == "caffe":
        if not caffe_def:
            raise ValueError("caffe models need --caffeDefPath")
        return Module.loadCaffeModel(caffe_def, model_path)
    if t == "torch":
        return Module.loadTorch(model_path)
    if t == "bigdl":
        return Module.loadModule(model_path)
    raise ValueError("only torch, caffe or bigdl supported")


def validate(model, folder: str, model_name: str, batch_size: int = 32, mean_file: Optional[str] = None):
    """[(result, method)] for Top1Accuracy and Top5Accuracy over the folder."""
    from ...dataset import Sample
    from ...dataset.image import LocalImageFiles, LocalImgReader
    from ...optim.validation import Top1Accuracy, Top5Accuracy
    mean = np.load(mean_file, allow_pickle=False) if mean_file else None
    samples: List = []
    for rec in LocalImgReader().apply(iter(LocalImageFiles.read_paths(folder))):
        samples.append(Sample.from_ndarray(preprocess(rec.content, model_name.lower(), mean).numpy(),
                                           np.array([rec.label()], dtype=np.float32)))
    return model.evaluate(samples, [Top1Accuracy(), Top5Accuracy()], batch_size)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m bigdl.models.utils.model_validator",
                                 description="BigDL Load Model Example")
    ap.add_argument("-f", "--folder", required=True, help="where you put your local image files")
    ap.add_argument("-m", "--modelName", required=True, help="alexnet | inception | resnet | vgg16")
    ap.add_argument("-t", "--modelType", required=True, help="torch, caffe or bigdl")
    ap.add_argument("--caffeDefPath")
    ap.add_argument("--modelPath", required=True)
    ap.add_argument("-b", "--batchSize", type=int, default=32)
    ap.add_argument("--meanFile")
    a = ap.parse_args(argv)
    model = load_model(a.modelType, a.modelPath, a.caffeDefPath)
    print(model)
    for result, method in validate(model, a.folder, a.modelName, a.batchSize, a.meanFile):
        print(f"{method} is {result}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
