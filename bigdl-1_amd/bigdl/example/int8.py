"""Int8 ImageNet inference (``DL/example/mkldnn/int8/{GenerateInt8Scales,ImageNetInference,Utils}.scala``).

* ``genscales -f <imagenet> -m model.bigdl [-b 128] [-n 1]``: the model (as a Graph, evaluation
  mode) gets input / output dimension mask 0 and weight mask 1 (per output channel), ``numOfBatch``
  validation batches run through it with ``calcScales`` after each forward, and the model with its
  recorded scales is saved as ``<model>.quantized.bigdl``.
* ``inference -f <imagenet> -m model.bigdl [-b 128]``: the model is quantized (``quantize()`` —
  int8 weights and activations on the ``mfma_i32_16x16x64_i8`` GEMM / conv kernels on a GPU,
  exact int32 accumulation on the host) and evaluated with Top-1 / Top-5 on the validation set.

The validation set is ``<folder>/val`` Hadoop sequence files of BGR records (the format of
``bigdl.models.utils.seqfile_generator``), centre-cropped to ``--imageSize`` (224) and normalised with
the ImageNet mean / std, as ``ImageNetDataSet.valDataSet``.
"""
from __future__ import annotations

import argparse
import logging
import os
import sys

import numpy as np
import torch

log = logging.getLogger("bigdl.example.int8")

MEAN = (0.485 * 255, 0.456 * 255, 0.406 * 255)
STD = (0.229 * 255, 0.224 * 255, 0.225 * 255)


def val_batches(folder: str, image_size: int, batch_size: int, limit_batches=None):
    """[MiniBatch] of the centre-cropped, normalised validation images (RGB, NCHW, 1-based labels)."""
    from ..dataset.core import MiniBatch
    from ..dataset.seqfile import SeqFileFolder
    path = os.path.join(folder, "val") if os.path.isdir(os.path.join(folder, "val")) else folder
    imgs, labels = SeqFileFolder.to_arrays(path)
    n, H, W, _ = imgs.shape
    y0, x0 = (H - image_size) // 2, (W - image_size) // 2
    if y0 < 0 or x0 < 0:
        raise ValueError(f"images {H}x{W} are smaller than the {image_size} crop")
    mean = torch.tensor(MEAN).view(1, 3, 1, 1)
    std = torch.tensor(STD).view(1, 3, 1, 1)
    out = []
    for s in range(0, n, batch_size):
        if limit_batches is not None and len(out) >= limit_batches:
            break
        crop = imgs[s:s + batch_size, y0:y0 + image_size, x0:x0 + image_size, ::-1]  # BGR → RGB
        x = (torch.from_numpy(np.ascontiguousarray(crop)).permute(0, 3, 1, 2).float() - mean) / std
        out.append(MiniBatch(x, torch.from_numpy(labels[s:s + batch_size]).float()))
    return out


def generate_int8_scales(model, model_name: str, batches):
    """``genereateInt8Scales``: masks, forward + calcScales over the sample batches."""
    model.evaluate()
    model.setInputDimMask(0, True)
    model.setOutputDimMask(0, True)
    model.setWeightDimMask(1, True)
    log.info(f"Generate the scales for {model_name} ...")
    with torch.no_grad():
        for b in batches:
            x = b.getInput()
            model.forward(x)
            model.calcScales(x)
    model.clearState()
    log.info(f"Generate the scales for {model_name} done.")
    return model


def save_quantized_model(model, model_name: str) -> str:
    prefix = model_name[:-len(".bigdl")] if model_name.endswith(".bigdl") else model_name
    name = prefix + ".quantized.bigdl"
    log.info(f"Save the quantized model {name} ...")
    model.saveModule(name, over_write=True)
    return name


def _parser():
    ap = argparse.ArgumentParser(description="BigDL int8 ImageNet example")
    ap.add_argument("cmd", choices=["genscales", "inference"])
    ap.add_argument("-f", "--folder", default="./")
    ap.add_argument("-m", "--model", required=True)
    ap.add_argument("-b", "--batchSize", type=int, default=128)
    ap.add_argument("-n", "--numOfBatch", type=int, default=1)
    ap.add_argument("--imageSize", type=int, default=224)
    return ap


def main(argv=None):
    a = _parser().parse_args(argv)
    from ..nn.module import Module
    from ..utils.engine import Engine
    Engine.init()
    if a.cmd == "genscales":
        model = Module.loadModule(a.model).toGraph()
        batches = val_batches(a.folder, a.imageSize, a.batchSize, limit_batches=a.numOfBatch)
        generate_int8_scales(model, a.model, batches)
        return save_quantized_model(model, a.model)
    from ..optim.validation import Top1Accuracy, Top5Accuracy
    model = Module.loadModule(a.model).quantize()
    model.evaluate()
    dev = Engine.device()
    model.to(dev)
    batches = val_batches(a.folder, a.imageSize, a.batchSize)
    if dev.type == "cuda":
        batches = [b.to(dev) for b in batches]
    res = model.evaluate(batches, [Top1Accuracy(), Top5Accuracy()])
    for r, m in res:
        print(f"{m} is {r}")
    return res


if __name__ == "__main__":
    main(sys.argv[1:])
