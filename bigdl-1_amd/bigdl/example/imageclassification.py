"""Batch image prediction with a saved model (``DL/example/imageclassification/ImagePredictor.scala``):
read every image under ``--folder`` (``DLImageReader``), resize / centre-crop / normalise, predict
with ``--model`` (.bigdl) in batches on the device and print ``file → class``."""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch


def predict_folder(model, folder, size=224, batch=32, mean=(123.0, 117.0, 104.0), std=(58.4, 57.1, 57.4)):
    from PIL import Image
    files = sorted(os.path.join(r, f) for r, _, fs in os.walk(folder) for f in fs
                   if f.lower().endswith((".jpg", ".jpeg", ".png", ".bmp")))
    model.evaluate()
    out = []
    for i in range(0, len(files), batch):
        ims = []
        for p in files[i:i + batch]:
            im = Image.open(p).convert("RGB").resize((size, size))
            a = (np.asarray(im, dtype=np.float32) - mean) / std
            ims.append(a.transpose(2, 0, 1))
        x = torch.from_numpy(np.stack(ims).astype(np.float32))
        with torch.no_grad():
            cls = model.forward(x).reshape(len(ims), -1).argmax(-1) + 1
        out += list(zip(files[i:i + batch], cls.tolist()))
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("-f", "--folder", required=True)
    ap.add_argument("--model", required=True)
    ap.add_argument("--imageSize", type=int, default=224)
    ap.add_argument("-b", "--batchSize", type=int, default=32)
    a = ap.parse_args(argv)
    from ..nn.module import Module
    from ..utils.engine import Engine
    Engine.init()
    res = predict_folder(Module.load(a.model), a.folder, a.imageSize, a.batchSize)
    for f, c in res:
        print(f"{f} -> {c}")
    return res


if __name__ == "__main__":
    main(sys.argv[1:])
