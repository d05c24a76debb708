"""DataFrame (dlframes) image examples (``DL/example/dlframes/imageInference/ImageInference.scala``,
``imageTransferLearning/ImageTransferLearning.scala``).

* ``inference``: images of ``--folder`` → Resize(256) → CenterCrop(224) → ChannelNormalize(123,
  117, 104) → MatToTensor → sample; a Caffe model (``--caffeDefPath`` / ``--modelPath``) wrapped in a
  ``DLClassifierModel`` adds the 1-based predicted class of every image.
* ``transfer``: label = 1 if the file name contains "cat" else 2; an 80/20 split; a ``Pipeline`` of
  the Caffe model as a ``DLModel`` featurizer (its 1000-way output) and a ``DLClassifier`` over
  ``Linear(1000, 2) → LogSoftMax`` (ClassNLL, lr 0.003, 20 epochs) is fitted on the training part
  and scored on the validation part with weighted precision.

    python -m bigdl.example.dlframes inference --caffeDefPath deploy.prototxt --modelPath m.caffemodel
        --folder images/ [-b 16]
    python -m bigdl.example.dlframes transfer  --caffeDefPath … --modelPath … --folder images/

``--imageSize`` / ``--resize`` (defaults 224 / 256, the reference's) and ``--featureSize`` (1000) make
the pipeline usable with smaller models.  The DataFrames are pandas (no Spark here).
"""
from __future__ import annotations

import argparse
import sys

import numpy as np


def load_images(path: str, image_size: int = 224, resize: int = 256):
    """DataFrame(imageName, features) of every image under ``path`` (``Utils.loadImages``)."""
    import pandas as pd
    from ..transform.vision.image import ImageFrame
    from ..transform.vision.image.augmentation import CenterCrop, ChannelNormalize, Resize
    from ..transform.vision.image.convertor import ImageFrameToSample, MatToTensor
    frame = ImageFrame.read(path)
    t = Resize(resize, resize) >> CenterCrop(image_size, image_size) >> ChannelNormalize(123, 117, 104, 1, 1, 1) \
        >> MatToTensor() >> ImageFrameToSample()
    frame = frame.transform(t)
    rows = []
    for f in frame.to_local():
        s = f["sample"]
        rows.append({"imageName": f["uri"], "features": np.asarray(s.feature().float().reshape(-1).numpy())})
    return pd.DataFrame(rows, columns=["imageName", "features"])


def _parser():
    ap = argparse.ArgumentParser(description="BigDL dlframes image examples")
    ap.add_argument("cmd", choices=["inference", "transfer"])
    ap.add_argument("--caffeDefPath", required=True)
    ap.add_argument("--modelPath", required=True)
    ap.add_argument("--folder", required=True)
    ap.add_argument("-b", "--batchSize", type=int, default=16)
    ap.add_argument("-e", "--nEpochs", type=int, default=10)
    ap.add_argument("--imageSize", type=int, default=224)
    ap.add_argument("--resize", type=int, default=256)
    ap.add_argument("--featureSize", type=int, default=1000)
    ap.add_argument("--maxEpoch", type=int, default=20, help="classifier epochs (transfer)")
    return ap


def image_inference(a):
    from ..dlframes import DLClassifierModel
    from ..nn.module import Module
    from ..utils.engine import Engine
    Engine.init()
    df = load_images(a.folder, a.imageSize, a.resize)
    print(df.head(10))
    model = Module.loadCaffeModel(a.caffeDefPath, a.modelPath)
    dl = DLClassifierModel(model, [3, a.imageSize, a.imageSize]).setBatchSize(a.batchSize) \
        .setFeaturesCol("features").setPredictionCol("prediction")
    out = dl.transform(df)
    print(out[["imageName", "prediction"]].to_string())
    return out


def image_transfer_learning(a):
    from ..dlframes import DLClassifier, DLModel, Pipeline, weighted_precision
    from ..nn import ClassNLLCriterion, Linear, LogSoftMax, Sequential
    from ..nn.module import Module
    from ..utils.engine import Engine
    Engine.init()
    df = load_images(a.folder, a.imageSize, a.resize)
    df["label"] = [1.0 if "cat" in str(n) else 2.0 for n in df["imageName"]]
    df = df.rename(columns={"features": "imageFeatures"})
    rng = np.random.default_rng(1)
    is_val = rng.random(len(df)) < 0.20
    val, train = df[is_val].reset_index(drop=True), df[~is_val].reset_index(drop=True)
    loaded = Module.loadCaffeModel(a.caffeDefPath, a.modelPath)
    featurizer = DLModel(loaded, [3, a.imageSize, a.imageSize]).setBatchSize(a.batchSize) \
        .setFeaturesCol("imageFeatures").setPredictionCol("features")
    lr_model = Sequential().add(Linear(a.featureSize, 2)).add(LogSoftMax())
    classifier = DLClassifier(lr_model, ClassNLLCriterion(), [a.featureSize]).setLearningRate(0.003) \
        .setBatchSize(a.batchSize).setMaxEpoch(a.maxEpoch)
    model = Pipeline().setStages([featurizer, classifier]).fit(train)
    pred = model.transform(val if len(val) else train)
    print(pred[["imageName", "label", "prediction"]].to_string())
    score = weighted_precision(pred)
    print(f"evaluation result on validationDF: {score}")
    return pred, score


def main(argv=None):
    a = _parser().parse_args(argv)
    return image_inference(a) if a.cmd == "inference" else image_transfer_learning(a)


if __name__ == "__main__":
    main(sys.argv[1:])
