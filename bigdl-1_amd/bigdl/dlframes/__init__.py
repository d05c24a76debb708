"""DataFrame estimators/transformers: ``DLEstimator`` / ``DLModel``, ``DLClassifier`` /
``DLClassifierModel``, ``DLImageReader`` and ``DLImageTransformer``.

Reference: ``DL/dlframes/DLEstimator.scala`` (fit: DataFrame rows → Samples → Optimizer, returns
a DLModel), ``DLClassifier.scala`` (1-based class labels, ClassNLL-style criteria; the model's
transform writes the arg-max class), ``DLImageReader.scala`` (image DataFrame with the OpenCV-style
``image`` struct: origin, height, width, nChannels, mode, data) and ``DLImageTransformer.scala``
(apply a vision FeatureTransformer to the ``image`` column); pyspark wrappers in ``PY/dlframes``.

There is no Spark here: the DataFrame is a pandas DataFrame (one row per record; feature / label
columns hold scalars, lists or ndarrays), the fit runs the local or distributed optimizer of this
process, and transform predicts in batches on the model's device.  Column names, setters and
defaults follow the reference (``features``, ``label``, ``prediction``; batch 1, maxEpoch 50,
learningRate 1e-3, SGD).
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence

import numpy as np
import torch


def _pd():
    import pandas as pd
    return pd


class _Params:
    def __init__(self):
        self.featuresCol, self.labelCol, self.predictionCol = "features", "label", "prediction"
        self.batchSize, self.maxEpoch, self.learningRate = 1, 50, 1e-3
        self.optimMethod = None

    def setFeaturesCol(self, v):
        self.featuresCol = v
        return self

    def setLabelCol(self, v):
        self.labelCol = v
        return self

    def setPredictionCol(self, v):
        self.predictionCol = v
        return self

    def setBatchSize(self, v):
        self.batchSize = int(v)
        return self

    def getBatchSize(self):
        return self.batchSize

    def setMaxEpoch(self, v):
        self.maxEpoch = int(v)
        return self

    def getMaxEpoch(self):
        return self.maxEpoch

    def setLearningRate(self, v):
        self.learningRate = float(v)
        return self

    def getLearningRate(self):
        return self.learningRate

    def setOptimMethod(self, m):
        self.optimMethod = m
        return self


def _column(df, col, size: Sequence[int]) -> torch.Tensor:
    rows = [np.asarray(v, dtype=np.float32).reshape(-1) for v in df[col].tolist()]
    t = torch.from_numpy(np.stack(rows)) if rows else torch.zeros(0, int(np.prod(size)))
    return t.reshape(len(rows), *size)


class DLEstimator(_Params):
    """``DLEstimator(model, criterion, featureSize, labelSize)``: ``fit(df)`` → :class:`DLModel`."""

    def __init__(self, model, criterion, feature_size, label_size, bigdl_type="float"):
        super().__init__()
        self.model, self.criterion = model, criterion
        self.featureSize = list(feature_size)
        self.labelSize = list(label_size)

    def _labels(self, df) -> torch.Tensor:
        return _column(df, self.labelCol, self.labelSize)

    def _make_model(self, model):
        return DLModel(model, self.featureSize)

    def fit(self, df):
        from ..dataset import Sample
        from ..optim import SGD, MaxEpoch
        from ..optim.optimizer import Optimizer
        x = _column(df, self.featuresCol, self.featureSize)
        y = self._labels(df)
        samples = [Sample(x[i], y[i]) for i in range(x.shape[0])]
        method = self.optimMethod or SGD(learningrate=self.learningRate)
        opt = Optimizer.create(self.model, samples, self.criterion, MaxEpoch(self.maxEpoch), self.batchSize, method,
                               distributed=False)
        trained = opt.optimize()
        return self._make_model(trained).setFeaturesCol(self.featuresCol).setPredictionCol(
            self.predictionCol).setBatchSize(self.batchSize)

    _fit = fit


class DLModel(_Params):
    """``transform(df)`` appends the model output (as a list per row) in ``predictionCol``."""

    def __init__(self, model, feature_size, bigdl_type="float"):
        super().__init__()
        self.model = model
        self.featureSize = list(feature_size)

    def setFeatureSize(self, v):
        self.featureSize = list(v)
        return self

    def getFeatureSize(self):
        return self.featureSize

    def _predict(self, x: torch.Tensor) -> torch.Tensor:
        from ..optim.predictor import LocalPredictor
        from ..dataset import Sample
        outs = LocalPredictor(self.model, batch_size=max(1, self.batchSize)).predict(
            [Sample(x[i]) for i in range(x.shape[0])])
        return torch.stack([o.float().reshape(-1) for o in outs]) if outs else torch.zeros(0)

    def _format(self, out: torch.Tensor):
        return [row.tolist() for row in out]

    def transform(self, df):
        x = _column(df, self.featuresCol, self.featureSize)
        out = df.copy()
        out[self.predictionCol] = self._format(self._predict(x))
        return out

    _transform = transform

    @staticmethod
    def of(model, feature_size=None, bigdl_type="float"):
        return DLModel(model, feature_size or [])


class DLClassifier(DLEstimator):
    """Classification estimator: scalar 1-based labels, ``labelSize = [1]``."""

    def __init__(self, model, criterion, feature_size, bigdl_type="float"):
        super().__init__(model, criterion, feature_size, [1])

    def _labels(self, df) -> torch.Tensor:
        return torch.tensor([float(np.asarray(v).reshape(-1)[0]) for v in df[self.labelCol].tolist()])

    def _make_model(self, model):
        return DLClassifierModel(model, self.featureSize)


class DLClassifierModel(DLModel):
    """``transform`` writes the 1-based arg-max class (a float, as the reference)."""

    def _format(self, out: torch.Tensor):
        return (out.argmax(-1) + 1).float().tolist()

    @staticmethod
    def of(model, feature_size=None, bigdl_type="float"):
        return DLClassifierModel(model, feature_size or [])


# ------------------------------------------------------------------------------------------------ images
def _image_row(origin: str, mat: np.ndarray) -> dict:
    h, w = mat.shape[:2]
    c = 1 if mat.ndim == 2 else mat.shape[2]
    mode = {1: 0, 3: 16, 4: 24}.get(c, 16)  # OpenCV CV_8UC1 / CV_8UC3 / CV_8UC4 type codes
    return {"origin": origin, "height": h, "width": w, "nChannels": c, "mode": mode,
            "data": np.ascontiguousarray(mat).astype(np.uint8).tobytes()}


def _row_to_mat(row: dict) -> np.ndarray:
    a = np.frombuffer(row["data"], dtype=np.uint8)
    if a.size == row["height"] * row["width"] * row["nChannels"]:
        return a.reshape(row["height"], row["width"], row["nChannels"]).astype(np.float32)
    return np.frombuffer(row["data"], dtype=np.float32).reshape(row["height"], row["width"], row["nChannels"])


class DLImageReader:
    """``DLImageReader.readImages(path)`` → DataFrame with one ``image`` struct column (BGR uint8)."""

    @staticmethod
    def readImages(path: str, sc=None, min_partitions: int = 1, bigdl_type="float"):
        from ..transform.vision.image import ImageFrame
        frame = ImageFrame.read(path)
        rows = []
        for f in frame.to_local().array if hasattr(frame, "to_local") else frame:
            m = f.opencv_mat().detach().cpu().numpy()
            rows.append({"image": _image_row(f.get_uri() or "", m)})
        return _pd().DataFrame(rows, columns=["image"])

    read_images = readImages


class DLImageTransformer(_Params):
    """Apply a vision ``FeatureTransformer`` to the ``image`` column (``DLImageTransformer.scala``);
    the output column holds the transformed image struct (float data after e.g. normalisation)."""

    def __init__(self, transformer, bigdl_type="float"):
        super().__init__()
        self.transformer = transformer
        self.inputCol, self.outputCol = "image", "output"

    def setInputCol(self, v):
        self.inputCol = v
        return self

    def setOutputCol(self, v):
        self.outputCol = v
        return self

    def transform(self, df):
        from ..transform.vision.image import ImageFeature
        outs = []
        for row in df[self.inputCol].tolist():
            f = ImageFeature(image=_row_to_mat(row), uri=row.get("origin"))
            f = self.transformer.transform(f)
            m = f.opencv_mat()
            m = m.detach().cpu().numpy() if isinstance(m, torch.Tensor) else np.asarray(m)
            if m.ndim == 2:
                m = m[..., None]
            outs.append({"origin": row.get("origin"), "height": m.shape[0], "width": m.shape[1],
                         "nChannels": m.shape[2], "mode": 21, "data": m.astype(np.float32).tobytes()})
        out = df.copy()
        out[self.outputCol] = outs
        return out

    _transform = transform


class Pipeline:
    """Spark ML ``Pipeline`` over these stages: ``fit(df)`` runs the stages in order — an estimator
    (``fit``) is fitted on the DataFrame as transformed so far and its model used as the stage — and
    returns a :class:`PipelineModel` whose ``transform`` applies every stage (the reference's
    ImageTransferLearning chains a ``DLModel`` featurizer and a ``DLClassifier``)."""

    def __init__(self, stages=None):
        self.stages = list(stages or [])

    def setStages(self, stages):
        self.stages = list(stages)
        return self

    def getStages(self):
        return self.stages

    def fit(self, df):
        fitted = []
        cur = df
        for i, st in enumerate(self.stages):
            if hasattr(st, "fit") and not hasattr(st, "transform"):
                st = st.fit(cur)
            fitted.append(st)
            if i + 1 < len(self.stages):
                cur = st.transform(cur)
        return PipelineModel(fitted)


class PipelineModel:
    def __init__(self, stages):
        self.stages = list(stages)

    def transform(self, df):
        for st in self.stages:
            df = st.transform(df)
        return df


def weighted_precision(df, label_col="label", prediction_col="prediction") -> float:
    """``MulticlassClassificationEvaluator(metricName = "weightedPrecision")``: per-class precision
    weighted by the class's share of the true labels."""
    y = np.asarray(df[label_col].tolist(), dtype=np.float64).reshape(-1)
    p = np.asarray(df[prediction_col].tolist(), dtype=np.float64).reshape(-1)
    if y.size == 0:
        return 0.0
    total = 0.0
    for c in np.unique(y):
        predicted = p == c
        prec = float((predicted & (y == c)).sum() / predicted.sum()) if predicted.any() else 0.0
        total += prec * float((y == c).sum()) / y.size
    return total
