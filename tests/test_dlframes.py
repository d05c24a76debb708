"""dlframes (``DL/dlframes``): DLEstimator/DLClassifier fit + transform on pandas DataFrames,
DLImageReader / DLImageTransformer (``DLClassifierSpec``, ``DLEstimatorSpec``, ``DLImageReaderSpec``)."""
import numpy as np
import pandas as pd
import torch

from bigdl.dlframes import DLEstimator, DLClassifier, DLClassifierModel, DLModel, DLImageReader, DLImageTransformer
from bigdl.nn import Sequential, Linear, LogSoftMax, MSECriterion, ClassNLLCriterion, ReLU


def _blobs(n=64):
    rng = np.random.RandomState(0)
    a = rng.randn(n // 2, 2) + 2
    b = rng.randn(n // 2, 2) - 2
    x = np.concatenate([a, b]).astype(np.float32)
    y = np.concatenate([np.ones(n // 2), 2 * np.ones(n // 2)])
    return pd.DataFrame({"features": list(x), "label": y})


def test_dl_classifier_fit_transform():
    torch.manual_seed(0)
    df = _blobs()
    model = Sequential().add(Linear(2, 8)).add(ReLU()).add(Linear(8, 2)).add(LogSoftMax())
    est = DLClassifier(model, ClassNLLCriterion(), [2]).setBatchSize(16).setMaxEpoch(20).setLearningRate(0.2)
    fitted = est.fit(df)
    assert isinstance(fitted, DLClassifierModel)
    out = fitted.transform(df)
    acc = float((out["prediction"].values == df["label"].values).mean())
    assert acc > 0.9


def test_dl_estimator_regression():
    torch.manual_seed(0)
    x = np.random.RandomState(1).randn(32, 3).astype(np.float32)
    y = (x @ np.array([[1.0], [-2.0], [0.5]], dtype=np.float32)).astype(np.float32)
    df = pd.DataFrame({"features": list(x), "label": list(y)})
    est = DLEstimator(Linear(3, 1), MSECriterion(), [3], [1]).setBatchSize(8).setMaxEpoch(60).setLearningRate(0.1)
    m = est.fit(df)
    assert isinstance(m, DLModel)
    pred = np.array([p[0] for p in m.transform(df)["prediction"]])
    assert np.abs(pred - y[:, 0]).max() < 0.1


def test_dl_image_reader_and_transformer(tmp_path):
    from PIL import Image
    for i in range(2):
        Image.fromarray((np.ones((10, 12, 3)) * (i * 50)).astype(np.uint8)).save(tmp_path / f"im{i}.png")
    df = DLImageReader.readImages(str(tmp_path))
    assert len(df) == 2 and df["image"][0]["height"] == 10 and df["image"][0]["nChannels"] == 3
    from bigdl.transform.vision.image import Resize, ChannelNormalize, Pipeline
    t = DLImageTransformer(Pipeline([Resize(6, 5), ChannelNormalize(10.0, 10.0, 10.0)]))
    out = t.transform(df)
    r = out["output"][1]
    assert (r["height"], r["width"]) == (6, 5)
    data = np.frombuffer(r["data"], dtype=np.float32)
    assert np.allclose(data, 40.0)
