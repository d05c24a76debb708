"""ML-pipeline estimators (``DL/example/MLPipeline``): DLClassifier on LeNet over an MNIST-shaped
DataFrame (DLClassifierLeNet.scala), DLClassifier logistic regression (DLClassifierLogisticRegression
.scala) and a multi-label DLEstimator regression (DLEstimatorMultiLabelLR.scala), each fit →
transform on a pandas DataFrame."""
from __future__ import annotations

import argparse
import sys

import numpy as np


def logistic_regression(n=200, seed=0):
    import pandas as pd
    from ..dlframes import DLClassifier
    from ..nn import ClassNLLCriterion, Linear, LogSoftMax, Sequential
    g = np.random.default_rng(seed)
    x = g.normal(0, 1, (n, 2)).astype(np.float32)
    y = (x[:, 0] + x[:, 1] > 0).astype(np.float32) + 1
    df = pd.DataFrame({"features": list(x), "label": y})
    model = Sequential().add(Linear(2, 2)).add(LogSoftMax())
    est = DLClassifier(model, ClassNLLCriterion(), [2]).setLabelCol("label").setBatchSize(20).setMaxEpoch(20)
    est.setLearningRate(0.5)
    out = est.fit(df).transform(df)
    return float((out["prediction"].to_numpy() == y).mean())


def multilabel_regression(n=100, seed=0):
    import pandas as pd
    from ..dlframes import DLEstimator
    from ..nn import Linear, MSECriterion, Sequential
    g = np.random.default_rng(seed)
    x = g.normal(0, 1, (n, 2)).astype(np.float32)
    y = np.stack([x[:, 0] * 2, x[:, 1] - 1], 1).astype(np.float32)
    df = pd.DataFrame({"features": list(x), "label": list(y)})
    est = DLEstimator(Sequential().add(Linear(2, 2)), MSECriterion(), [2], [2]).setBatchSize(10).setMaxEpoch(30)
    est.setLearningRate(0.1)
    out = est.fit(df).transform(df)
    pred = np.stack(out["prediction"].to_numpy())
    return float(np.abs(pred - y).mean())


def lenet(n=256, seed=0):
    import pandas as pd
    from ..dlframes import DLClassifier
    from ..models.lenet import LeNet5
    from ..models.train.common import synthetic_images
    from ..nn import ClassNLLCriterion
    x, y = synthetic_images(n, 28, 28, 1, 10, seed)
    feats = [((im[..., 0].astype(np.float32) - 33.3) / 78.6).reshape(-1) for im in x]
    df = pd.DataFrame({"features": feats, "label": y})
    est = DLClassifier(LeNet5(10), ClassNLLCriterion(), [28, 28]).setBatchSize(32).setMaxEpoch(3)
    est.setLearningRate(0.05)
    out = est.fit(df).transform(df)
    return float((out["prediction"].to_numpy() == y).mean())


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--which", default="all", choices=["all", "lr", "multilabel", "lenet"])
    a = ap.parse_args(argv)
    from ..utils.engine import Engine
    Engine.init()
    res = {}
    if a.which in ("all", "lr"):
        res["logistic_regression_accuracy"] = logistic_regression()
    if a.which in ("all", "multilabel"):
        res["multilabel_mae"] = multilabel_regression()
    if a.which in ("all", "lenet"):
        res["lenet_accuracy"] = lenet()
    print(res)
    return res


if __name__ == "__main__":
    main(sys.argv[1:])
