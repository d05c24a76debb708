"""The runnable examples (reference DL/example/*) on synthetic data, CPU."""
import numpy as np


def test_textclassification_learns_keywords():
    from bigdl.example.textclassification import synthetic_corpus, train
    docs, labels, w2v = synthetic_corpus(320, 4)
    _, acc = train(docs, labels, w2v, 20, 40, 4, 32, 4, lr=0.05)
    assert acc > 0.5, acc  # chance 0.25


def test_udfpredictor_adds_prediction_column():
    from bigdl.example import udfpredictor
    df, picked = udfpredictor.main(["--synthetic", "200", "--seqLen", "40"])
    assert "textType" in df and len(df) == 200
    assert set(df["textType"]) <= {1, 2, 3, 4}
    assert (picked["textType"] == 1).all()


def test_mlpipeline_estimators():
    from bigdl.example import mlpipeline
    assert mlpipeline.logistic_regression() > 0.9
    assert mlpipeline.multilabel_regression() < 0.3


def test_keras_lenet_example_runs():
    from bigdl.example import keras as kex
    res = kex.main(["--synthetic", "128", "-e", "1"])
    assert res is not None


def test_imageclassification_predicts_folder(tmp_path):
    from PIL import Image
    from bigdl.example.imageclassification import predict_folder
    from bigdl.nn import Sequential, SpatialAveragePooling, Reshape, Linear
    for i in range(3):
        Image.fromarray((np.random.default_rng(i).integers(0, 255, (40, 40, 3))).astype(np.uint8)).save(
            tmp_path / f"im{i}.png")
    m = Sequential().add(SpatialAveragePooling(32, 32, 32, 32)).add(Reshape([3])).add(Linear(3, 5))
    res = predict_folder(m, str(tmp_path), size=32, batch=2)
    assert len(res) == 3 and all(1 <= c <= 5 for _, c in res)
