"""The Keras backend path (pyspark/bigdl/keras/backend.py + optimization.py): a compiled Keras
model object is converted (definition, weights, loss, optimizer, metrics) and trained / evaluated /
used for prediction on the BigDL engine.  Keras is not installed: a stand-in object implements
the Keras model protocol with a Keras 1.2.2 JSON config (parity with Keras itself unpinned)."""
import json

import numpy as np
import pytest

from bigdl.keras.backend import with_bigdl_backend
from bigdl.keras.optimization import OptimConverter


class _Layer:
    def __init__(self, name, weights):
        self.name, self._w = name, weights

    def get_weights(self):
        return self._w


class SGD:  # class name is what the converter keys on, as with keras.optimizers.SGD
    def __init__(self, lr=0.1, momentum=0.9, decay=0.0, nesterov=False):
        self.lr, self.momentum, self.decay, self.nesterov = lr, momentum, decay, nesterov


class Adam:
    def get_config(self):
        return {"learning_rate": 0.002, "beta_1": 0.8, "beta_2": 0.99, "epsilon": 1e-7, "decay": 0.0}


class _KModel:
    def __init__(self, loss="categorical_crossentropy", optimizer=None, metrics=("accuracy",)):
        rng = np.random.RandomState(0)
        self.W1, self.b1 = (rng.randn(4, 16) * 0.5).astype(np.float32), np.zeros(16, np.float32)
        self.W2, self.b2 = (rng.randn(16, 3) * 0.5).astype(np.float32), np.zeros(3, np.float32)
        self.layers = [_Layer("dense_1", [self.W1, self.b1]), _Layer("dense_2", [self.W2, self.b2])]
        self.loss, self.optimizer, self.metrics = loss, optimizer or SGD(), list(metrics)

    def to_json(self):
        return json.dumps({"class_name": "Sequential", "keras_version": "1.2.2", "config": [
            {"class_name": "Dense", "config": {"name": "dense_1", "output_dim": 16, "activation": "relu",
                                               "batch_input_shape": [None, 4], "bias": True}},
            {"class_name": "Dense", "config": {"name": "dense_2", "output_dim": 3, "activation": "softmax",
                                               "bias": True}}]})


def _data(n=300):
    rng = np.random.RandomState(1)
    x = rng.randn(n, 4).astype(np.float32)
    cls = (x[:, 0] > 0).astype(int) + (x[:, 1] > 0.5).astype(int)
    return x, np.eye(3, dtype=np.float32)[cls], cls


def test_weights_and_predict_match_keras_math():
    km = _KModel()
    w = with_bigdl_backend(km)
    x, _, _ = _data(5)
    h = np.maximum(x @ km.W1 + km.b1, 0) @ km.W2 + km.b2
    ref = np.exp(h - h.max(1, keepdims=True))
    ref /= ref.sum(1, keepdims=True)
    np.testing.assert_allclose(w.predict(x), ref, rtol=1e-5, atol=1e-6)


def test_fit_evaluate_local():
    w = with_bigdl_backend(_KModel())
    x, y, cls = _data()
    before = (w.predict(x).argmax(1) == cls).mean()
    w.fit(x, y, batch_size=30, nb_epoch=15, validation_data=(x[:60], y[:60]))
    acc = w.evaluate(x, y, batch_size=50)[0]
    assert acc > max(0.8, before + 0.1), (before, acc)


def test_optim_and_loss_conversion():
    from bigdl.optim import optim_method as O
    from bigdl.nn import criterion as C
    s = OptimConverter.to_bigdl_optim_method(SGD(lr=0.05, momentum=0.5, nesterov=True))
    assert isinstance(s, O.SGD) and s.learningRate == 0.05 and s.momentum == 0.5 and s.nesterov
    a = OptimConverter.to_bigdl_optim_method(Adam())
    assert isinstance(a, O.Adam) and a.learningRate == pytest.approx(0.002) and a.beta1 == pytest.approx(0.8)
    assert isinstance(OptimConverter.to_bigdl_criterion("mse"), C.MSECriterion)
    assert isinstance(OptimConverter.to_bigdl_criterion("sparse_categorical_crossentropy"), C.ClassNLLCriterion)
    with pytest.raises(ValueError):
        OptimConverter.to_bigdl_criterion("focal")
    with pytest.raises(NotImplementedError):
        with_bigdl_backend(_KModel()).fit(*_data()[:2], callbacks=[object()])
