"""Keras 1.2.2 JSON definition + weights import (``pyspark/bigdl/keras/converter.py``).  Keras is not
installed: the JSON configs are written in Keras 1.2.2's format by hand and outputs are compared
with numpy references of the same math (parity against Keras itself is unpinned)."""
import json

import numpy as np
import torch

from bigdl.keras.converter import DefinitionLoader, WeightLoader, load_keras


def _seq_json():
    return {"class_name": "Sequential", "keras_version": "1.2.2", "config": [
        {"class_name": "Dense", "config": {"name": "dense_1", "output_dim": 8, "activation": "relu", "init": "glorot_uniform",
                                           "batch_input_shape": [None, 5], "input_dtype": "float32", "bias": True,
                                           "W_regularizer": None, "b_regularizer": None, "trainable": True}},
        {"class_name": "Dropout", "config": {"name": "dropout_1", "p": 0.3, "trainable": True}},
        {"class_name": "Dense", "config": {"name": "dense_2", "output_dim": 3, "activation": "softmax", "init": "glorot_uniform",
                                           "bias": True, "trainable": True}},
    ]}


def test_sequential_dense_json_and_weights(tmp_path):
    p = tmp_path / "m.json"
    p.write_text(json.dumps(_seq_json()))
    m = DefinitionLoader.from_json_path(str(p))
    rng = np.random.RandomState(0)
    W1, b1 = rng.randn(5, 8).astype(np.float32), rng.randn(8).astype(np.float32)
    W2, b2 = rng.randn(8, 3).astype(np.float32), rng.randn(3).astype(np.float32)
    WeightLoader.load_weights(m, {"dense_1": [W1, b1], "dense_2": [W2, b2]})
    m.evaluate()
    x = rng.randn(4, 5).astype(np.float32)
    h = np.maximum(x @ W1 + b1, 0) @ W2 + b2
    ref = np.exp(h - h.max(1, keepdims=True))
    ref /= ref.sum(1, keepdims=True)
    np.testing.assert_allclose(m.forward(torch.from_numpy(x)).numpy(), ref, rtol=1e-5, atol=1e-6)


def test_conv_tf_ordering_and_npz(tmp_path):
    cfg = {"class_name": "Sequential", "config": [
        {"class_name": "Convolution2D", "config": {"name": "conv", "nb_filter": 4, "nb_row": 3, "nb_col": 3,
                                                   "border_mode": "valid", "dim_ordering": "th", "activation": "linear",
                                                   "subsample": [1, 1], "batch_input_shape": [None, 2, 6, 6],
                                                   "bias": True}},
        {"class_name": "MaxPooling2D", "config": {"name": "pool", "pool_size": [2, 2], "strides": [2, 2],
                                                  "border_mode": "valid", "dim_ordering": "th"}},
        {"class_name": "Flatten", "config": {"name": "flat"}},
    ]}
    p = tmp_path / "c.json"
    p.write_text(json.dumps(cfg))
    rng = np.random.RandomState(1)
    W = rng.randn(4, 2, 3, 3).astype(np.float32)
    b = rng.randn(4).astype(np.float32)
    np.savez(tmp_path / "w.npz", **{"conv/0": W, "conv/1": b})
    m = load_keras(str(p), str(tmp_path / "w.npz"))
    x = rng.randn(2, 2, 6, 6).astype(np.float32)
    ref = torch.nn.functional.max_pool2d(torch.nn.functional.conv2d(torch.from_numpy(x), torch.from_numpy(W),
                                                                    torch.from_numpy(b)), 2).reshape(2, -1)
    torch.testing.assert_close(m.forward(torch.from_numpy(x)), ref, rtol=1e-4, atol=1e-5)


def test_functional_model_with_merge():
    cfg = {"class_name": "Model", "config": {
        "name": "fm",
        "layers": [
            {"class_name": "InputLayer", "name": "in", "config": {"name": "in", "batch_input_shape": [None, 4]},
             "inbound_nodes": []},
            {"class_name": "Dense", "name": "a", "config": {"name": "a", "output_dim": 3, "activation": "linear"},
             "inbound_nodes": [[["in", 0, 0]]]},
            {"class_name": "Dense", "name": "b", "config": {"name": "b", "output_dim": 3, "activation": "tanh"},
             "inbound_nodes": [[["in", 0, 0]]]},
            {"class_name": "Merge", "name": "m", "config": {"name": "m", "mode": "sum"},
             "inbound_nodes": [[["a", 0, 0], ["b", 0, 0]]]},
        ],
        "input_layers": [["in", 0, 0]], "output_layers": [["m", 0, 0]]}}
    m = DefinitionLoader.from_json_str(json.dumps(cfg))
    rng = np.random.RandomState(2)
    Wa, ba, Wb, bb = (rng.randn(4, 3).astype(np.float32), rng.randn(3).astype(np.float32),
                      rng.randn(4, 3).astype(np.float32), rng.randn(3).astype(np.float32))
    WeightLoader.load_weights(m, {"a": [Wa, ba], "b": [Wb, bb]})
    x = rng.randn(2, 4).astype(np.float32)
    ref = x @ Wa + ba + np.tanh(x @ Wb + bb)
    np.testing.assert_allclose(m.forward(torch.from_numpy(x)).numpy(), ref, rtol=1e-5, atol=1e-5)


def test_lstm_weight_conversion():
    cfg = {"class_name": "Sequential", "config": [
        {"class_name": "LSTM", "config": {"name": "lstm", "output_dim": 4, "activation": "tanh",
                                          "inner_activation": "sigmoid", "return_sequences": False,
                                          "batch_input_shape": [None, 3, 2]}}]}
    m = DefinitionLoader.from_json_str(json.dumps(cfg))
    rng = np.random.RandomState(3)
    H, D = 4, 2
    ws = []
    for _ in range(4):  # gates i, c, f, o: W, U, b
        ws += [rng.randn(D, H).astype(np.float32) * 0.5, rng.randn(H, H).astype(np.float32) * 0.5,
               rng.randn(H).astype(np.float32) * 0.1]
    WeightLoader.load_weights(m, {"lstm": ws})
    x = rng.randn(2, 3, D).astype(np.float32)
    sig = lambda v: 1 / (1 + np.exp(-v))  # noqa: E731
    h = np.zeros((2, H), np.float32)
    c = np.zeros((2, H), np.float32)
    Wi, Ui, bi, Wc, Uc, bc, Wf, Uf, bf, Wo, Uo, bo = ws
    for t in range(3):
        xt = x[:, t]
        i = sig(xt @ Wi + h @ Ui + bi)
        f = sig(xt @ Wf + h @ Uf + bf)
        g = np.tanh(xt @ Wc + h @ Uc + bc)
        o = sig(xt @ Wo + h @ Uo + bo)
        c = f * c + i * g
        h = o * np.tanh(c)
    np.testing.assert_allclose(m.forward(torch.from_numpy(x)).numpy(), h, rtol=1e-4, atol=1e-5)
