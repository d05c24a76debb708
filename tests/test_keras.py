"""Keras-style API (DL/nn/keras, pyspark/bigdl/nn/keras): every layer's inferred output shape must
equal the shape its forward actually produces; compile/fit/evaluate/predict; functional Model."""
import numpy as np
import pytest
import torch

from bigdl.nn import keras as K

CASES = [
    (lambda: K.Dense(7, activation="relu", input_shape=(5,)), (5,)),
    (lambda: K.Dense(7, input_shape=(3, 5)), (3, 5)),
    (lambda: K.MaxoutDense(4, 3, input_shape=(6,)), (6,)),
    (lambda: K.Activation("tanh", input_shape=(4, 3)), (4, 3)),
    (lambda: K.Dropout(0.3, input_shape=(4,)), (4,)),
    (lambda: K.Flatten(input_shape=(2, 3, 4)), (2, 3, 4)),
    (lambda: K.Reshape((6, -1), input_shape=(2, 3, 4)), (2, 3, 4)),
    (lambda: K.Permute((3, 1, 2), input_shape=(2, 3, 4)), (2, 3, 4)),
    (lambda: K.RepeatVector(3, input_shape=(5,)), (5,)),
    (lambda: K.Highway(activation="relu", input_shape=(6,)), (6,)),
    (lambda: K.Masking(0.0, input_shape=(3, 4)), (3, 4)),
    (lambda: K.BatchNormalization(input_shape=(3, 8, 8)), (3, 8, 8)),
    (lambda: K.BatchNormalization(input_shape=(6,)), (6,)),
    (lambda: K.Convolution1D(5, 3, input_shape=(10, 4)), (10, 4)),
    (lambda: K.Convolution2D(6, 3, 3, border_mode="same", subsample=(2, 2), input_shape=(3, 9, 9)), (3, 9, 9)),
    (lambda: K.Convolution2D(6, 3, 3, dim_ordering="tf", input_shape=(9, 9, 3)), (9, 9, 3)),
    (lambda: K.AtrousConvolution2D(4, 3, 3, atrous_rate=(2, 2), input_shape=(2, 11, 11)), (2, 11, 11)),
    (lambda: K.AtrousConvolution1D(4, 3, atrous_rate=2, input_shape=(12, 3)), (12, 3)),
    (lambda: K.Deconvolution2D(4, 3, 3, subsample=(2, 2), input_shape=(2, 5, 5)), (2, 5, 5)),
    (lambda: K.SeparableConvolution2D(6, 3, 3, depth_multiplier=2, input_shape=(3, 8, 8)), (3, 8, 8)),
    (lambda: K.Convolution3D(4, 2, 2, 2, input_shape=(2, 5, 5, 5)), (2, 5, 5, 5)),
    (lambda: K.LocallyConnected1D(4, 3, input_shape=(8, 3)), (8, 3)),
    (lambda: K.LocallyConnected2D(4, 3, 3, input_shape=(2, 6, 6)), (2, 6, 6)),
    (lambda: K.MaxPooling2D(input_shape=(3, 8, 8)), (3, 8, 8)),
    (lambda: K.AveragePooling2D((3, 3), (2, 2), input_shape=(3, 9, 9)), (3, 9, 9)),
    (lambda: K.MaxPooling1D(2, input_shape=(8, 3)), (8, 3)),
    (lambda: K.AveragePooling1D(2, input_shape=(8, 3)), (8, 3)),
    (lambda: K.MaxPooling3D(input_shape=(2, 4, 4, 4)), (2, 4, 4, 4)),
    (lambda: K.AveragePooling3D(input_shape=(2, 4, 4, 4)), (2, 4, 4, 4)),
    (lambda: K.GlobalMaxPooling1D(input_shape=(5, 3)), (5, 3)),
    (lambda: K.GlobalAveragePooling1D(input_shape=(5, 3)), (5, 3)),
    (lambda: K.GlobalMaxPooling2D(input_shape=(3, 4, 4)), (3, 4, 4)),
    (lambda: K.GlobalAveragePooling2D(dim_ordering="tf", input_shape=(4, 4, 3)), (4, 4, 3)),
    (lambda: K.GlobalAveragePooling3D(input_shape=(2, 3, 3, 3)), (2, 3, 3, 3)),
    (lambda: K.ZeroPadding1D(2, input_shape=(5, 3)), (5, 3)),
    (lambda: K.ZeroPadding2D((1, 2), input_shape=(2, 4, 4)), (2, 4, 4)),
    (lambda: K.ZeroPadding3D((1, 1, 1), input_shape=(2, 3, 3, 3)), (2, 3, 3, 3)),
    (lambda: K.Cropping1D((1, 2), input_shape=(7, 3)), (7, 3)),
    (lambda: K.Cropping2D(((1, 1), (2, 0)), input_shape=(2, 6, 6)), (2, 6, 6)),
    (lambda: K.Cropping3D(((1, 1), (1, 0), (0, 1)), input_shape=(2, 4, 4, 4)), (2, 4, 4, 4)),
    (lambda: K.UpSampling1D(2, input_shape=(4, 3)), (4, 3)),
    (lambda: K.UpSampling2D((2, 3), input_shape=(2, 3, 3)), (2, 3, 3)),
    (lambda: K.UpSampling3D((2, 2, 2), input_shape=(1, 2, 2, 2)), (1, 2, 2, 2)),
    (lambda: K.SpatialDropout1D(0.2, input_shape=(4, 3)), (4, 3)),
    (lambda: K.SpatialDropout2D(0.2, input_shape=(2, 4, 4)), (2, 4, 4)),
    (lambda: K.SpatialDropout3D(0.2, input_shape=(2, 3, 3, 3)), (2, 3, 3, 3)),
    (lambda: K.GaussianDropout(0.2, input_shape=(5,)), (5,)),
    (lambda: K.GaussianNoise(0.1, input_shape=(5,)), (5,)),
    (lambda: K.ELU(input_shape=(5,)), (5,)),
    (lambda: K.LeakyReLU(0.2, input_shape=(5,)), (5,)),
    (lambda: K.ThresholdedReLU(0.5, input_shape=(5,)), (5,)),
    (lambda: K.SReLU(input_shape=(3, 4)), (3, 4)),
    (lambda: K.SimpleRNN(5, input_shape=(6, 3)), (6, 3)),
    (lambda: K.LSTM(5, return_sequences=True, input_shape=(6, 3)), (6, 3)),
    (lambda: K.GRU(5, go_backwards=True, input_shape=(6, 3)), (6, 3)),
    (lambda: K.ConvLSTM2D(3, 3, return_sequences=True, input_shape=(4, 2, 5, 5)), (4, 2, 5, 5)),
    (lambda: K.TimeDistributed(K.Dense(4), input_shape=(5, 3)), (5, 3)),
    (lambda: K.Bidirectional(K.LSTM(4, return_sequences=True), input_shape=(5, 3)), (5, 3)),
    (lambda: K.Bidirectional(K.GRU(4), merge_mode="sum", input_shape=(5, 3)), (5, 3)),
]


@pytest.mark.parametrize("i", range(len(CASES)))
def test_layer_shape_inference(i):
    make, shp = CASES[i]
    m = K.Sequential()
    m.add(make())
    m.evaluate()
    x = torch.randn((2,) + tuple(shp))
    y = m.forward(x)
    assert tuple(y.shape[1:]) == tuple(m.output_shape), (type(m.layers[0]).__name__, y.shape, m.output_shape)


def test_embedding_and_merge_functional():
    inp = K.Input(shape=(5,))
    a = K.Dense(4, activation="relu")(inp)
    b = K.Dense(3)(inp)
    c = K.Merge(mode="concat")(a, b)
    d = K.Dense(2)(c)
    model = K.Model(inp, d)
    assert model.output_shape == (2,)
    assert model.forward(torch.randn(3, 5)).shape == (3, 2)
    s = K.Sequential()
    s.add(K.Embedding(20, 6, input_length=4))
    s.add(K.Flatten())
    assert s.forward(torch.randint(0, 20, (2, 4)).float()).shape == (2, 24)


def test_compile_fit_evaluate_predict():
    rng = np.random.RandomState(0)
    x = rng.randn(200, 4).astype(np.float32)
    y = (x[:, 0] - x[:, 1] > 0).astype(np.float32)  # 0/1 labels for categorical via one-hot
    yy = np.stack([1 - y, y], 1)
    m = K.Sequential()
    m.add(K.Dense(16, activation="relu", input_shape=(4,)))
    m.add(K.Dense(2, activation="softmax"))
    m.compile(optimizer="adam", loss="categorical_crossentropy", metrics=["accuracy"])
    m.fit(x, yy, batch_size=20, nb_epoch=40, validation_data=(x, y + 1))
    res = m.evaluate(x, y + 1, batch_size=50)
    assert res[0][0].result()[0] > 0.9
    p = m.predict(x[:7])
    assert p.shape == (7, 2) and np.allclose(p.sum(1), 1, atol=1e-4)
