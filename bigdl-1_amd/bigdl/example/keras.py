"""LeNet through the Keras-style API (``DL/example/keras/Train.scala`` / ``keras/LeNet.scala``):
Reshape → Convolution2D(32, 3, 3, relu) → Convolution2D(32, 3, 3, relu) → MaxPooling2D →
Dropout → Flatten → Dense(128, relu) → Dropout → Dense(10, softmax), compiled with
``adadelta`` / ``sparse_categorical_crossentropy`` (1-based class labels) / ``accuracy`` and
trained with ``fit``."""
from __future__ import annotations

import argparse
import sys

import numpy as np


def lenet_keras(input_shape=(28, 28, 1), classes=10):
    from ..nn.keras import Sequential, Reshape, Convolution2D, MaxPooling2D, Dropout, Flatten, Dense
    m = Sequential()
    m.add(Reshape((1, 28, 28), input_shape=input_shape))
    m.add(Convolution2D(32, 3, 3, activation="relu"))
    m.add(Convolution2D(32, 3, 3, activation="relu"))
    m.add(MaxPooling2D(pool_size=(2, 2)))
    m.add(Dropout(0.25))
    m.add(Flatten())
    m.add(Dense(128, activation="relu"))
    m.add(Dropout(0.5))
    m.add(Dense(classes, activation="softmax"))
    return m


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--synthetic", type=int, default=256)
    ap.add_argument("-b", "--batchSize", type=int, default=32)
    ap.add_argument("-e", "--maxEpoch", type=int, default=2)
    a = ap.parse_args(argv)
    from ..utils.engine import Engine
    from ..models.train.common import synthetic_images
    Engine.init()
    x, y = synthetic_images(a.synthetic, 28, 28, 1, 10, 0)
    x = (x.astype(np.float32) - 33.3) / 78.6
    m = lenet_keras()
    m.compile(optimizer="adadelta", loss="sparse_categorical_crossentropy", metrics=["accuracy"])
    m.fit(x, y, batch_size=a.batchSize, nb_epoch=a.maxEpoch, validation_data=(x[:64], y[:64]))
    res = m.evaluate(x[:128], y[:128], batch_size=a.batchSize)
    print(res)
    return res


if __name__ == "__main__":
    main(sys.argv[1:])
