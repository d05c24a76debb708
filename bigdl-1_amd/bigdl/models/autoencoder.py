"""MNIST autoencoder (``DL/models/autoencoder/Autoencoder.scala``): Reshape(784) → Linear(784, n)
→ ReLU → Linear(n, 784) → Sigmoid."""
from __future__ import annotations

from ..nn import Graph, Linear, ReLU, Reshape, Sequential, Sigmoid

FEATURE_SIZE = 28 * 28


def Autoencoder(class_num=32):
    return Sequential(Reshape([FEATURE_SIZE]), Linear(FEATURE_SIZE, class_num), ReLU(), Linear(class_num, FEATURE_SIZE),
                      Sigmoid())


def _graph(class_num=32):
    inp = Reshape([FEATURE_SIZE])()
    out = Sigmoid()(Linear(class_num, FEATURE_SIZE)(ReLU()(Linear(FEATURE_SIZE, class_num)(inp))))
    return Graph(inp, out)


Autoencoder.graph = _graph
