"""Load a TensorFlow GraphDef as a BigDL model, and save a BigDL model as a GraphDef
(``DL/example/tensorflow/loadandsave/{Load,Save}.scala``).

    python -m bigdl.example.tensorflow.loadandsave load model.pb [--inputs Placeholder]
                                                                 [--outputs LeNet/fc4/BiasAdd]
    python -m bigdl.example.tensorflow.loadandsave save [./bigdl.pb]

``load`` runs the imported model on one random 1×1×28×28 input (the reference's ``model.pb`` is
the LeNet of its ``model.py``); ``save`` writes the reference's LeNet ``Graph`` (conv1_5x5 → tanh
→ pool → tanh → conv2_5x5 → pool → reshape → fc1 → tanh → fc2 → LogSoftMax) with an ``input``
placeholder of shape (1, 1, 28, 28).
"""
from __future__ import annotations

import argparse
import sys

import torch


def lenet():
    """The LeNet graph of Save.scala, with its layer names."""
    from ...nn import (Graph, Linear, LogSoftMax, Reshape, SpatialConvolution, SpatialMaxPooling, Tanh)
    conv1 = SpatialConvolution(1, 6, 5, 5).set_name("conv1_5x5").inputs()
    tanh1 = Tanh().set_name("tanh1").inputs(conv1)
    pool1 = SpatialMaxPooling(2, 2, 2, 2).set_name("pool1").inputs(tanh1)
    tanh2 = Tanh().set_name("tanh2").inputs(pool1)
    conv2 = SpatialConvolution(6, 12, 5, 5).set_name("conv2_5x5").inputs(tanh2)
    pool2 = SpatialMaxPooling(2, 2, 2, 2).set_name("pool2").inputs(conv2)
    reshape2 = Reshape([1, 12 * 4 * 4]).set_name("reshape2").inputs(pool2)
    fc1 = Linear(12 * 4 * 4, 100).set_name("fc1").inputs(reshape2)
    tanh3 = Tanh().set_name("tanh3").inputs(fc1)
    fc2 = Linear(100, 10).set_name("fc2").inputs(tanh3)
    output = LogSoftMax().set_name("output").inputs(fc2)
    return Graph(conv1, output)


def save(path: str = "./bigdl.pb", model=None):
    from ...utils.tf.saver import TensorflowSaver
    model = model if model is not None else lenet()
    TensorflowSaver.saveGraph(model, [("input", [1, 1, 28, 28])], path)
    return model


def load(path: str, inputs=("Placeholder",), outputs=("LeNet/fc4/BiasAdd",), x=None):
    from ...nn.module import Module
    model = Module.loadTF(path, list(inputs), list(outputs))
    x = torch.rand(1, 1, 28, 28) if x is None else x
    result = model.forward(x)
    print(result)
    return model, result


def main(argv=None):
    ap = argparse.ArgumentParser(description="BigDL TensorFlow load / save example")
    sub = ap.add_subparsers(dest="cmd", required=True)
    lp = sub.add_parser("load")
    lp.add_argument("path")
    lp.add_argument("--inputs", nargs="+", default=["Placeholder"])
    lp.add_argument("--outputs", nargs="+", default=["LeNet/fc4/BiasAdd"])
    sp = sub.add_parser("save")
    sp.add_argument("path", nargs="?", default="./bigdl.pb")
    a = ap.parse_args(argv)
    if a.cmd == "load":
        return load(a.path, a.inputs, a.outputs)
    return save(a.path)


if __name__ == "__main__":
    main(sys.argv[1:])
