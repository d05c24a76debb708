"""pyspark-compatible ``bigdl.nn.layer`` (``pyspark/bigdl/nn/layer.py``): every layer class, plus
``Layer`` (= AbstractModule), ``Container``, ``Model`` (a Graph with the model loaders) and
``Node``."""
from __future__ import annotations

from . import *  # noqa: F401,F403
from .. import nn as _nn

_nn_all = [n for n in dir(_nn) if not n.startswith("_") and isinstance(getattr(_nn, n), type)]
from .abstractnn import AbstractModule as Layer, TensorModule  # noqa: F401
from .containers import Container  # noqa: F401
from .graph import Graph, ModuleNode as Node  # noqa: F401
from .module import Module


class Model(Graph):
    """``Model(inputs, outputs)`` graph container with the static loaders of pyspark ``Model``."""

    @staticmethod
    def loadModel(model_path, weight_path=None, bigdl_type="float"):
        return Module.loadModule(model_path, weight_path)

    load = loadModel

    @staticmethod
    def load_torch(path, bigdl_type="float"):
        return Module.loadTorch(path)

    @staticmethod
    def load_caffe(model, defPath, modelPath, match_all=True, bigdl_type="float"):
        return Module.loadCaffe(model, defPath, modelPath, match_all)

    @staticmethod
    def load_caffe_model(defPath, modelPath, bigdl_type="float"):
        return Module.loadCaffeModel(defPath, modelPath)

    @staticmethod
    def load_tensorflow(path, inputs, outputs, byte_order="little_endian", bin_file=None, bigdl_type="float"):
        return Module.loadTF(path, inputs, outputs, byte_order, bin_file)

    @staticmethod
    def load_keras(json_path=None, hdf5_path=None, by_name=False):
        from ..keras.converter import load_keras
        return load_keras(json_path, hdf5_path, by_name)

    @staticmethod
    def load_onnx(path):
        from ..contrib.onnx import load as _load
        return _load(path)


__all__ = list(_nn_all) + ["Layer", "Container", "Model", "Node", "TensorModule"]
