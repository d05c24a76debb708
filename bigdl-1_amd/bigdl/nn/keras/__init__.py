"""Keras-1.2.2-style API over bigdl.nn (``DL/nn/keras``, ``pyspark/bigdl/nn/keras``)."""
from .topology import KerasLayer, KerasModel, Sequential, Model, Input, InputLayer
from .layers import *  # noqa: F401,F403
from . import layers as _layers

__all__ = ["KerasLayer", "KerasModel", "Sequential", "Model", "Input", "InputLayer"] + \
    [n for n in dir(_layers) if not n.startswith("_") and isinstance(getattr(_layers, n), type)
     and issubclass(getattr(_layers, n), KerasLayer)]
