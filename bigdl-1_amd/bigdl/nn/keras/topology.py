"""Keras-1.2.2-style API (``DL/nn/keras/Topology.scala:55-262``, ``pyspark/bigdl/nn/keras/topology.py``).

``KerasLayer`` wraps one ``bigdl.nn`` module (its "labor") that is created once the input shape
is known, so every layer does shape inference (batch dimension excluded from all shapes).
``Sequential`` builds layers as they are added; ``Model(input, output)`` is the functional graph
form built from ``Input(shape=...)`` nodes.  ``compile`` / ``fit`` / ``evaluate`` / ``predict``
drive the same Optimizer / Evaluator / Predictor as the Torch-style API.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from ..abstractnn import AbstractModule, to_torch
from ..containers import Sequential as _NNSequential
from ..graph import Graph, ModuleNode, _InputLayer

Shape = Tuple[int, ...]


def _as_shape(s) -> Optional[Shape]:
    if s is None:
        return None
    if isinstance(s, int):
        return (s,)
    return tuple(int(v) if v is not None else -1 for v in s)


class KerasLayer(AbstractModule):
    """Base: subclasses implement ``build_labor(input_shape)`` (returns the inner nn module) and
    ``compute_output_shape(input_shape)``.  Shapes exclude the batch dimension; multi-input layers
    receive a list of shapes."""

    SCALA_PACKAGE = "com.intel.analytics.bigdl.nn.keras"

    def __init__(self, input_shape=None, name=None):
        super().__init__()
        self.input_shape = _as_shape(input_shape) if not (isinstance(input_shape, list) and input_shape and
                                                           isinstance(input_shape[0], (list, tuple))) else \
            [_as_shape(s) for s in input_shape]
        self.labor: Optional[AbstractModule] = None
        self.output_shape = None
        if name:
            self.set_name(name)

    # --- shape inference -------------------------------------------------------------------------
    def build_labor(self, input_shape) -> AbstractModule:  # pragma: no cover - abstract
        raise NotImplementedError

    def compute_output_shape(self, input_shape):
        return input_shape

    def build(self, input_shape):
        if self.labor is not None:
            return self.output_shape
        self.input_shape = input_shape
        self.labor = self.build_labor(input_shape)
        self.output_shape = self.compute_output_shape(input_shape)
        return self.output_shape

    def get_input_shape(self):
        return self.input_shape

    def get_output_shape(self):
        return self.output_shape

    # --- module protocol: delegate to the labor --------------------------------------------------
    def _need(self):
        if self.labor is None:
            if self.input_shape is None:
                raise ValueError(f"{type(self).__name__}: input shape unknown; pass input_shape=")
            self.build(self.input_shape)
        return self.labor

    def updateOutput(self, input):
        return self._need().forward(input)

    def updateGradInput(self, input, gradOutput):
        return self._need().updateGradInput(input, gradOutput)

    def accGradParameters(self, input, gradOutput):
        self._need().accGradParameters(input, gradOutput)

    def backward(self, input, gradOutput):
        self.gradInput = self._need().backward(input, gradOutput)
        for h in self._grad_ready_hooks:
            h(self)
        return self.gradInput

    def children(self):
        return [self.labor] if self.labor is not None else []

    def parameters(self):
        return self.labor.parameters() if self.labor is not None else None

    def _param_entries(self):
        return self.labor._param_entries() if self.labor is not None else []

    def _set_arena_recursive(self, arena):
        self._arena = arena
        if self.labor is not None:
            self.labor._set_arena_recursive(arena)

    def getExtraParameter(self):
        return self.labor.getExtraParameter() if self.labor is not None else None

    def __call__(self, *nodes):
        """Functional API: build from the input node shapes, return the output node."""
        shapes = [getattr(n, "_keras_shape", None) for n in nodes]
        shp = shapes[0] if len(shapes) == 1 else shapes
        if self.labor is None:
            if any(s is None for s in (shapes if len(shapes) > 1 else [shp])):
                raise ValueError("Keras functional API needs nodes created from Input(shape=...)")
            self.build(shp)
        node = ModuleNode.create(self, list(nodes))
        node._keras_shape = self.output_shape
        return node

    def __repr__(self):
        return f"{type(self).__name__}[{self.get_name()}]"


class InputLayer(KerasLayer):
    """``InputLayer(input_shape)`` — identity carrying a shape (first layer of a Sequential)."""

    def __init__(self, input_shape=None, name=None):
        super().__init__(input_shape, name)

    def build_labor(self, input_shape):
        from ..layers.shape import Identity
        return Identity()


def Input(shape=None, name=None):
    """Functional-API input node with a known shape (``Input(shape=(3, 32, 32))``)."""
    m = _InputLayer()
    if name:
        m.set_name(name)
    node = ModuleNode(m)
    node._keras_shape = _as_shape(shape)
    return node


# ------------------------------------------------------------------------------------------------ models
_OPTIMS = {
    "sgd": lambda: __import__("bigdl.optim", fromlist=["SGD"]).SGD(learningrate=0.01),
    "adagrad": lambda: __import__("bigdl.optim", fromlist=["Adagrad"]).Adagrad(learningrate=0.01),
    "adam": lambda: __import__("bigdl.optim", fromlist=["Adam"]).Adam(),
    "rmsprop": lambda: __import__("bigdl.optim", fromlist=["RMSprop"]).RMSprop(learningrate=0.001, decayrate=0.9),
    "adadelta": lambda: __import__("bigdl.optim", fromlist=["Adadelta"]).Adadelta(decayrate=0.95, epsilon=1e-8),
    "adamax": lambda: __import__("bigdl.optim", fromlist=["Adamax"]).Adamax(epsilon=1e-8),
}


def _criterion(name: str):
    from .. import criterion as C
    n = name.lower()
    table = {
        "categorical_crossentropy": lambda: C.CategoricalCrossEntropy(),
        "mse": lambda: C.MSECriterion(), "mean_squared_error": lambda: C.MSECriterion(),
        "binary_crossentropy": lambda: C.BCECriterion(),
        "mae": lambda: C.AbsCriterion(), "mean_absolute_error": lambda: C.AbsCriterion(),
        "hinge": lambda: C.MarginCriterion(),
        "squared_hinge": lambda: C.MarginCriterion(squared=True),
        "mape": lambda: C.MeanAbsolutePercentageCriterion(),
        "mean_absolute_percentage_error": lambda: C.MeanAbsolutePercentageCriterion(),
        "msle": lambda: C.MeanSquaredLogarithmicCriterion(),
        "mean_squared_logarithmic_error": lambda: C.MeanSquaredLogarithmicCriterion(),
        "sparse_categorical_crossentropy": lambda: C.ClassNLLCriterion(logProbAsInput=False),
        "kld": lambda: C.KullbackLeiblerDivergenceCriterion(),
        "kullback_leibler_divergence": lambda: C.KullbackLeiblerDivergenceCriterion(),
        "poisson": lambda: C.PoissonCriterion(),
        "cosine_proximity": lambda: C.CosineProximityCriterion(), "cosine": lambda: C.CosineProximityCriterion(),
    }
    if n not in table:
        raise TypeError(f"Unsupported loss: {name}")
    return table[n]()


class KerasModel(KerasLayer):
    def __init__(self, name=None):
        super().__init__(None, name)
        self.optim_method = None
        self.criterion = None
        self.metrics = None

    def compile(self, optimizer, loss, metrics=None):
        if isinstance(optimizer, str):
            if optimizer.lower() not in _OPTIMS:
                raise TypeError(f"Unsupported optimizer: {optimizer}")
            optimizer = _OPTIMS[optimizer.lower()]()
        if isinstance(loss, str):
            loss = _criterion(loss)
        ms = []
        for m in (metrics or []):
            if isinstance(m, str):
                if m.lower() != "accuracy":
                    raise TypeError(f"Unsupported metrics: {m}")
                from ...optim.validation import Top1Accuracy
                ms.append(Top1Accuracy())
            else:
                ms.append(m)
        self.optim_method, self.criterion, self.metrics = optimizer, loss, ms
        return self

    @staticmethod
    def _samples(x, y):
        from ...dataset import Sample
        if y is None:
            return list(x)
        xs = x if isinstance(x, (list, tuple)) else [x]
        n = len(xs[0])
        out = []
        for i in range(n):
            feats = [np.asarray(v[i], dtype=np.float32) for v in xs]
            lab = np.asarray(y[i], dtype=np.float32).reshape(-1)
            out.append(Sample(feats if len(feats) > 1 else feats[0], lab))
        return out

    def fit(self, x, y=None, batch_size=32, nb_epoch=10, validation_data=None, distributed=False):
        if self.criterion is None:
            raise ValueError("compile() must be called before fit()")
        from ...optim.optimizer import Optimizer
        from ...optim.trigger import MaxEpoch, EveryEpoch
        train = self._samples(x, y)
        opt = Optimizer.create(self, train, self.criterion, MaxEpoch(nb_epoch), batch_size, self.optim_method,
                               distributed=distributed)
        if validation_data is not None and self.metrics:
            vx, vy = validation_data if isinstance(validation_data, tuple) else (validation_data, None)
            opt.setValidation(EveryEpoch(), self._samples(vx, vy), self.metrics, batch_size)
        opt.optimize()
        return self

    def evaluate(self, x=None, y=None, batch_size=32):
        if x is None:
            return self.training(False)
        from ...optim.evaluator import Evaluator
        return Evaluator(self).test(self._samples(x, y), self.metrics or [], batch_size)

    def predict(self, x, distributed=False, batch_size=32):
        from ...optim.predictor import LocalPredictor
        out = LocalPredictor(self, batch_size=batch_size).predict(
            self._samples(x if not isinstance(x, np.ndarray) else list(x), None) if not isinstance(x, np.ndarray)
            else x)
        return np.stack([o.numpy() for o in out]) if out and isinstance(out[0], torch.Tensor) else out

    def get_weights(self):
        return super().get_weights()


class Sequential(KerasModel):
    """``Sequential()`` whose layers are built as they are added (first needs ``input_shape``)."""

    def __init__(self, name=None):
        super().__init__(name)
        self.labor = _NNSequential()
        self.layers: List[KerasLayer] = []

    def add(self, layer: KerasLayer):
        if not self.layers:
            shp = layer.input_shape
            if shp is None:
                raise ValueError("The first layer of a Sequential needs input_shape")
            self.input_shape = shp
        else:
            shp = self.layers[-1].output_shape
        layer.build(shp) if isinstance(layer, KerasLayer) else None
        self.layers.append(layer)
        self.labor.add(layer)
        self.output_shape = layer.output_shape if isinstance(layer, KerasLayer) else shp
        return self

    def build_labor(self, input_shape):
        return self.labor

    def compute_output_shape(self, input_shape):
        return self.output_shape


class Model(KerasModel):
    """Functional model ``Model(input, output)`` over nodes from ``Input`` and layer calls."""

    def __init__(self, input, output, name=None):
        super().__init__(name)
        ins = input if isinstance(input, (list, tuple)) else [input]
        outs = output if isinstance(output, (list, tuple)) else [output]
        self.labor = Graph(list(ins), list(outs))
        shapes_in = [getattr(n, "_keras_shape", None) for n in ins]
        shapes_out = [getattr(n, "_keras_shape", None) for n in outs]
        self.input_shape = shapes_in[0] if len(shapes_in) == 1 else shapes_in
        self.output_shape = shapes_out[0] if len(shapes_out) == 1 else shapes_out

    def build_labor(self, input_shape):
        return self.labor

    def compute_output_shape(self, input_shape):
        return self.output_shape
