"""Run a compiled Keras model on the BigDL engine (``pyspark/bigdl/keras/backend.py``):
``with_bigdl_backend(kmodel)`` converts the model definition (``kmodel.to_json()``,
:class:`bigdl.keras.converter.DefinitionLoader`), copies its weights layer by layer
(``layer.get_weights()``), maps the compile settings (:class:`OptimConverter`), and returns a
wrapper whose ``fit`` / ``evaluate`` / ``predict`` train and infer with BigDL's optimizers — the
LocalOptimizer in one process, the RCCL DistriOptimizer (``is_distributed=True`` under
``python -m bigdl.launch``).  Unlike the reference, local ``evaluate`` and local validation data
are supported.  Keras itself is not installed here; any object with the Keras model protocol
(``to_json``, ``layers[i].name / get_weights``, ``loss``, ``optimizer``, ``metrics``) works."""
from __future__ import annotations

import numpy as np
import torch

from .converter import DefinitionLoader, WeightLoader
from .optimization import OptimConverter


def _unsupported(what):
    raise NotImplementedError(f"{what} is not supported by the BigDL Keras backend")


def _samples(x, y):
    from ..dataset import Sample
    xs = x if isinstance(x, (list, tuple)) else [x]
    n = len(xs[0])
    out = []
    for i in range(n):
        f = [np.asarray(v[i], dtype=np.float32) for v in xs]
        lab = None if y is None else np.asarray(y[i], dtype=np.float32).reshape(-1)
        out.append(Sample(f if len(f) > 1 else f[0], lab))
    return out


class KerasModelWrapper:
    def __init__(self, kmodel):
        self.bmodel = DefinitionLoader.from_json_str(kmodel.to_json())
        weights = {l.name: l.get_weights() for l in getattr(kmodel, "layers", []) if l.get_weights()}
        if weights:
            WeightLoader.load_weights(self.bmodel, weights, by_name=True)
        loss = getattr(kmodel, "loss", None)
        opt = getattr(kmodel, "optimizer", None)
        metrics = getattr(kmodel, "metrics", None)
        self.criterion = OptimConverter.to_bigdl_criterion(loss) if loss else None
        self.optim_method = OptimConverter.to_bigdl_optim_method(opt) if opt else None
        self.metrics = OptimConverter.to_bigdl_metrics(metrics) if metrics else None

    def fit(self, x, y=None, batch_size=32, nb_epoch=10, verbose=1, callbacks=None, validation_split=0.,
            validation_data=None, shuffle=True, class_weight=None, sample_weight=None, initial_epoch=0,
            is_distributed=False):
        for flag, name in ((callbacks, "callbacks"), (class_weight, "class_weight"), (sample_weight, "sample_weight"),
                           (initial_epoch != 0, "initial_epoch"), (shuffle is not True, "shuffle=False"),
                           (validation_split != 0., "validation_split")):
            if flag:
                _unsupported(name)
        if self.criterion is None:
            raise ValueError("the Keras model must be compiled (loss) before fit")
        from ..optim.optimizer import Optimizer
        from ..optim.trigger import MaxEpoch, EveryEpoch
        data = _samples(x, y) if isinstance(x, (np.ndarray, list, tuple)) else x
        opt = Optimizer.create(self.bmodel, data, self.criterion, MaxEpoch(nb_epoch), batch_size,
                               self.optim_method, distributed=bool(is_distributed))
        if validation_data is not None and self.metrics:
            vx, vy = validation_data
            opt.setValidation(EveryEpoch(), _samples(vx, vy), self.metrics, batch_size)
        opt.optimize()
        return self

    def evaluate(self, x, y, batch_size=32, sample_weight=None, is_distributed=False):
        if sample_weight:
            _unsupported("sample_weight")
        if not self.metrics:
            raise ValueError("no metrics: compile the Keras model with metrics=['accuracy']")
        from ..optim.evaluator import Evaluator
        res = Evaluator(self.bmodel).test(_samples(x, y), self.metrics, batch_size)
        return [r.result()[0] for r, _ in res]

    def predict(self, x, batch_size=None, verbose=None, is_distributed=False):
        self.bmodel.evaluate()
        bs = batch_size or 32
        xt = torch.as_tensor(np.asarray(x, dtype=np.float32))
        outs = []
        with torch.no_grad():
            for i in range(0, xt.shape[0], bs):
                outs.append(self.bmodel.forward(xt[i:i + bs]).float().cpu())
        return torch.cat(outs).numpy()


def with_bigdl_backend(kmodel):
    from ..utils.engine import Engine
    if not Engine.is_inited():
        Engine.init()
    return KerasModelWrapper(kmodel)


__all__ = ["KerasModelWrapper", "with_bigdl_backend"]
