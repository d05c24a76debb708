"""Keras compile settings → BigDL (``pyspark/bigdl/keras/optimization.py`` OptimConverter).

Keras is not installed here, so optimizers are recognised by class name and read through their
attributes (Keras 1.x ``lr``/``decay`` variables, or Keras 2 ``learning_rate`` / ``get_config()``);
any object with those attributes converts.  Losses map as the reference's table; ``"accuracy"``
is the only metric the reference converts."""
from __future__ import annotations

import warnings

from ..nn import criterion as C
from ..optim import optim_method as O
from ..optim.validation import Top1Accuracy


def _val(x, default=0.0):
    if x is None:
        return default
    if hasattr(x, "numpy"):
        x = x.numpy()
    try:
        return float(x)
    except TypeError:
        import numpy as np
        return float(np.asarray(x))


def _attr(o, *names, default=None):
    cfg = o.get_config() if hasattr(o, "get_config") else {}
    for n in names:
        if hasattr(o, n):
            return getattr(o, n)
        if n in cfg:
            return cfg[n]
    return default


class OptimConverter:
    @staticmethod
    def to_bigdl_metrics(metrics):
        out = []
        for m in (metrics if isinstance(metrics, (list, tuple)) else [metrics]):
            if m == "accuracy" or m == "acc":
                out.append(Top1Accuracy())
            else:
                raise ValueError(f"unsupported Keras metric {m!r}")
        return out

    _LOSSES = {
        "categorical_crossentropy": lambda: C.CategoricalCrossEntropy(),
        "mse": lambda: C.MSECriterion(), "mean_squared_error": lambda: C.MSECriterion(),
        "binary_crossentropy": lambda: C.BCECriterion(),
        "mae": lambda: C.AbsCriterion(), "mean_absolute_error": lambda: C.AbsCriterion(),
        "hinge": lambda: C.MarginCriterion(),
        "mean_absolute_percentage_error": lambda: C.MeanAbsolutePercentageCriterion(),
        "mape": lambda: C.MeanAbsolutePercentageCriterion(),
        "mean_squared_logarithmic_error": lambda: C.MeanSquaredLogarithmicCriterion(),
        "msle": lambda: C.MeanSquaredLogarithmicCriterion(),
        "squared_hinge": lambda: C.MarginCriterion(squared=True),
        "sparse_categorical_crossentropy": lambda: C.ClassNLLCriterion(logProbAsInput=False),
        "kullback_leibler_divergence": lambda: C.KullbackLeiblerDivergenceCriterion(),
        "kld": lambda: C.KullbackLeiblerDivergenceCriterion(),
        "poisson": lambda: C.PoissonCriterion(),
        "cosine_proximity": lambda: C.CosineProximityCriterion(), "cosine": lambda: C.CosineProximityCriterion(),
    }

    @staticmethod
    def to_bigdl_criterion(kloss):
        name = kloss if isinstance(kloss, str) else getattr(kloss, "__name__", str(kloss))
        f = OptimConverter._LOSSES.get(name.lower())
        if f is None:
            raise ValueError(f"unsupported Keras loss {kloss!r}")
        return f()

    @staticmethod
    def to_bigdl_optim_method(kopt):
        if isinstance(kopt, str):
            return {"sgd": O.SGD, "adagrad": O.Adagrad, "adam": O.Adam, "rmsprop": O.RMSprop,
                    "adadelta": O.Adadelta, "adamax": O.Adamax}[kopt.lower()]()
        kind = type(kopt).__name__
        lr = _val(_attr(kopt, "lr", "learning_rate"), 0.01)
        decay = _val(_attr(kopt, "decay"), 0.0)
        eps = _val(_attr(kopt, "epsilon"), 1e-8)
        if kind == "Adagrad":
            warnings.warn("For Adagrad, we don't support epsilon for now")
            return O.Adagrad(learningrate=lr, learningrate_decay=decay)
        if kind == "SGD":
            return O.SGD(learningrate=lr, learningrate_decay=decay, momentum=_val(_attr(kopt, "momentum")),
                         nesterov=bool(_attr(kopt, "nesterov", default=False)))
        if kind == "Adam":
            return O.Adam(learningrate=lr, learningrate_decay=decay, beta1=_val(_attr(kopt, "beta_1"), 0.9),
                          beta2=_val(_attr(kopt, "beta_2"), 0.999), epsilon=eps)
        if kind == "RMSprop":
            return O.RMSprop(learningrate=lr, learningrate_decay=decay, decayrate=_val(_attr(kopt, "rho"), 0.9),
                             epsilon=eps)
        if kind == "Adadelta":
            warnings.warn("For Adadelta, we don't support learning rate and learning rate decay for now")
            return O.Adadelta(decayrate=_val(_attr(kopt, "rho"), 0.95), epsilon=eps)
        if kind == "Adamax":
            warnings.warn("For Adamax, we don't support learning rate decay for now")
            return O.Adamax(learningrate=lr, beta1=_val(_attr(kopt, "beta_1"), 0.9),
                            beta2=_val(_attr(kopt, "beta_2"), 0.999), epsilon=eps)
        raise ValueError(f"unsupported Keras optimizer {kind}")


__all__ = ["OptimConverter"]
