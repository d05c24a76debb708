"""Evaluation drivers.

* ``Evaluator(model).test(dataset, vmethods, batch_size)`` (``DL/optim/Evaluator.scala:30-111``):
  every rank evaluates its shard; the per-method results are merged with one all-reduce of the
  packed result vectors (collective X12) instead of a Spark ``reduce``.
* ``Validator(model, dataset)`` → ``LocalValidator`` / ``DistriValidator``
  (``DL/optim/{Validator,LocalValidator,DistriValidator}.scala``): ``test(vmethods)`` returns
  ``[(ValidationResult, ValidationMethod)]``.
* ``evaluate_model`` backs ``AbstractModule.evaluate(dataset, vmethods, batch_size)``.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch

from ..utils.engine import Engine
from .predictor import _batches, _model_device
from .validation import ValidationMethod, ValidationResult, allreduce_results


def _run(model, batches, vmethods: Sequence[ValidationMethod]):
    dev = _model_device(model)
    was_training = model.isTraining()
    model.evaluate()
    results = None
    try:
        with torch.no_grad():
            for b in batches:
                b = b.to(dev, dtype=Engine.compute_dtype() if dev.type == "cuda" else None)
                out = model.forward(b.getInput())
                rs = [vm(out, b.getTarget()) for vm in vmethods]
                results = rs if results is None else [a + r for a, r in zip(results, rs)]
    finally:
        if was_training:
            model.training()
    if results is None:
        return []
    results = allreduce_results(results)
    return list(zip(results, vmethods))


class Evaluator:
    def __init__(self, model):
        self.model = model

    @staticmethod
    def apply(model):
        return Evaluator(model)

    def test(self, dataset, vmethods: Sequence[ValidationMethod], batch_size: int = 32
             ) -> List[Tuple[ValidationResult, ValidationMethod]]:
        return _run(self.model, _batches(dataset, batch_size), vmethods)

    def test_mini_batch(self, dataset, vmethods):
        return _run(self.model, _batches(dataset, -1), vmethods)

    testMiniBatch = test_mini_batch


class Validator:
    """``Validator(model, dataset)`` factory → Local or Distri validator by dataset kind."""

    def __new__(cls, model, dataset):
        from ..dataset import DistributedDataSet
        if cls is Validator:
            if isinstance(dataset, DistributedDataSet) or Engine.is_distributed():
                return DistriValidator(model, dataset)
            return LocalValidator(model, dataset)
        return super().__new__(cls)

    def __init__(self, model, dataset):
        self.model = model
        self.dataset = dataset

    def test(self, vmethods):
        raise NotImplementedError


class LocalValidator(Validator):
    def test(self, vmethods):
        return _run(self.model, _batches(self.dataset, -1), vmethods)


class DistriValidator(Validator):
    def test(self, vmethods):
        return _run(self.model, _batches(self.dataset, -1), vmethods)


def evaluate_model(model, dataset, vmethods, batch_size: int = 32):
    return Evaluator(model).test(dataset, vmethods, batch_size)
