"""Finite-difference gradient checking (the reference's test oracle,
``spark/dl/src/test/scala/.../nn/GradientChecker.scala:33-256``).

The check is independent of autograd and of any reference implementation of the layer: the loss is
``L = ½ Σ output²`` (so ``∂L/∂output = output``), the analytic input gradient comes from the
layer's own ``updateGradInput`` and the analytic parameter gradient from ``accGradParameters``, and
both are compared elementwise with the central difference ``(L(x + h) − L(x − h)) / 2h``.  By
default everything runs in float64 on the host (``module.to(dtype=torch.float64)``), so the
comparison tolerances can be tight.

``checkLayer`` / ``checkWeight`` / ``checkCriterion`` keep the reference names; ``num`` samples that
many random coordinates (the reference's ``PartCheck``), ``num=None`` checks every coordinate
(``FullCheck``).  Each returns ``True`` on success; ``last_report`` holds the worst
(coordinate, numeric, analytic, error) for diagnostics.
"""
from __future__ import annotations

import random
from typing import Optional

import torch


def _out_tensor(o):
    if isinstance(o, torch.Tensor):
        return o
    # Table outputs: concatenate the flattened tensors
    from ..utils.table import Table
    if isinstance(o, Table):
        return torch.cat([_out_tensor(v).reshape(-1) for v in o.values()])
    if isinstance(o, (list, tuple)):
        return torch.cat([_out_tensor(v).reshape(-1) for v in o])
    raise TypeError(f"unsupported output {type(o)}")


def _loss_and_grad(out):
    if isinstance(out, torch.Tensor):
        o = out.detach()
        return 0.5 * float((o.double() * o.double()).sum()), o.clone()
    from ..utils.table import Table
    if isinstance(out, Table):
        t = Table()
        loss = 0.0
        for k, v in out.items():
            l, g = _loss_and_grad(v)
            loss += l
            t[k] = g
        return loss, t
    raise TypeError(f"unsupported output {type(out)}")


def _leaves(x):
    if isinstance(x, torch.Tensor):
        return [x]
    from ..utils.table import Table
    if isinstance(x, Table):
        return [t for v in x.values() for t in _leaves(v)]
    if isinstance(x, (list, tuple)):
        return [t for v in x for t in _leaves(v)]
    raise TypeError(f"unsupported input {type(x)}")


class _FlatView:
    """Index the concatenation of several tensors (a Table input) without copying."""

    def __init__(self, ts):
        self.ts = [t.view(-1) for t in ts]
        self.sizes = [t.numel() for t in self.ts]

    def numel(self):
        return sum(self.sizes)

    def _loc(self, i):
        t = 0
        while i >= self.sizes[t]:
            i -= self.sizes[t]
            t += 1
        return self.ts[t], i

    def __getitem__(self, i):
        t, k = self._loc(i)
        return t[k]

    def __setitem__(self, i, v):
        t, k = self._loc(i)
        t[k] = v


class GradientChecker:
    def __init__(self, stepSize: float = 1e-6, threshold: float = 1e-6, relative: bool = True):
        self.stepSize = float(stepSize)
        self.threshold = float(threshold)
        self.relative = relative
        self.last_report = None

    def _ok(self, numeric, analytic):
        err = abs(numeric - analytic)
        if self.relative:
            err = err / max(1.0, abs(numeric), abs(analytic))
        return err, err <= self.threshold

    def _coords(self, n, num):
        if num is None or num >= n:
            return list(range(n))
        return [random.randrange(n) for _ in range(num)]

    def _record(self, worst, cand):
        return cand if worst is None or cand[3] > worst[3] else worst

    def checkLayer(self, layer, input, epsilon: Optional[float] = None, num: Optional[int] = 50) -> bool:
        """∂L/∂input of ``layer.updateGradInput`` vs central differences (``input``: a floating
        tensor or a Table of them, perturbed in place and restored)."""
        if epsilon is not None:
            self.threshold = epsilon
        out = layer.forward(input)
        _, gout = _loss_and_grad(out)
        gi = _out_tensor(layer.updateGradInput(input, gout)).reshape(-1).double().clone()
        flat = _FlatView(_leaves(input))
        ok, worst, h = True, None, self.stepSize
        for i in self._coords(flat.numel(), num):
            v = float(flat[i])
            flat[i] = v + h
            lp, _ = _loss_and_grad(layer.forward(input))
            flat[i] = v - h
            lm, _ = _loss_and_grad(layer.forward(input))
            flat[i] = v
            numeric = (lp - lm) / (2 * h)
            err, good = self._ok(numeric, float(gi[i]))
            worst = self._record(worst, (i, numeric, float(gi[i]), err))
            ok &= good
        layer.forward(input)
        self.last_report = worst
        return ok

    def checkWeight(self, layer, input, epsilon: Optional[float] = None, num: Optional[int] = 50) -> bool:
        """∂L/∂w of ``accGradParameters`` (over every parameter tensor of ``layer``) vs central
        differences on the same parameters."""
        if epsilon is not None:
            self.threshold = epsilon
        params = layer.parameters()
        if not params or not params[0]:
            raise ValueError(f"{layer} has no parameters")
        ws, gs = params
        layer.zeroGradParameters()
        out = layer.forward(input)
        _, gout = _loss_and_grad(out)
        layer.backward(input, gout)
        analytic = torch.cat([g.detach().contiguous().reshape(-1).double() for g in gs]).clone()
        sizes = [w.numel() for w in ws]
        ok, worst, h = True, None, self.stepSize
        total = sum(sizes)
        for j in self._coords(total, num):
            t, k = 0, j
            while k >= sizes[t]:
                k -= sizes[t]
                t += 1
            w = ws[t]
            # logical (row-major) coordinate, written through the parameter itself so its version
            # counter moves and compute-dtype caches (AbstractModule.cw) see the change; works for
            # the device-layout (permuted) weights too
            idx = tuple(int(i) for i in torch.unravel_index(torch.tensor(k), tuple(w.shape)))
            v = float(w[idx])
            with torch.no_grad():
                w[idx] = v + h
            lp, _ = _loss_and_grad(layer.forward(input))
            with torch.no_grad():
                w[idx] = v - h
            lm, _ = _loss_and_grad(layer.forward(input))
            with torch.no_grad():
                w[idx] = v
            numeric = (lp - lm) / (2 * h)
            err, good = self._ok(numeric, float(analytic[j]))
            worst = self._record(worst, (j, numeric, float(analytic[j]), err))
            ok &= good
        self.last_report = worst
        return ok

    def checkCriterion(self, criterion, input, target, epsilon: Optional[float] = None,
                       num: Optional[int] = 50) -> bool:
        """∂loss/∂input of ``criterion.backward`` vs central differences of ``criterion.forward``."""
        if epsilon is not None:
            self.threshold = epsilon
        criterion.forward(input, target)
        gi = _out_tensor(criterion.backward(input, target)).reshape(-1).double().clone()
        flat = input.view(-1)
        ok, worst, h = True, None, self.stepSize
        for i in self._coords(flat.numel(), num):
            v = float(flat[i])
            flat[i] = v + h
            lp = float(criterion.forward(input, target))
            flat[i] = v - h
            lm = float(criterion.forward(input, target))
            flat[i] = v
            numeric = (lp - lm) / (2 * h)
            err, good = self._ok(numeric, float(gi[i]))
            worst = self._record(worst, (i, numeric, float(gi[i]), err))
            ok &= good
        self.last_report = worst
        return ok

    # pyspark-style aliases
    check_layer = checkLayer
    check_weight = checkWeight
    check_criterion = checkCriterion


__all__ = ["GradientChecker"]
