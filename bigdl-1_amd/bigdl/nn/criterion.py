"""Criteria (the reference's 38, ``DL/nn/*Criterion.scala``; pyspark ``bigdl/nn/criterion.py``).

Hot: ``ClassNLLCriterion`` (1-based targets, ``paddingValue`` skip, class weights, sizeAverage;
``ClassNLLCriterion.scala:70-230``) and ``CrossEntropyCriterion`` (= LogSoftMax + ClassNLL,
``CrossEntropyCriterion.scala:35-36``) — on device one fused log-softmax+NLL kernel produces the
loss and the gradient in a single pass (K12+K13).  ``TimeDistributedCriterion`` drives PTB.
The rest derive their gradient from the loss by AD.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from .. import ops
from ..utils.table import Table
from .abstractnn import AbstractCriterion, AutogradCriterion
from ..utils import acc_float


def _targets_1b(target):
    return target.reshape(-1)


class ClassNLLCriterion(AbstractCriterion):
    def __init__(self, weights=None, size_average=True, logProbAsInput=True, padding_value=-1, bigdl_type="float"):
        super().__init__(size_average)
        self.weights = None if weights is None else torch.as_tensor(weights, dtype=torch.float32)
        self.logProbAsInput = logProbAsInput
        self.paddingValue = padding_value

    def _w(self, x):
        if self.weights is not None and self.weights.device != x.device:
            self.weights = self.weights.to(x.device)
        return self.weights

    def updateOutput(self, input, target):
        lp = input if self.logProbAsInput else torch.log(acc_float(input).clamp_min(1e-8))
        return ops.class_nll_forward(lp, target, self._w(input), self.sizeAverage, self.paddingValue)

    def updateGradInput(self, input, target):
        lp = input if self.logProbAsInput else torch.log(acc_float(input).clamp_min(1e-8))
        g = ops.class_nll_backward(lp, target, self._w(input), self.sizeAverage, self.paddingValue)
        if not self.logProbAsInput:
            g = g / acc_float(input).clamp_min(1e-8)
        return g


class CrossEntropyCriterion(AbstractCriterion):
    def __init__(self, weights=None, size_average=True, bigdl_type="float"):
        super().__init__(size_average)
        self.weights = None if weights is None else torch.as_tensor(weights, dtype=torch.float32)
        self._cache = None

    def _w(self, x):
        if self.weights is not None and self.weights.device != x.device:
            self.weights = self.weights.to(x.device)
        return self.weights

    def updateOutput(self, input, target):
        loss, grad = ops.cross_entropy_fused(input, target, self._w(input), self.sizeAverage)
        self._cache = (id(input), id(target), grad)
        return loss

    def updateGradInput(self, input, target):
        if self._cache is not None and self._cache[0] == id(input) and self._cache[1] == id(target):
            g = self._cache[2]
        else:
            _, g = ops.cross_entropy_fused(input, target, self._w(input), self.sizeAverage)
        self._cache = None
        return g


class MSECriterion(AbstractCriterion):
    def __init__(self, size_average=True, bigdl_type="float"):
        super().__init__(size_average)

    def updateOutput(self, input, target):
        d = acc_float(input) - acc_float(target).reshape(input.shape)
        s = (d * d).sum()
        return s / input.numel() if self.sizeAverage else s

    def updateGradInput(self, input, target):
        d = acc_float(input) - acc_float(target).reshape(input.shape)
        g = 2 * d / (input.numel() if self.sizeAverage else 1)
        return g.to(input.dtype)


class AbsCriterion(AbstractCriterion):
    def __init__(self, size_average=True, bigdl_type="float"):
        super().__init__(size_average)

    def updateOutput(self, input, target):
        s = (acc_float(input) - acc_float(target).reshape(input.shape)).abs().sum()
        return s / input.numel() if self.sizeAverage else s

    def updateGradInput(self, input, target):
        g = torch.sign(acc_float(input) - acc_float(target).reshape(input.shape))
        return (g / (input.numel() if self.sizeAverage else 1)).to(input.dtype)


class BCECriterion(AutogradCriterion):
    def __init__(self, weights=None, size_average=True, bigdl_type="float"):
        super().__init__(size_average)
        self.weights = None if weights is None else torch.as_tensor(weights, dtype=torch.float32)

    def _loss(self, x, t):
        w = None if self.weights is None else self.weights.to(x.device)
        eps = 1e-12
        t = acc_float(t).reshape(x.shape)
        l = -(t * torch.log(x + eps) + (1 - t) * torch.log(1 - x + eps))
        if w is not None:
            l = l * w
        return l.sum() / x.numel() if self.sizeAverage else l.sum()


class SmoothL1Criterion(AutogradCriterion):
    def __init__(self, size_average=True, bigdl_type="float"):
        super().__init__(size_average)

    def _loss(self, x, t):
        return F.smooth_l1_loss(acc_float(x), acc_float(t).reshape(x.shape), reduction="mean" if self.sizeAverage else "sum")


class SmoothL1CriterionWithWeights(AutogradCriterion):
    """Fast-RCNN box loss: Table(target, insideW, outsideW) (``SmoothL1CriterionWithWeights.scala``)."""

    def __init__(self, sigma, num=0, bigdl_type="float"):
        super().__init__(False)
        self.sigma, self.num = sigma, num

    def _loss(self, x, target):
        t, inw, outw = (target[1], target[2], target[3]) if isinstance(target, Table) else (target, None, None)
        s2 = self.sigma * self.sigma
        d = acc_float(x) - acc_float(t)
        if inw is not None:
            d = d * acc_float(inw)
        ad = d.abs()
        l = torch.where(ad < 1.0 / s2, 0.5 * d * d * s2, ad - 0.5 / s2)
        if outw is not None:
            l = l * acc_float(outw)
        s = l.sum()
        return s / self.num if self.num > 0 else s


class MarginCriterion(AutogradCriterion):
    def __init__(self, margin=1.0, size_average=True, squared=False, bigdl_type="float"):
        super().__init__(size_average)
        self.margin, self.squared = margin, squared

    def _loss(self, x, t):
        l = torch.clamp(self.margin - acc_float(x) * acc_float(t).reshape(x.shape), min=0)
        if self.squared:
            l = l * l
        return l.sum() / x.numel() if self.sizeAverage else l.sum()


class MarginRankingCriterion(AutogradCriterion):
    def __init__(self, margin=1.0, size_average=True, bigdl_type="float"):
        super().__init__(size_average)
        self.margin = margin

    def _loss(self, x, t):
        y = t[1] if isinstance(t, Table) else t
        l = torch.clamp(-acc_float(y) * (acc_float(x[1]) - acc_float(x[2])) + self.margin, min=0)
        return l.mean() if self.sizeAverage else l.sum()


class HingeEmbeddingCriterion(AutogradCriterion):
    def __init__(self, margin=1.0, size_average=True, bigdl_type="float"):
        super().__init__(size_average)
        self.margin = margin

    def _loss(self, x, t):
        t = acc_float(t).reshape(x.shape)
        l = torch.where(t > 0, acc_float(x), torch.clamp(self.margin - acc_float(x), min=0))
        return l.sum() / x.numel() if self.sizeAverage else l.sum()


class L1HingeEmbeddingCriterion(AutogradCriterion):
    def __init__(self, margin=1.0, bigdl_type="float"):
        super().__init__(False)
        self.margin = margin

    def _loss(self, x, t):
        d = (acc_float(x[1]) - acc_float(x[2])).abs().sum()
        y = float(t.reshape(-1)[0]) if isinstance(t, torch.Tensor) else float(t)
        return d if y > 0 else torch.clamp(self.margin - d, min=0)


class CosineEmbeddingCriterion(AutogradCriterion):
    def __init__(self, margin=0.0, size_average=True, bigdl_type="float"):
        super().__init__(size_average)
        self.margin = margin

    def _loss(self, x, t):
        y = t[1] if isinstance(t, Table) else t
        return F.cosine_embedding_loss(acc_float(x[1]), acc_float(x[2]), acc_float(y).reshape(-1), self.margin,
                                       reduction="mean" if self.sizeAverage else "sum")


class CosineDistanceCriterion(AutogradCriterion):
    def __init__(self, size_average=True, bigdl_type="float"):
        super().__init__(size_average)

    def _loss(self, x, t):
        l = 1 - F.cosine_similarity(acc_float(x), acc_float(t).reshape(x.shape), dim=-1)
        return l.mean() if self.sizeAverage else l.sum()


class DistKLDivCriterion(AutogradCriterion):
    """KL(target ‖ exp(input)) with log-prob input (``DistKLDivCriterion.scala``)."""

    def __init__(self, size_average=True, bigdl_type="float"):
        super().__init__(size_average)

    def _loss(self, x, t):
        t = acc_float(t).reshape(x.shape)
        l = torch.where(t > 0, t * (torch.log(t.clamp_min(1e-30)) - acc_float(x)), torch.zeros_like(t))
        return l.sum() / x.numel() if self.sizeAverage else l.sum()


class CategoricalCrossEntropy(AutogradCriterion):
    """Keras categorical crossentropy on probabilities with one-hot targets."""

    def __init__(self, bigdl_type="float"):
        super().__init__(True)

    def _loss(self, x, t):
        p = acc_float(x) / acc_float(x).sum(-1, keepdim=True)
        p = p.clamp(1e-7, 1 - 1e-7)
        return -(acc_float(t).reshape(p.shape) * torch.log(p)).sum(-1).mean()


class ClassSimplexCriterion(AutogradCriterion):
    """MSE against regular-simplex embeddings of the 1-based class (``ClassSimplexCriterion.scala``)."""

    def __init__(self, n_classes, bigdl_type="float"):
        super().__init__(True)
        self.nClasses = n_classes
        self.simplex = self._simplex(n_classes)

    @staticmethod
    def _simplex(k):
        n = k
        a = torch.zeros(n, n - 1 if n > 1 else 1, dtype=torch.float64)
        for kk in range(n - 1):
            a[kk, kk] = math.sqrt(max(1 - float((a[kk, :kk] ** 2).sum()), 0))
            c = (a[kk, kk] ** 2 - 1 - 1 / (n - 1)) / a[kk, kk]
            a[kk + 1:, kk] = c
        pad = torch.zeros(n, max(n, 1) - a.shape[1], dtype=torch.float64)
        return torch.cat([a, pad], 1).float()

    def _loss(self, x, t):
        s = self.simplex.to(x.device)[t.long().reshape(-1) - 1][:, :x.shape[-1]]
        d = acc_float(x) - s
        return (d * d).sum() / x.numel()


class MultiLabelMarginCriterion(AutogradCriterion):
    def __init__(self, size_average=True, bigdl_type="float"):
        super().__init__(size_average)

    def _loss(self, x, t):
        xx = acc_float(x) if x.dim() == 2 else acc_float(x).unsqueeze(0)
        tt = (t.long() if t.dim() == 2 else t.long().unsqueeze(0)) - 1  # 1-based, 0 terminates → -1
        return F.multilabel_margin_loss(xx, tt, reduction="mean" if self.sizeAverage else "sum")


class MultiLabelSoftMarginCriterion(AutogradCriterion):
    def __init__(self, weights=None, size_average=True, bigdl_type="float"):
        super().__init__(size_average)
        self.weights = None if weights is None else torch.as_tensor(weights, dtype=torch.float32)

    def _loss(self, x, t):
        w = None if self.weights is None else self.weights.to(x.device)
        l = F.binary_cross_entropy_with_logits(acc_float(x), acc_float(t).reshape(x.shape), weight=w, reduction="none")
        l = l.mean(-1)
        return l.mean() if self.sizeAverage else l.sum()


class MultiMarginCriterion(AutogradCriterion):
    def __init__(self, p=1, weights=None, margin=1.0, size_average=True, bigdl_type="float"):
        super().__init__(size_average)
        self.p, self.margin = p, margin
        self.weights = None if weights is None else torch.as_tensor(weights, dtype=torch.float32)

    def _loss(self, x, t):
        xx = acc_float(x) if x.dim() == 2 else acc_float(x).unsqueeze(0)
        w = None if self.weights is None else self.weights.to(x.device)
        return F.multi_margin_loss(xx, t.long().reshape(-1) - 1, self.p, self.margin, w,
                                   reduction="mean" if self.sizeAverage else "sum")


class SoftMarginCriterion(AutogradCriterion):
    def __init__(self, size_average=True, bigdl_type="float"):
        super().__init__(size_average)

    def _loss(self, x, t):
        return F.soft_margin_loss(acc_float(x), acc_float(t).reshape(x.shape), reduction="mean" if self.sizeAverage else "sum")


class DiceCoefficientCriterion(AutogradCriterion):
    def __init__(self, size_average=True, epsilon=1.0, bigdl_type="float"):
        super().__init__(size_average)
        self.epsilon = epsilon

    def _loss(self, x, t):
        xx = acc_float(x).reshape(x.shape[0], -1) if x.dim() > 1 else acc_float(x).unsqueeze(0)
        tt = acc_float(t).reshape(xx.shape)
        inter = (xx * tt).sum(1)
        l = 1 - (2 * inter + self.epsilon) / (xx.sum(1) + tt.sum(1) + self.epsilon)
        return l.mean() if self.sizeAverage else l.sum()


class L1Cost(AutogradCriterion):
    def __init__(self, bigdl_type="float"):
        super().__init__(False)

    def _loss(self, x, t):
        return acc_float(x).abs().sum()


class CosineProximityCriterion(AutogradCriterion):
    def __init__(self, bigdl_type="float"):
        super().__init__(True)

    def _loss(self, x, t):
        xn = F.normalize(acc_float(x), dim=-1)
        tn = F.normalize(acc_float(t).reshape(x.shape), dim=-1)
        return -(xn * tn).sum(-1).mean()


class MeanAbsolutePercentageCriterion(AutogradCriterion):
    def __init__(self, bigdl_type="float"):
        super().__init__(True)

    def _loss(self, x, t):
        t = acc_float(t).reshape(x.shape)
        return 100 * ((t - acc_float(x)).abs() / t.abs().clamp_min(1e-7)).mean()


class MeanSquaredLogarithmicCriterion(AutogradCriterion):
    def __init__(self, bigdl_type="float"):
        super().__init__(True)

    def _loss(self, x, t):
        t = acc_float(t).reshape(x.shape)
        a = torch.log(acc_float(x).clamp_min(1e-7) + 1)
        b = torch.log(t.clamp_min(1e-7) + 1)
        return ((a - b) ** 2).mean()


class KullbackLeiblerDivergenceCriterion(AutogradCriterion):
    def __init__(self, bigdl_type="float"):
        super().__init__(True)

    def _loss(self, x, t):
        xx = acc_float(x).clamp(1e-7, 1)
        tt = acc_float(t).reshape(x.shape).clamp(1e-7, 1)
        return (tt * torch.log(tt / xx)).sum(-1).mean()


class PoissonCriterion(AutogradCriterion):
    def __init__(self, bigdl_type="float"):
        super().__init__(True)

    def _loss(self, x, t):
        return (acc_float(x) - acc_float(t).reshape(x.shape) * torch.log(acc_float(x) + 1e-7)).mean()


class KLDCriterion(AutogradCriterion):
    """VAE KL of N(mean, exp(logvar)) to N(0,1): input Table(mean, logvar)."""

    def __init__(self, size_average=True, bigdl_type="float"):
        super().__init__(size_average)

    def _loss(self, x, t):
        mean, logvar = acc_float(x[1]), acc_float(x[2])
        l = -0.5 * (1 + logvar - mean * mean - torch.exp(logvar))
        return l.sum() / mean.shape[0] if self.sizeAverage else l.sum()


class GaussianCriterion(AutogradCriterion):
    """Negative log-likelihood of target under N(mean, exp(logvar)): input Table(mean, logvar)."""

    def __init__(self, bigdl_type="float"):
        super().__init__(False)

    def _loss(self, x, t):
        mean, logvar = acc_float(x[1]), acc_float(x[2])
        return (0.5 * math.log(2 * math.pi) + 0.5 * logvar + (acc_float(t) - mean) ** 2 / (2 * torch.exp(logvar))).sum()


class SoftmaxWithCriterion(AutogradCriterion):
    """Caffe SoftmaxWithLoss over dim 1 of (N, C, ...) with 1-based labels; ignore_label;
    normalize_mode ∈ FULL | VALID | BATCH_SIZE | NONE."""

    def __init__(self, ignore_label=None, normalize_mode="VALID", bigdl_type="float"):
        super().__init__(True)
        self.ignoreLabel, self.normalizeMode = ignore_label, normalize_mode

    def _loss(self, x, t):
        lp = torch.log_softmax(acc_float(x), dim=1)
        tt = t.long().reshape(lp.shape[0], *lp.shape[2:]) - 1
        valid = torch.ones_like(tt, dtype=torch.bool) if self.ignoreLabel is None else (tt != self.ignoreLabel - 1)
        picked = lp.gather(1, tt.clamp_min(0).unsqueeze(1)).squeeze(1)
        l = -(picked * acc_float(valid)).sum()
        mode = self.normalizeMode
        if mode == "FULL":
            return l / tt.numel()
        if mode == "VALID":
            return l / acc_float(valid).sum().clamp_min(1)
        if mode == "BATCH_SIZE":
            return l / lp.shape[0]
        return l


class TimeDistributedCriterion(AbstractCriterion):
    """Apply a criterion at every time step of (N, T, ...) and sum (average if sizeAverage)
    (``TimeDistributedCriterion.scala``)."""

    def __init__(self, criterion, size_average=False, dimension=2, bigdl_type="float"):
        super().__init__(size_average)
        self.critrn = criterion
        self.dimension = dimension

    def _fold(self, x, t):
        d = self.dimension - 1
        T = x.shape[d]
        xs = x.movedim(d, 1).reshape(x.shape[0] * T if d == 1 else -1, *x.shape[d + 1:]) if d == 1 else x
        ts = t.movedim(d, 1).reshape(-1, *t.shape[d + 1:]) if (t.dim() > d and d == 1) else t
        return xs, ts, T

    def updateOutput(self, input, target):
        d = self.dimension - 1
        T = input.shape[d]
        if d == 1 and isinstance(self.critrn, (ClassNLLCriterion, CrossEntropyCriterion)) and not self.critrn.sizeAverage is None:
            # fused path: fold time into batch; each step's loss is averaged over its batch
            x = input.reshape(-1, input.shape[-1])
            t = target.reshape(-1)
            N = input.shape[0]
            crit = self.critrn
            loss = crit.updateOutput(x, t)
            if crit.sizeAverage:
                loss = loss * T  # sum over steps of per-step batch means
            self._fused = True
            self._loss = loss
            return loss / T if self.sizeAverage else loss
        self._fused = False
        total = 0.0
        for i in range(T):
            total = total + self.critrn.forward(input.select(d, i), target.select(d, i) if target.dim() > d else target)
        return total / T if self.sizeAverage else total

    def updateGradInput(self, input, target):
        d = self.dimension - 1
        T = input.shape[d]
        if getattr(self, "_fused", False):
            x = input.reshape(-1, input.shape[-1])
            t = target.reshape(-1)
            g = self.critrn.updateGradInput(x, t)
            if self.critrn.sizeAverage:
                g = g * T
            if self.sizeAverage:
                g = g / T
            return g.reshape(input.shape)
        gi = torch.zeros_like(input, dtype=torch.float32)
        for i in range(T):
            g = self.critrn.backward(input.select(d, i), target.select(d, i) if target.dim() > d else target)
            gi.select(d, i).copy_(g)
            if self.sizeAverage:
                gi.select(d, i).div_(T)
        return gi


class TimeDistributedMaskCriterion(AbstractCriterion):
    """Like TimeDistributedCriterion but averages over non-padding targets."""

    def __init__(self, criterion, padding_value=0, bigdl_type="float"):
        super().__init__(True)
        self.critrn = criterion
        self.paddingValue = padding_value

    def updateOutput(self, input, target):
        T = input.shape[1]
        mask = (target != self.paddingValue).float()
        total = 0.0
        for i in range(T):
            total = total + self.critrn.forward(input.select(1, i), target.select(1, i)) * float(mask[:, i].sum())
        return total / max(float(mask.sum()), 1.0)

    def updateGradInput(self, input, target):
        T = input.shape[1]
        mask = (target != self.paddingValue).float()
        tot = max(float(mask.sum()), 1.0)
        gi = torch.zeros_like(input, dtype=torch.float32)
        for i in range(T):
            g = self.critrn.backward(input.select(1, i), target.select(1, i))
            gi.select(1, i).copy_(g * float(mask[:, i].sum()) / tot)
        return gi


class MultiCriterion(AbstractCriterion):
    """Weighted sum of criteria on the same input/target."""

    def __init__(self, bigdl_type="float"):
        super().__init__(True)
        self.criterions = []
        self.weights = []

    def add(self, criterion, weight=1.0):
        self.criterions.append(criterion)
        self.weights.append(weight)
        return self

    def updateOutput(self, input, target):
        return sum(w * c.forward(input, target) for c, w in zip(self.criterions, self.weights))

    def updateGradInput(self, input, target):
        g = None
        for c, w in zip(self.criterions, self.weights):
            gi = c.backward(input, target) * w
            g = gi if g is None else g + gi
        return g


class ParallelCriterion(AbstractCriterion):
    """i-th criterion on i-th input (and target unless repeat_target)."""

    def __init__(self, repeat_target=False, bigdl_type="float"):
        super().__init__(True)
        self.repeatTarget = repeat_target
        self.criterions = []
        self.weights = []

    def add(self, criterion, weight=1.0):
        self.criterions.append(criterion)
        self.weights.append(weight)
        return self

    def updateOutput(self, input, target):
        total = 0.0
        for i, (c, w) in enumerate(zip(self.criterions, self.weights)):
            t = target if self.repeatTarget else target[i + 1]
            total = total + w * c.forward(input[i + 1], t)
        return total

    def updateGradInput(self, input, target):
        gi = Table()
        for i, (c, w) in enumerate(zip(self.criterions, self.weights)):
            t = target if self.repeatTarget else target[i + 1]
            gi[i + 1] = c.backward(input[i + 1], t) * w
        return gi


class TransformerCriterion(AbstractCriterion):
    """Apply transformer modules to input/target before the criterion."""

    def __init__(self, criterion, input_transformer=None, target_transformer=None, bigdl_type="float"):
        super().__init__(True)
        self.criterion, self.inputTransformer, self.targetTransformer = criterion, input_transformer, target_transformer

    def updateOutput(self, input, target):
        x = self.inputTransformer.forward(input) if self.inputTransformer else input
        t = self.targetTransformer.forward(target) if self.targetTransformer else target
        self._xt = (x, t)
        return self.criterion.forward(x, t)

    def updateGradInput(self, input, target):
        x, t = self._xt
        g = self.criterion.backward(x, t)
        if self.inputTransformer:
            g = self.inputTransformer.backward(input, g)
        return g


class DotProductCriterion(AbstractCriterion):
    def __init__(self, size_average=False, bigdl_type="float"):
        super().__init__(size_average)

    def updateOutput(self, input, target):
        s = (acc_float(input) * acc_float(target)).sum()
        return s / input.shape[0] if self.sizeAverage else s

    def updateGradInput(self, input, target):
        g = acc_float(target).reshape(input.shape)
        return g / input.shape[0] if self.sizeAverage else g


class PGCriterion(AbstractCriterion):
    """Policy-gradient loss −Σ log(p)·reward (``PGCriterion.scala``)."""

    def __init__(self, sizeAverage=False, bigdl_type="float"):
        super().__init__(sizeAverage)

    def updateOutput(self, input, target):
        l = -(torch.log(acc_float(input).clamp_min(1e-12)) * acc_float(target)).sum()
        return l / input.shape[0] if self.sizeAverage else l

    def updateGradInput(self, input, target):
        g = -acc_float(target) / acc_float(input).clamp_min(1e-12)
        return g / input.shape[0] if self.sizeAverage else g


Criterion = AbstractCriterion  # pyspark ``bigdl.nn.criterion.Criterion``
