"""Validation methods and mergeable results (``DL/optim/ValidationMethod.scala:37-1117``).

Each method maps (output, target) → a ``ValidationResult`` that supports ``+`` so per-rank
partials can be merged; :func:`allreduce_results` merges them across ranks with ONE RCCL
all-reduce of a small fp64 vector (X12).  Targets are 1-based class indices.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..utils.table import Table


class ValidationResult:
    def result(self):
        raise NotImplementedError

    def __add__(self, other):
        raise NotImplementedError

    def to_vector(self):
        raise NotImplementedError

    def from_vector(self, v):
        raise NotImplementedError


class AccuracyResult(ValidationResult):
    def __init__(self, correct=0, count=0):
        self.correct, self.count = int(correct), int(count)

    def result(self):
        return (self.correct / self.count if self.count else 0.0), self.count

    def __add__(self, o):
        return AccuracyResult(self.correct + o.correct, self.count + o.count)

    def to_vector(self):
        return [self.correct, self.count]

    def from_vector(self, v):
        return AccuracyResult(v[0], v[1])

    def __repr__(self):
        r, n = self.result()
        return f"Accuracy(correct: {self.correct}, count: {self.count}, accuracy: {r})"


class LossResult(ValidationResult):
    def __init__(self, loss=0.0, count=0):
        self.loss, self.count = float(loss), int(count)

    def result(self):
        return (self.loss / self.count if self.count else 0.0), self.count

    def __add__(self, o):
        return LossResult(self.loss + o.loss, self.count + o.count)

    def to_vector(self):
        return [self.loss, self.count]

    def from_vector(self, v):
        return LossResult(v[0], int(v[1]))

    def __repr__(self):
        return f"(Loss: {self.loss}, count: {self.count}, Average Loss: {self.result()[0]})"


class ContiguousResult(LossResult):
    def __repr__(self):
        return f"(Average score: {self.result()[0]}, count: {self.count})"


class ValidationMethod:
    SCALA_PACKAGE = "com.intel.analytics.bigdl.optim"

    def __call__(self, output, target) -> ValidationResult:
        raise NotImplementedError

    def format(self):
        return type(self).__name__

    def __repr__(self):
        return self.format()


def _to_2d(output):
    if isinstance(output, Table):
        output = output[1]
    return output.unsqueeze(0) if output.dim() == 1 else output


class Top1Accuracy(ValidationMethod):
    def __call__(self, output, target):
        o = _to_2d(output).float()
        if target.dim() == 2 and target.shape == o.shape and o.shape[1] > 1:
            # one-hot / probability targets (Keras "accuracy" with categorical_crossentropy)
            target = target.float().argmax(1) + 1
        t = target.reshape(-1).long()
        if o.shape[1] == 1:  # binary
            pred = (o.reshape(-1) > 0.5).long()
            correct = int((pred == t).sum())
        else:
            pred = o.argmax(1) + 1
            correct = int((pred == t).sum())
        return AccuracyResult(correct, t.numel())


class Top5Accuracy(ValidationMethod):
    def __call__(self, output, target):
        o = _to_2d(output).float()
        t = target.reshape(-1).long()
        k = min(5, o.shape[1])
        top = o.topk(k, dim=1)[1] + 1
        correct = int((top == t.unsqueeze(1)).any(1).sum())
        return AccuracyResult(correct, t.numel())


class TreeNNAccuracy(ValidationMethod):
    def __call__(self, output, target):
        o = output.float()
        if o.dim() == 3:
            o = o[:, 0, :]          # node 1 = the root in the TensorTree encoding
        elif o.dim() == 2:
            o = o[0:1, :]
        t = target.float()
        t = t[:, 0] if t.dim() == 2 else t.reshape(-1)[:1]
        # one output unit = binary classifier thresholded at 0.5 (``ValidationMethod.scala:121-166``)
        pred = (o[:, 0] >= 0.5).float() if o.shape[-1] == 1 else o.argmax(-1) + 1
        return AccuracyResult(int((pred == t.long()).sum()), t.numel())


class Loss(ValidationMethod):
    def __init__(self, criterion=None):
        from ..nn.criterion import ClassNLLCriterion
        self.criterion = criterion or ClassNLLCriterion()

    def __call__(self, output, target):
        n = output.shape[0] if isinstance(output, torch.Tensor) and output.dim() > 1 else 1
        loss = float(self.criterion.forward(output, target))
        return LossResult(loss * n, n)


class MAE(ValidationMethod):
    def __call__(self, output, target):
        o = output.float()
        d = (o - target.float().reshape(o.shape)).abs()
        n = o.shape[0] if o.dim() > 1 else 1
        return ContiguousResult(float(d.sum()) / (d.numel() / n), n)


class HitRatio(ValidationMethod):
    """HR@k for recommendation (``ValidationMethod.scala`` HitRatio): output scores of one
    positive + negNum negatives; target marks the positive with 1."""

    def __init__(self, k=10, neg_num=100):
        self.k, self.negNum = k, neg_num

    def __call__(self, output, target):
        o = output.reshape(-1).float()
        t = target.reshape(-1).float()
        pos = int(t.argmax())
        rank = int((o > o[pos]).sum()) + 1
        return ContiguousResult(1.0 if rank <= self.k else 0.0, 1)


class NDCG(HitRatio):
    def __call__(self, output, target):
        o = output.reshape(-1).float()
        t = target.reshape(-1).float()
        pos = int(t.argmax())
        rank = int((o > o[pos]).sum()) + 1
        return ContiguousResult(math.log(2) / math.log(rank + 1) if rank <= self.k else 0.0, 1)


class MeanAveragePrecision(ValidationMethod):
    """Multi-class mAP over (N, C) scores and 1-based labels (``MeanAveragePrecision``)."""

    def __init__(self, k, classes):
        self.k, self.classes = k, classes

    def __call__(self, output, target):
        o = _to_2d(output).float().cpu()
        t = target.reshape(-1).long().cpu()
        aps = []
        for c in range(self.classes):
            scores = o[:, c]
            order = torch.argsort(scores, descending=True)[: self.k if self.k > 0 else len(scores)]
            rel = (t[order] == c + 1).float()
            if rel.sum() == 0:
                continue
            prec = torch.cumsum(rel, 0) / torch.arange(1, len(rel) + 1)
            aps.append(float((prec * rel).sum() / rel.sum()))
        return ContiguousResult(float(np.mean(aps)) if aps else 0.0, 1)


class MeanAveragePrecisionObjectDetection(ValidationMethod):
    """Detection mAP (VOC07 11-point / VOC10 / COCO-style IoU sweep) over per-image detections
    Table{(label, score, x1,y1,x2,y2)} and ground truth (label, difficult, x1,y1,x2,y2)."""

    def __init__(self, classes, iou=0.5, use_voc2007=False, skip_class=-1):
        self.classes, self.iou, self.voc07, self.skip = classes, iou, use_voc2007, skip_class
        self._dets = {c: [] for c in range(classes)}
        self._npos = {c: 0 for c in range(classes)}

    @staticmethod
    def _iou(a, b):
        ix1, iy1 = max(a[0], b[0]), max(a[1], b[1])
        ix2, iy2 = min(a[2], b[2]), min(a[3], b[3])
        iw, ih = max(ix2 - ix1 + 1, 0), max(iy2 - iy1 + 1, 0)
        inter = iw * ih
        ua = (a[2] - a[0] + 1) * (a[3] - a[1] + 1) + (b[2] - b[0] + 1) * (b[3] - b[1] + 1) - inter
        return inter / ua if ua > 0 else 0.0

    def __call__(self, output, target):
        dets = output.reshape(-1, 6).tolist()
        gts = target.reshape(-1, 6).tolist()
        used = [False] * len(gts)
        for g in gts:
            if int(g[0]) != self.skip and not g[1]:
                self._npos[int(g[0])] = self._npos.get(int(g[0]), 0) + 1
        for d in sorted(dets, key=lambda r: -r[1]):
            c = int(d[0])
            best, bj = 0.0, -1
            for j, g in enumerate(gts):
                if int(g[0]) == c:
                    o = self._iou(d[2:], g[2:])
                    if o > best:
                        best, bj = o, j
            tp = best >= self.iou and bj >= 0 and not used[bj]
            if tp:
                used[bj] = True
            self._dets.setdefault(c, []).append((d[1], 1 if tp else 0))
        return ContiguousResult(self.mAP(), 1)

    def mAP(self):
        aps = []
        for c in range(self.classes):
            if c == self.skip or self._npos.get(c, 0) == 0:
                continue
            ds = sorted(self._dets.get(c, []), key=lambda r: -r[0])
            tp = np.cumsum([x[1] for x in ds]) if ds else np.zeros(0)
            fp = np.cumsum([1 - x[1] for x in ds]) if ds else np.zeros(0)
            rec = tp / self._npos[c] if len(tp) else np.zeros(0)
            prec = tp / np.maximum(tp + fp, 1e-12) if len(tp) else np.zeros(0)
            if self.voc07:
                ap = np.mean([np.max(prec[rec >= t]) if np.any(rec >= t) else 0 for t in np.arange(0, 1.1, 0.1)])
            else:
                mrec = np.concatenate([[0], rec, [1]])
                mpre = np.concatenate([[0], prec, [0]])
                for i in range(len(mpre) - 1, 0, -1):
                    mpre[i - 1] = max(mpre[i - 1], mpre[i])
                idx = np.where(mrec[1:] != mrec[:-1])[0]
                ap = np.sum((mrec[idx + 1] - mrec[idx]) * mpre[idx + 1])
            aps.append(ap)
        return float(np.mean(aps)) if aps else 0.0


class PRAUCResult(ValidationResult):
    """(score, label) pairs; ``result()`` = area under the precision-recall curve
    (``PrecisionRecallAUC.scala``: scores sorted descending, trapezoids in (recall, precision)
    starting from (0, 1), stopping once every positive is recalled)."""

    gather = True  # variable-size: merged by all-gather, not by a fixed-size all-reduce

    def __init__(self, results=None):
        self.results = list(results or [])

    def result(self):
        srt = sorted(self.results, key=lambda r: r[0], reverse=True)
        total_pos = sum(1 for _, t in srt if t == 1.0)
        tp = fp = 0.0
        auc, prev_p, prev_r = 0.0, 1.0, 0.0
        i = 0
        while tp != total_pos:
            if srt[i][1] == 1.0:
                tp += 1
            else:
                fp += 1
            prec, rec = tp / (tp + fp), tp / total_pos
            auc += (rec - prev_r) * (prec + prev_p)
            prev_r, prev_p = rec, prec
            i += 1
        return auc / 2, len(self.results)

    def __add__(self, o):
        return PRAUCResult(self.results + o.results)

    def __repr__(self):
        r, n = self.result()
        return f"Precision Recall AUC is {r} on {n}"


class PrecisionRecallAUC(ValidationMethod):
    """Binary PR-AUC over (score, 0/1 label) tensors of the same size."""

    def __call__(self, output, target):
        o = output.detach().float().reshape(-1).cpu().tolist()
        t = target.detach().float().reshape(-1).cpu().tolist()
        if not o or not t:
            raise ValueError("the output and target should not be empty")
        return PRAUCResult(list(zip(o, t)))

    def format(self):
        return "PrecisionRecallAUC"


class EvaluateMethods:
    """``EvaluateMethods.calcAccuracy`` / ``calcTop5Accuracy``: (correct, count) for a batch of
    scores (N, C) or one score vector (C) against 1-based targets."""

    @staticmethod
    def _rows(output, target):
        o = output.detach().float()
        t = target.detach().reshape(-1).long()
        if o.dim() == 1:
            if t.numel() != 1:
                raise ValueError("a single score vector needs a single target")
            o = o.unsqueeze(0)
        elif o.dim() != 2:
            raise ValueError("output must be 1-D or 2-D")
        return o, t

    @staticmethod
    def calcAccuracy(output, target):
        o, t = EvaluateMethods._rows(output, target)
        return int(((o.argmax(1) + 1).cpu() == t.cpu()).sum()), o.shape[0]

    @staticmethod
    def calcTop5Accuracy(output, target):
        o, t = EvaluateMethods._rows(output, target)
        top = o.topk(min(5, o.shape[1]), 1).indices.cpu() + 1
        return int((top == t.cpu()[:, None]).any(1).sum()), o.shape[0]


def allreduce_results(results):
    """Merge per-rank results (X12): one all-reduce of the concatenated small vectors; variable-size
    results (``gather = True``, e.g. PR-AUC pairs) are all-gathered and summed instead."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
        return results
    if any(getattr(r, "gather", False) for r in results):
        gathered = [None] * dist.get_world_size()
        dist.all_gather_object(gathered, results)
        out = list(gathered[0])
        for other in gathered[1:]:
            out = [a + b for a, b in zip(out, other)]
        return out
    vecs = [r.to_vector() for r in results]
    lens = [len(v) for v in vecs]
    flat = torch.tensor([x for v in vecs for x in v], dtype=torch.float64)
    if dist.get_backend() == "nccl":
        flat = flat.cuda()
    dist.all_reduce(flat)
    flat = flat.cpu().tolist()
    out, p = [], 0
    for r, n in zip(results, lens):
        out.append(r.from_vector(flat[p:p + n]))
        p += n
    return out
