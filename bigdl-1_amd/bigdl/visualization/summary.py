"""TrainSummary / ValidationSummary (``DL/visualization/{Summary,TrainSummary,ValidationSummary}.scala``).

``TrainSummary(log_dir, app_name)`` writes to ``log_dir/app_name/train``; ``ValidationSummary``
to ``log_dir/app_name/validation``.  Scalars ("Loss", "Throughput", "LearningRate" — every
iteration by default, ``TrainSummary.scala:37-40``) and histograms ("Parameters", off by default)
are written as TensorBoard events; ``read_scalar(tag)`` returns ``[(step, value, wall_time)]``.

Histograms use the reference's bucket limits (±1e-12·1.1^i, 1549 edges, ``Summary.scala``
``makeHistogramBuckets``); the bucketing runs on the tensor's device (``torch.bucketize``) so only
the non-empty counts leave HBM.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from .tensorboard import FileReader, FileWriter, HistogramProto, Summary as _SummaryPB


def _make_buckets() -> np.ndarray:
    b = np.zeros(1549, dtype=np.float64)
    v = 1e-12
    for i in range(1, 775):
        b[774 + i] = v
        b[774 - i] = -v
        v *= 1.1
    return b


_LIMITS = _make_buckets()
_LIMITS_T: Dict[torch.device, torch.Tensor] = {}


def scalar(tag: str, value: float):
    s = _SummaryPB()
    v = s.value.add()
    v.tag = tag
    v.simple_value = float(value)
    return s


def histogram(tag: str, values) -> "_SummaryPB":
    t = values if isinstance(values, torch.Tensor) else torch.as_tensor(np.asarray(values))
    t = t.detach().reshape(-1)
    if not t.is_floating_point():
        t = t.float()
    t64 = t.double() if t.device.type == "cpu" else t.float()
    lim = _LIMITS_T.get(t.device)
    if lim is None:
        lim = torch.as_tensor(_LIMITS, dtype=t64.dtype, device=t.device)
        _LIMITS_T[t.device] = lim
    # bisect_left semantics of the reference: index of the first limit >= v
    idx = torch.bucketize(t64, lim, right=False).clamp_max(len(_LIMITS) - 1)
    counts = torch.bincount(idx, minlength=len(_LIMITS)).cpu().numpy()
    h = HistogramProto()
    if t.numel():
        h.min = float(t64.min())
        h.max = float(t64.max())
        h.sum = float(t64.sum())
        h.sum_squares = float((t64 * t64).sum())
    h.num = float(t.numel())
    nz = np.nonzero(counts)[0]
    h.bucket_limit.extend(_LIMITS[nz].tolist())
    h.bucket.extend(counts[nz].astype(np.float64).tolist())
    s = _SummaryPB()
    v = s.value.add()
    v.tag = tag
    v.histo.CopyFrom(h)
    return s


class Summary:
    """Base: ``add_scalar``, ``add_histogram``, ``read_scalar``, ``close``."""

    def __init__(self, log_dir: str, app_name: str, sub: str):
        self.log_dir = log_dir
        self.app_name = app_name
        self.folder = os.path.join(log_dir, app_name, sub)
        self._writer: Optional[FileWriter] = None
        self._triggers: Dict[str, object] = {}

    @property
    def writer(self) -> FileWriter:
        if self._writer is None:
            self._writer = FileWriter(self.folder)
        return self._writer

    def add_scalar(self, tag: str, value: float, step: int):
        self.writer.add_summary(scalar(tag, value), step)
        return self

    addScalar = add_scalar

    def add_histogram(self, tag: str, value, step: int):
        self.writer.add_summary(histogram(tag, value), step)
        return self

    addHistogram = add_histogram

    def read_scalar(self, tag: str) -> List[Tuple[int, float, float]]:
        if self._writer is not None:
            self._writer.flush()
        return FileReader.read_scalar(self.folder, tag)

    readScalar = read_scalar

    def should_write(self, tag: str, state) -> bool:
        trig = self._triggers.get(tag)
        return trig is not None and bool(trig(state))

    def flush(self):
        if self._writer is not None:
            self._writer.flush()

    def close(self):
        if self._writer is not None:
            self._writer.close()
            self._writer = None


class TrainSummary(Summary):
    """``TrainSummary.scala:32-95``.  Supported tags: LearningRate, Loss, Throughput, Parameters."""

    _TAGS = ("LearningRate", "Loss", "Throughput", "Parameters")

    def __init__(self, log_dir: str, app_name: str):
        super().__init__(log_dir, app_name, "train")
        from ..optim.trigger import SeveralIteration
        self._triggers = {"Loss": SeveralIteration(1), "Throughput": SeveralIteration(1),
                          "LearningRate": SeveralIteration(1)}

    def set_summary_trigger(self, tag: str, trigger):
        if tag not in self._TAGS:
            raise ValueError("TrainSummary: only support LearningRate, Loss, Parameters and Throughput")
        self._triggers[tag] = trigger
        return self

    setSummaryTrigger = set_summary_trigger

    def get_summary_trigger(self, tag: str):
        return self._triggers.get(tag)

    getSummaryTrigger = get_summary_trigger

    def get_scalar_triggers(self):
        return [(k, v) for k, v in self._triggers.items() if k != "Parameters"]


class ValidationSummary(Summary):
    """``ValidationSummary.scala``: one scalar per validation method, written on validation."""

    def __init__(self, log_dir: str, app_name: str):
        super().__init__(log_dir, app_name, "validation")

    def should_write(self, tag: str, state) -> bool:
        return True
