"""Parameter processors: global gradient transforms applied between the gradient all-reduce and the
optimizer update (reference ``DL/parameters/ParameterOperations.scala:33-115``,
``DL/optim/LarsSGD.scala:288-330``).

The reference runs each processor in two phases over the Spark-partitioned gradient: a
``collectGlobalData`` RDD reduce (e.g. Σg² over every partition) and a per-partition
``processParameters``.  Here a rank owns a contiguous shard of the flat fp32 gradient arena (after
the RCCL reduce-scatter), and the global reduction is one ``all_reduce`` of a small vector
(``global_sum``; identity on one process), so a processor is:

    state = {}
    for p in processors: p.collect_global_data(weight_shard, grad_shard, state, global_sum)
    for p in processors: p.process_parameters(grad_shard, state)

``Optimizer.setConstantGradientClipping`` / ``setGradientClippingByl2Norm`` install
:class:`ConstantClippingProcessor` / :class:`L2NormClippingProcessor` (``Optimizer.scala:76,
688``).  Every collective is issued by all ranks in the same order (one per processor), which keeps
RCCL's call sequence identical across ranks.
"""
from __future__ import annotations

import math
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch

GlobalSum = Callable[[torch.Tensor], torch.Tensor]


def _identity(t: torch.Tensor) -> torch.Tensor:
    return t


def sum_square(t: torch.Tensor) -> torch.Tensor:
    """Σ t² in fp32 as a 0-d tensor on t's device (``Util.getSumsquareInParallel``)."""
    return t.float().pow(2).sum()


def global_l2_norm(grad_shard: torch.Tensor, global_sum: GlobalSum = _identity) -> torch.Tensor:
    """‖g‖₂ of the whole (sharded) gradient."""
    return torch.sqrt(global_sum(sum_square(grad_shard)))


class ParameterProcessor:
    def collect_global_data(self, weight_shard: Optional[torch.Tensor], grad_shard: torch.Tensor,
                            state: Dict, global_sum: GlobalSum = _identity) -> None:
        pass

    def process_parameters(self, grad_shard: torch.Tensor, state: Dict) -> None:
        pass

    collectGlobalData = collect_global_data
    processParameters = process_parameters


class ConstantClippingProcessor(ParameterProcessor):
    """Clamp every gradient element into [min, max] (``ParameterOperations.scala:71-87``)."""

    def __init__(self, min_value: float, max_value: float):
        if min_value > max_value:
            raise ValueError(f"min {min_value} > max {max_value}")
        self.min, self.max = float(min_value), float(max_value)

    def process_parameters(self, grad_shard, state):
        grad_shard.clamp_(self.min, self.max)


class L2NormClippingProcessor(ParameterProcessor):
    """Scale the gradient by min(1, threshold / ‖g‖₂) (``ParameterOperations.scala:89-115``); the
    norm is taken over the gradient as collected, before any processor of the same step ran."""

    def __init__(self, l2_norm_threshold: float):
        if l2_norm_threshold <= 0:
            raise ValueError("l2NormThreshold must be positive")
        self.threshold = float(l2_norm_threshold)

    def collect_global_data(self, weight_shard, grad_shard, state, global_sum=_identity):
        state["l2Norm"] = global_l2_norm(grad_shard, global_sum)

    def process_parameters(self, grad_shard, state):
        norm = state["l2Norm"]
        # stays on the device (no host sync): scale = min(1, thr / ‖g‖)
        scale = torch.clamp(self.threshold / (norm + 1e-6), max=1.0)
        grad_shard.mul_(scale.to(grad_shard.dtype))


class LarsProcessor(ParameterProcessor):
    """Per-layer LARS scale (‖g_l‖ + wd·‖w_l‖) / ‖w_l‖ (``LarsSGD.scala:288-330``).

    ``parameter_splits`` maps a layer name to its (offset, length) in the flat arena;
    ``shard_range`` is the (offset, length) of this rank's shard.  The per-layer Σw², Σg² of the
    local intersection are packed into ONE vector and summed across ranks with a single collective
    (the reference's ``reduceByKey``).  Result: ``state["larsScale"][name]`` (python floats)."""

    def __init__(self, parameter_splits: Dict[str, Tuple[int, int]], weight_decay: float,
                 shard_range: Optional[Tuple[int, int]] = None):
        self.splits = dict(parameter_splits)
        self.weight_decay = float(weight_decay)
        self.shard_range = shard_range

    def collect_global_data(self, weight_shard, grad_shard, state, global_sum=_identity):
        lo, n = self.shard_range if self.shard_range is not None else (0, grad_shard.numel())
        names = sorted(self.splits)
        sums = torch.zeros(2 * len(names), dtype=torch.float32, device=grad_shard.device)
        for i, name in enumerate(names):
            off, ln = self.splits[name]
            s, e = max(lo, off), min(lo + n, off + ln)
            if e > s:
                sums[2 * i] = sum_square(weight_shard[s - lo:e - lo])
                sums[2 * i + 1] = sum_square(grad_shard[s - lo:e - lo])
        sums = global_sum(sums).tolist()
        scales = {}
        for i, name in enumerate(names):
            nw, ng = math.sqrt(sums[2 * i]), math.sqrt(sums[2 * i + 1])
            scales[name] = (ng + self.weight_decay * nw) / nw if nw > 0 else 1.0
        state["larsScale"] = scales


def run_processors(processors: Sequence[ParameterProcessor], weight_shard: Optional[torch.Tensor],
                   grad_shard: torch.Tensor, global_sum: GlobalSum = _identity) -> Dict:
    """Both phases of every processor over this rank's shard; returns the shared state table."""
    state: Dict = {}
    for p in processors:
        p.collect_global_data(weight_shard, grad_shard, state, global_sum)
    for p in processors:
        p.process_parameters(grad_shard, state)
    return state


ParameterOperations = run_processors

__all__ = ["ParameterProcessor", "ConstantClippingProcessor", "L2NormClippingProcessor", "LarsProcessor",
           "run_processors", "ParameterOperations", "global_l2_norm", "sum_square"]
