"""Triggers over the driver state table (``DL/optim/Trigger.scala:26-155``).

State keys: ``epoch`` (1-based), ``neval`` (1-based iteration counter), ``Loss``, ``score``,
``recordsProcessedThisEpoch``.
"""
from __future__ import annotations


class Trigger:
    SCALA_PACKAGE = "com.intel.analytics.bigdl.optim"

    def __call__(self, state) -> bool:
        raise NotImplementedError

    @staticmethod
    def everyEpoch():
        return EveryEpoch()

    @staticmethod
    def severalIteration(interval):
        return SeveralIteration(interval)

    @staticmethod
    def maxEpoch(m):
        return MaxEpoch(m)

    @staticmethod
    def maxIteration(m):
        return MaxIteration(m)

    @staticmethod
    def maxScore(m):
        return MaxScore(m)

    @staticmethod
    def minLoss(m):
        return MinLoss(m)

    @staticmethod
    def and_(*t):
        return TriggerAnd(*t)

    @staticmethod
    def or_(*t):
        return TriggerOr(*t)


class EveryEpoch(Trigger):
    def __init__(self, bigdl_type="float"):
        self.lastEpoch = -1

    def __call__(self, state):
        if self.lastEpoch == -1:
            self.lastEpoch = state.get("epoch", 1)
            return False
        e = state.get("epoch", 1)
        if e == self.lastEpoch:
            return False
        self.lastEpoch = e
        return True


class SeveralIteration(Trigger):
    def __init__(self, interval, bigdl_type="float"):
        self.interval = interval

    def __call__(self, state):
        n = state.get("neval", 1) - 1
        return n > 0 and n % self.interval == 0


class MaxEpoch(Trigger):
    def __init__(self, max_epoch, bigdl_type="float"):
        self.max = max_epoch

    def __call__(self, state):
        return state.get("epoch", 1) > self.max


class MaxIteration(Trigger):
    def __init__(self, max_iteration, bigdl_type="float"):
        self.max = max_iteration

    def __call__(self, state):
        return state.get("neval", 1) > self.max


class MaxScore(Trigger):
    def __init__(self, max_score, bigdl_type="float"):
        self.max = max_score

    def __call__(self, state):
        s = state.get("score")
        return s is not None and float(s) > self.max


class MinLoss(Trigger):
    def __init__(self, min_loss, bigdl_type="float"):
        self.min = min_loss

    def __call__(self, state):
        l = state.get("Loss")
        return l is not None and float(l) < self.min


class TriggerAnd(Trigger):
    def __init__(self, first, *others, bigdl_type="float"):
        self.triggers = [first, *others]

    def __call__(self, state):
        return all(t(state) for t in self.triggers)


class TriggerOr(Trigger):
    def __init__(self, first, *others, bigdl_type="float"):
        self.triggers = [first, *others]

    def __call__(self, state):
        return any(t(state) for t in self.triggers)
