"""Optimisation methods (``DL/optim/OptimMethod.scala:28-180`` and friends).

Interface kept: ``optimize(feval, x) -> (x, [fx])`` where ``feval(x) -> (loss, grad)``;
``state`` holds ``epoch``/``neval``/``evalCounter`` and the method's buffers; hyper-parameters
are attributes (``loadFromTable`` / ``getHyperParameter`` / ``updateHyperParameter``).

Device path: ``x``/``grad`` are flat fp32 arenas (or this rank's shard of one); the whole update is
ONE fused HIP kernel over the flat buffer (``ops.sgd_step`` / ``ops.adam_step``, K22) that also
folds in the 1/N gradient averaging (``grad_scale``) and writes the bf16 shadow copy used by the
next forward.  ``SGD``'s learning rate follows the reference's negative ``clr`` convention
(``SGD.scala:61-124``): schedules produce ``currentRate = -lr``.
"""
from __future__ import annotations

import math
from typing import Callable, List, Optional

import torch

from .. import ops
from ..utils.table import Table


class OptimMethod:
    SCALA_PACKAGE = "com.intel.analytics.bigdl.optim"

    def __init__(self):
        self.state = {"epoch": 1, "neval": 1, "evalCounter": 0}
        #: fold the data-parallel gradient average into the fused update
        self.grad_scale = 1.0
        #: optional bf16 shadow of x written by the fused kernel
        self.shadow: Optional[torch.Tensor] = None

    def optimize(self, feval: Callable, x: torch.Tensor):
        raise NotImplementedError

    # ---- HIP-graph capture (optim/graph_step.py) ----------------------------------------------
    def prepare_graph(self) -> bool:
        """Switch to a replay-safe form (no per-iteration host scalars baked into kernels); False
        when this method/configuration cannot be captured."""
        return False

    def after_graph_replay(self):
        """Advance the host-side counters one iteration (a replay runs no Python)."""
        self.state["evalCounter"] = self.state.get("evalCounter", 0) + 1

    def sync_device_counter(self):
        """Set the device-side iteration counter (graph mode) from the host ``evalCounter`` — after
        a checkpoint restore or when a graph capture's warmup steps are undone."""
        nt = self.state.get("_dev_n")
        if isinstance(nt, torch.Tensor):
            nt.fill_(float(self.state.get("evalCounter", 0)))

    def graph_state_restored(self, fresh):
        """Called after a graph capture's warmup was undone; ``fresh`` = state keys the warmup
        created (now zeroed)."""

    def clearHistory(self):
        keep = {k: self.state[k] for k in ("epoch", "neval", "evalCounter", "recordsProcessedThisEpoch", "Loss",
                                           "score", "trainingTime") if k in self.state}
        self.state = keep
        return self

    def updateHyperParameter(self):
        pass

    def getHyperParameter(self) -> str:
        return ""

    def getLearningRate(self) -> float:
        return float("nan")

    def loadFromTable(self, config):
        for k, v in (config.items() if isinstance(config, (dict, Table)) else []):
            if hasattr(self, k):
                setattr(self, k, v)
        return self

    def clone(self):
        import copy
        return copy.deepcopy(self)

    def save(self, path: str, overWrite: bool = False):
        from ..serialization.checkpoint import save_optim_method
        save_optim_method(self, path, overWrite)
        return self

    @staticmethod
    def load(path: str) -> "OptimMethod":
        from ..serialization.checkpoint import load_optim_method
        return load_optim_method(path)

    @classmethod
    def scala_class_name(cls):
        return f"{cls.SCALA_PACKAGE}.{cls.__name__}"

    # --- bucketed update API used by the distributed driver ------------------------------------
    #: True when ``apply_update`` can update an arbitrary slice independently (fused kernels)
    supports_slices = False

    def begin_iteration(self, x: torch.Tensor):
        """Advance schedules once per iteration before any ``apply_update`` on slices of ``x``."""
        raise NotImplementedError

    def apply_update(self, x: torch.Tensor, g: torch.Tensor, lo: int, hi: int, shadow=None):
        raise NotImplementedError

    def _state_tensor(self, name: str, like: torch.Tensor, init: str = "zeros") -> torch.Tensor:
        t = self.state.get(name)
        if not isinstance(t, torch.Tensor) or t.shape != like.shape or t.device != like.device:
            t = torch.zeros_like(like, dtype=torch.float32)
            self.state[name] = t
        return t


# ----------------------------------------------------------------------------------------- LR schedules
class LearningRateSchedule:
    def __init__(self):
        self.currentRate = 0.0
        self.excludeIterations = 0
        self.excludeEpochs = 0
        self.maxIterations = 2 ** 31 - 1

    def updateHyperParameter(self, method: "SGD"):
        raise NotImplementedError

    def _bump(self, method):
        n = method.state.get("evalCounter", 0)
        method.state["evalCounter"] = n + 1
        return n


class Default(LearningRateSchedule):
    def updateHyperParameter(self, m):
        n = self._bump(m)
        self.currentRate = -m.learningRate / (1 + (n - self.excludeIterations) * m.learningRateDecay)


class Step(LearningRateSchedule):
    def __init__(self, step_size, gamma):
        super().__init__()
        self.stepSize, self.gamma = step_size, gamma

    def updateHyperParameter(self, m):
        n = self._bump(m)
        self.currentRate = -m.learningRate * self.gamma ** max(0, (n - self.excludeIterations) // self.stepSize)


class MultiStep(LearningRateSchedule):
    def __init__(self, step_sizes, gamma):
        super().__init__()
        self.stepSizes, self.gamma = list(step_sizes), gamma

    def updateHyperParameter(self, m):
        n = self._bump(m)
        k = sum(1 for s in self.stepSizes if (n - self.excludeIterations) >= s)
        self.currentRate = -m.learningRate * self.gamma ** k


class EpochStep(LearningRateSchedule):
    def __init__(self, step_size, gamma):
        super().__init__()
        self.stepSize, self.gamma = step_size, gamma

    def updateHyperParameter(self, m):
        e = m.state.get("epoch", 1)
        self.currentRate = -m.learningRate * self.gamma ** max(0, (e - self.excludeEpochs) // self.stepSize)


class EpochDecay(LearningRateSchedule):
    def __init__(self, decay_type: Callable[[int], float]):
        super().__init__()
        self.decayType = decay_type

    def updateHyperParameter(self, m):
        e = m.state.get("epoch", 1)
        self.currentRate = -m.learningRate * 0.1 ** self.decayType(e - self.excludeEpochs)


class Regime:
    def __init__(self, start_epoch, end_epoch, config):
        self.startEpoch, self.endEpoch, self.config = start_epoch, end_epoch, dict(config)


class EpochSchedule(LearningRateSchedule):
    def __init__(self, regimes):
        super().__init__()
        self.regimes = list(regimes)

    def updateHyperParameter(self, m):
        e = m.state.get("epoch", 1) - self.excludeEpochs
        for r in self.regimes:
            if r.startEpoch <= e <= r.endEpoch:
                for k, v in r.config.items():
                    if not hasattr(m, k):
                        raise ValueError(f"EpochSchedule: {k} is not a member of SGD")
                    setattr(m, k, v)
        self.currentRate = -m.learningRate


class Poly(LearningRateSchedule):
    def __init__(self, power, max_iteration):
        super().__init__()
        self.power, self.maxIteration = power, max_iteration

    def updateHyperParameter(self, m):
        n = self._bump(m)
        self.currentRate = 0.0 if n > self.maxIteration else -m.learningRate * (1.0 - n / self.maxIteration) ** self.power


class NaturalExp(LearningRateSchedule):
    def __init__(self, decay_step, gamma):
        super().__init__()
        self.decayStep, self.gamma = decay_step, gamma

    def updateHyperParameter(self, m):
        n = self._bump(m)
        p = (n - self.excludeIterations) // self.decayStep
        self.currentRate = -m.learningRate * math.exp(-self.gamma * p)


class Exponential(LearningRateSchedule):
    def __init__(self, decay_step, decay_rate, stair_case=False):
        super().__init__()
        self.decayStep, self.decayRate, self.stairCase = decay_step, decay_rate, stair_case

    def updateHyperParameter(self, m):
        n = self._bump(m)
        p = (n - self.excludeIterations) / self.decayStep
        if self.stairCase:
            p = math.floor(p)
        self.currentRate = -m.learningRate * self.decayRate ** p


class Plateau(LearningRateSchedule):
    def __init__(self, monitor, factor=0.1, patience=10, mode="min", epsilon=1e-4, cooldown=0, min_lr=0.0):
        super().__init__()
        if factor >= 1:
            raise ValueError("Plateau does not support a factor >= 1.0")
        if mode not in ("min", "max"):
            raise ValueError(f"Learning Rate Plateau Reducing mode {mode} is unknown, please use min | max")
        self.monitor, self.factor, self.patience, self.mode = monitor, factor, patience, mode
        self.epsilon, self.cooldown, self.minLr = epsilon, cooldown, min_lr
        self.best = float("inf") if mode == "min" else float("-inf")
        self.cooldownCounter = 0
        self.waitCounter = 0
        self.curEpoch = 1

    def _better(self, a, b):
        return a < b - self.epsilon if self.mode == "min" else a > b + self.epsilon

    def updateHyperParameter(self, m):
        e = m.state.get("epoch", 1) - self.excludeEpochs
        if e == 1 and self.currentRate == 0.0:
            self.currentRate = -m.learningRate
        if e == self.curEpoch:
            return
        self.curEpoch = e
        cur = m.state.get(self.monitor)
        if cur is None:
            raise ValueError(f"Learning Rate Plateau Reducing requires {self.monitor} available!")
        cur = float(cur)
        if self.cooldownCounter > 0:
            self.cooldownCounter -= 1
            self.waitCounter = 0
        if self._better(cur, self.best):
            self.best = cur
            self.waitCounter = 0
        elif self.cooldownCounter <= 0:
            if self.waitCounter >= self.patience:
                if abs(self.currentRate) > self.minLr + self.minLr * 1e-4:
                    self.currentRate = -max(abs(self.currentRate) * self.factor, self.minLr)
                    self.cooldownCounter = self.cooldown
                    self.waitCounter = 0
            self.waitCounter += 1


class Warmup(LearningRateSchedule):
    def __init__(self, delta):
        super().__init__()
        self.delta = delta

    def updateHyperParameter(self, m):
        n = self._bump(m)
        self.currentRate = -m.learningRate - self.delta * (n - self.excludeIterations)


class SequentialSchedule(LearningRateSchedule):
    def __init__(self, iteration_per_epoch):
        super().__init__()
        self.iterationPerEpoch = iteration_per_epoch
        self.schedules: List[LearningRateSchedule] = []
        self.cur = 0

    def add(self, schedule, max_iteration):
        schedule.excludeIterations = 0 if not self.schedules else self.schedules[-1].maxIterations
        schedule.maxIterations = schedule.excludeIterations + max_iteration
        schedule.excludeEpochs = schedule.excludeIterations // self.iterationPerEpoch
        self.schedules.append(schedule)
        return self

    def updateHyperParameter(self, m):
        n = m.state.get("evalCounter", 0)
        if n > self.schedules[self.cur].maxIterations:
            m.learningRate = -self.currentRate
            self.cur += 1
        self.schedules[self.cur].updateHyperParameter(m)
        self.currentRate = self.schedules[self.cur].currentRate


class EpochDecayWithWarmUp(LearningRateSchedule):
    def __init__(self, warm_up_iteration, warm_up_delta, decay_type):
        super().__init__()
        self.warmUpIteration, self.warmUpDelta, self.decayType = warm_up_iteration, warm_up_delta, decay_type

    def updateHyperParameter(self, m):
        n = self._bump(m)
        if n < self.warmUpIteration:
            self.currentRate = -m.learningRate - self.warmUpDelta * n
        else:
            max_lr = m.learningRate + self.warmUpDelta * self.warmUpIteration
            self.currentRate = -max_lr * 0.1 ** self.decayType(m.state.get("epoch", 1))


# ----------------------------------------------------------------------------------------- SGD
class SGD(OptimMethod):
    reads_bf16_grad = True  # apply_update takes the bf16 wire gradient shard (widened in the kernel)

    def prepare_graph(self) -> bool:
        # the fused kernel takes lr by value: replayable only while the schedule is constant
        if type(self.learningRateSchedule) is Default and self.learningRateDecay == 0:
            self._graph_mode = True
            return True
        return False

    def graph_state_restored(self, fresh):
        # the warmup created the momentum buffer: the next (replayed) update must apply the
        # first-iteration rule v = g — raised through the device flag the kernel reads
        if "dfdx" in fresh and isinstance(self.state.get("_dev_first"), torch.Tensor):
            self.state["_dev_first"].fill_(1.0)

    def __init__(self, learningrate=1e-3, learningrate_decay=0.0, weightdecay=0.0, momentum=0.0,
                 dampening=float("inf"), nesterov=False, leaningrate_schedule=None, learningrates=None,
                 weightdecays=None, bigdl_type="float"):
        super().__init__()
        self.learningRate = learningrate
        self.learningRateDecay = learningrate_decay
        self.weightDecay = weightdecay
        self.momentum = momentum
        self.dampening = dampening
        self.nesterov = nesterov
        self.learningRateSchedule = leaningrate_schedule or Default()
        self.learningRates = None if learningrates is None else torch.as_tensor(learningrates, dtype=torch.float32)
        self.weightDecays = None if weightdecays is None else torch.as_tensor(weightdecays, dtype=torch.float32)

    def updateHyperParameter(self):
        self.learningRateSchedule.updateHyperParameter(self)

    def getLearningRate(self) -> float:
        return self.learningRateSchedule.currentRate

    def getHyperParameter(self) -> str:
        return f"Current learning rate is {self.getLearningRate()}. "

    supports_slices = True

    def begin_iteration(self, x):
        self.updateHyperParameter()
        if self.dampening == float("inf") or self.dampening >= 1.7e308:
            self.dampening = self.momentum
        if self.nesterov and not (self.momentum > 0 and self.dampening == 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        t = self.state.get("dfdx")
        self._first = not isinstance(t, torch.Tensor) or t.shape != x.shape or t.device != x.device
        if self.momentum != 0:
            self._state_tensor("dfdx", x)

    #: per-element vectors in the coordinate space of the ``x`` the optimizer passes (arena slice or
    #: rank shard), installed by the optimizer: folded L2-regularizer decays, remapped user vectors
    _reg_decay = None
    _space_wds = None
    _space_lrs = None

    def _decays(self, dev, lo=None, hi=None):
        def sl(t):
            return t if (t is None or lo is None) else t[lo:hi]
        wds = self._space_wds if self._space_wds is not None else (
            self.weightDecays.to(dev) if self.weightDecays is not None else None)
        lrs = self._space_lrs if self._space_lrs is not None else (
            self.learningRates.to(dev) if self.learningRates is not None else None)
        wds, lrs, reg = sl(wds), sl(lrs), sl(self._reg_decay)
        # SGD.scala:79-93: a scalar weightDecay wins; the per-element weightDecays apply only when
        # the scalar is 0
        wd = self.weightDecay
        if reg is not None:
            key = (wd, lo, hi, None if wds is None else wds.data_ptr())
            cache = getattr(self, "_eff_cache", None)
            if cache is None or cache[0] != key:
                eff = reg + (wd if wd != 0 else (wds if wds is not None else 0.0))
                self._eff_cache = cache = (key, eff)
            return lrs, 1.0, cache[1]
        if wd != 0:
            return lrs, wd, None
        if wds is not None:
            return lrs, 1.0, wds
        return lrs, 0.0, None

    def apply_update(self, x, g, lo, hi, shadow=None):
        clr = self.learningRateSchedule.currentRate
        buf = self.state["dfdx"][lo:hi] if self.momentum != 0 else None
        lrs, wd, wds = self._decays(x.device, lo, hi)
        ops.sgd_step(x[lo:hi], g[lo:hi], buf, -clr, self.momentum, self.dampening, wd, self.nesterov, self._first,
                     self.grad_scale, shadow, lrs, wds)

    def optimize(self, feval, x):
        self.updateHyperParameter()
        if self.dampening == float("inf") or self.dampening >= 1.7e308:
            self.dampening = self.momentum
        if self.nesterov and not (self.momentum > 0 and self.dampening == 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        fx, dfdx = feval(x)
        clr = self.learningRateSchedule.currentRate  # negative
        first = "dfdx" not in self.state or not isinstance(self.state.get("dfdx"), torch.Tensor) or \
            self.state["dfdx"].shape != x.shape
        buf = self._state_tensor("dfdx", x) if self.momentum != 0 else None
        lrs, wd, wds = self._decays(x.device)
        fdev = None
        if getattr(self, "_graph_mode", False) and x.is_cuda and self.momentum != 0:
            # replay-safe first-iteration rule: a device flag read by the kernel, cleared after it
            fdev = self.state.get("_dev_first")
            if not isinstance(fdev, torch.Tensor) or fdev.device != x.device:
                fdev = self.state["_dev_first"] = torch.zeros(1, device=x.device)
        ops.sgd_step(x, dfdx, buf, -clr, self.momentum, self.dampening, wd, self.nesterov, first,
                     self.grad_scale, self.shadow, lrs, wds, first_dev=fdev)
        if fdev is not None:
            fdev.zero_()
        return x, [fx]

    def __getstate__(self):
        d = dict(self.__dict__)
        for k in ("_reg_decay", "_space_wds", "_space_lrs", "_eff_cache"):
            d.pop(k, None)
        return d


# ----------------------------------------------------------------------------------------- Adam family
class Adam(OptimMethod):
    def __init__(self, learningrate=1e-3, learningrate_decay=0.0, beta1=0.9, beta2=0.999, epsilon=1e-8,
                 bigdl_type="float"):
        super().__init__()
        self.learningRate, self.learningRateDecay = learningrate, learningrate_decay
        self.beta1, self.beta2, self.epsilon = beta1, beta2, epsilon

    def getLearningRate(self):
        n = self.state.get("evalCounter", 0)
        return self.learningRate / (1 + n * self.learningRateDecay)

    supports_slices = True

    def begin_iteration(self, x):
        n = self.state.get("evalCounter", 0)
        self._clr = self.learningRate / (1 + n * self.learningRateDecay)
        self._t = n + 1
        self._state_tensor("s", x)
        self._state_tensor("r", x)
        self.state["evalCounter"] = self._t

    def apply_update(self, x, g, lo, hi, shadow=None):
        ops.adam_step(x[lo:hi], g[lo:hi], self.state["s"][lo:hi], self.state["r"][lo:hi], self._clr, self.beta1,
                      self.beta2, self.epsilon, self._t, 0.0, self.grad_scale, shadow)

    def optimize(self, feval, x):
        fx, g = feval(x)
        n = self.state.get("evalCounter", 0)
        clr = self.learningRate / (1 + n * self.learningRateDecay)
        t = n + 1
        m = self._state_tensor("s", x)
        v = self._state_tensor("r", x)
        if getattr(self, "_graph_mode", False) and x.is_cuda:
            # replay-safe: iteration count on the device, decayed rate / bias corrections in the kernel
            nt = self.state.get("_dev_n")
            if not isinstance(nt, torch.Tensor) or nt.device != x.device:
                nt = torch.full((1,), float(n), device=x.device)
                self.state["_dev_n"] = nt
            r = ops.native_ops.adam_step_dev(x, g, m, v, nt, self.learningRate, self.learningRateDecay, self.beta1,
                                             self.beta2, self.epsilon, 0.0, self.grad_scale, self.shadow)
            if r is NotImplemented:
                raise NotImplementedError("Adam graph mode needs the native fused kernel")
            nt.add_(1)
        else:
            ops.adam_step(x, g, m, v, clr, self.beta1, self.beta2, self.epsilon, t, 0.0, self.grad_scale,
                          self.shadow)
        self.state["evalCounter"] = t
        return x, [fx]

    def prepare_graph(self) -> bool:
        if not ops.native_has("adam_step_dev"):
            return False
        self._graph_mode = True
        return True


class ParallelAdam(Adam):
    """The reference splits Adam over host threads (``ParallelAdam.scala:38``); on the GPU one fused
    kernel already covers the whole buffer, so this is Adam with the same hyper-parameters."""

    def __init__(self, learningrate=1e-3, learningrate_decay=0.0, beta1=0.9, beta2=0.999, epsilon=1e-8,
                 parallel_num=-1, bigdl_type="float"):
        super().__init__(learningrate, learningrate_decay, beta1, beta2, epsilon)


class _Elementwise(OptimMethod):
    """An update that is elementwise in (x, g, state): ``begin_iteration`` advances the per-iteration
    scalars and sizes the state like ``x``; ``apply_update`` runs the update on ``[lo, hi)`` — so the
    DistriOptimizer can run it on this rank's shard only, bucket by bucket (the reference runs every
    OptimMethod on its partition ``[paramLocalStart, +paramLocalLen)``,
    ``DL/optim/DistriOptimizer.scala:378-386``).  ``optimize`` (local) is the same two calls over
    the whole buffer, so the sharded and local updates are one implementation."""

    supports_slices = True

    def _begin(self, x):  # per-iteration scalars + state tensors shaped like x
        raise NotImplementedError

    def _update(self, x, g, sl, shadow):  # x, g: the [lo, hi) slices; sl: slice object for state
        raise NotImplementedError

    def begin_iteration(self, x):
        self._begin(x)
        self.state["evalCounter"] = self.state.get("evalCounter", 0) + 1

    def apply_update(self, x, g, lo, hi, shadow=None):
        self._update(x[lo:hi], g[lo:hi], slice(lo, hi), shadow)

    def optimize(self, feval, x):
        fx, g = feval(x)
        self.begin_iteration(x)
        self._update(x, g, slice(0, x.numel()), self.shadow)
        return x, [fx]


def _write_shadow(shadow, x):
    if shadow is not None:
        if ops.cast_copy(shadow, x) is NotImplemented:
            shadow.copy_(x)


class Adamax(_Elementwise):
    def __init__(self, learningrate=0.002, beta1=0.9, beta2=0.999, epsilon=1e-38, bigdl_type="float"):
        super().__init__()
        self.learningRate, self.beta1, self.beta2, self.epsilon = learningrate, beta1, beta2, epsilon

    def _begin(self, x):
        self._t = self.state.get("evalCounter", 0) + 1
        self._state_tensor("m", x)
        self._state_tensor("u", x)

    def _update(self, x, g, sl, shadow):
        g = g * self.grad_scale
        m, u = self.state["m"][sl], self.state["u"][sl]
        m.mul_(self.beta1).add_(g, alpha=1 - self.beta1)
        torch.maximum(u * self.beta2, g.abs() + self.epsilon, out=u)
        x.addcdiv_(m, u, value=-self.learningRate / (1 - self.beta1 ** self._t))
        _write_shadow(shadow, x)


class Adagrad(_Elementwise):
    def __init__(self, learningrate=1e-3, learningrate_decay=0.0, weightdecay=0.0, bigdl_type="float"):
        super().__init__()
        self.learningRate, self.learningRateDecay, self.weightDecay = learningrate, learningrate_decay, weightdecay

    def _begin(self, x):
        self._n = self.state.get("evalCounter", 0)
        self._state_tensor("paramVariance", x)

    reads_bf16_grad = True  # apply_update takes the bf16 wire gradient shard (widened in the kernel)

    def _update(self, x, g, sl, shadow):
        n = self._n
        s = self.state["paramVariance"][sl]
        if x.is_cuda and ops.native_has("adagrad_step"):
            # one fused pass (k_adagrad) over w, g, the accumulator and the bf16 shadow
            r = ops.native_ops.adagrad_step(x, g, s, self.learningRate, self.learningRateDecay, n, self.weightDecay,
                                            self.grad_scale, shadow)
            if r is not NotImplemented:
                return
        g = g.float() * self.grad_scale
        if self.weightDecay != 0:
            g = g + self.weightDecay * x
        s.addcmul_(g, g)
        clr = self.learningRate / (1 + n * self.learningRateDecay)
        x.addcdiv_(g, s.sqrt().add_(1e-10), value=-clr)
        _write_shadow(shadow, x)

    def optimize(self, feval, x):
        if not getattr(self, "_graph_mode", False):
            return super().optimize(feval, x)
        fx, g = feval(x)
        n = self.state.get("evalCounter", 0)
        s = self._state_tensor("paramVariance", x)
        # replay-safe: the iteration counter lives on the device and the decayed rate is a tensor
        nt = self.state.get("_dev_n")
        if not isinstance(nt, torch.Tensor) or nt.device != x.device:
            nt = torch.full((1,), float(n), device=x.device)
            self.state["_dev_n"] = nt
        if x.is_cuda and ops.native_has("adagrad_step"):
            r = ops.native_ops.adagrad_step(x, g, s, self.learningRate, self.learningRateDecay, n, self.weightDecay,
                                            self.grad_scale, self.shadow, dev_n=nt)
            if r is not NotImplemented:
                nt.add_(1)
                self.state["evalCounter"] = n + 1
                return x, [fx]
        g = g * self.grad_scale
        if self.weightDecay != 0:
            g = g + self.weightDecay * x
        s.addcmul_(g, g)
        clr_t = (1 + nt * self.learningRateDecay).reciprocal_().mul_(self.learningRate)
        x.sub_(g / s.sqrt().add_(1e-10) * clr_t)
        nt.add_(1)
        self.state["evalCounter"] = n + 1
        _sync_shadow(self, x)
        return x, [fx]

    def prepare_graph(self) -> bool:
        self._graph_mode = True
        return True


class Adadelta(_Elementwise):
    def __init__(self, decayrate=0.9, epsilon=1e-10, bigdl_type="float"):
        super().__init__()
        self.decayRate, self.epsilon = decayrate, epsilon

    def _begin(self, x):
        self._state_tensor("paramVariance", x)
        self._state_tensor("delta", x)

    def _update(self, x, g, sl, shadow):
        g = g * self.grad_scale
        v, d = self.state["paramVariance"][sl], self.state["delta"][sl]
        v.mul_(self.decayRate).addcmul_(g, g, value=1 - self.decayRate)
        upd = (d + self.epsilon).sqrt() / (v + self.epsilon).sqrt() * g
        d.mul_(self.decayRate).addcmul_(upd, upd, value=1 - self.decayRate)
        x.sub_(upd)
        _write_shadow(shadow, x)


class RMSprop(_Elementwise):
    def __init__(self, learningrate=1e-2, learningrate_decay=0.0, decayrate=0.99, epsilon=1e-8, bigdl_type="float"):
        super().__init__()
        self.learningRate, self.learningRateDecay = learningrate, learningrate_decay
        self.decayRate, self.epsilon = decayrate, epsilon

    def _begin(self, x):
        n = self.state.get("evalCounter", 0)
        self._clr = self.learningRate / (1 + n * self.learningRateDecay)
        self._state_tensor("sumSquare", x)

    def _update(self, x, g, sl, shadow):
        g = g * self.grad_scale
        s = self.state["sumSquare"][sl]
        s.mul_(self.decayRate).addcmul_(g, g, value=1 - self.decayRate)
        x.addcdiv_(g, s.sqrt().add_(self.epsilon), value=-self._clr)
        _write_shadow(shadow, x)


class Ftrl(_Elementwise):
    """FTRL-proximal (``Ftrl.scala:39``)."""

    def __init__(self, learningrate=1e-3, learningrate_power=-0.5, initial_accumulator_value=0.1,
                 l1_regularization_strength=0.0, l2_regularization_strength=0.0,
                 l2_shrinkage_regularization_strength=0.0, bigdl_type="float"):
        super().__init__()
        self.learningRate, self.learningRatePower = learningrate, learningrate_power
        self.initialAccumulatorValue = initial_accumulator_value
        self.l1, self.l2, self.l2Shrinkage = (l1_regularization_strength, l2_regularization_strength,
                                              l2_shrinkage_regularization_strength)

    def _begin(self, x):
        acc = self.state.get("accum")
        if not isinstance(acc, torch.Tensor) or acc.shape != x.shape or acc.device != x.device:
            self.state["accum"] = torch.full_like(x, self.initialAccumulatorValue, dtype=torch.float32)
        self._state_tensor("linear", x)

    def _update(self, x, g, sl, shadow):
        g = g * self.grad_scale
        acc, lin = self.state["accum"][sl], self.state["linear"][sl]
        gs = g + 2 * self.l2Shrinkage * x if self.l2Shrinkage > 0 else g
        new_acc = acc + g * g
        p = -self.learningRatePower
        sigma = (new_acc.pow(p) - acc.pow(p)) / self.learningRate
        lin.add_(gs - sigma * x)
        quad = new_acc.pow(p) / self.learningRate + 2 * self.l2
        l1r = torch.clamp(lin.abs() - self.l1, min=0) * torch.sign(lin)
        x.copy_(torch.where(lin.abs() > self.l1, -l1r / quad, torch.zeros_like(x)))
        acc.copy_(new_acc)
        _write_shadow(shadow, x)


class LBFGS(OptimMethod):
    """Limited-memory BFGS with optional line search (``LBFGS.scala:48``); host-driven loop over
    device vectors (each iteration re-evaluates ``feval``)."""

    def __init__(self, max_iter=20, max_eval=float("inf"), tolfun=1e-5, tolx=1e-9, ncorrection=100,
                 learningrate=1.0, verbose=False, linesearch=None, linesearch_options=None, bigdl_type="float"):
        super().__init__()
        self.maxIter, self.maxEval = max_iter, (max_eval if max_eval != float("inf") else max_iter * 1.25)
        self.tolFun, self.tolX, self.nCorrection = tolfun, tolx, ncorrection
        self.learningRate, self.verbose, self.lineSearch = learningrate, verbose, linesearch

    def optimize(self, feval, x):
        fx, g = feval(x)
        f_hist = [float(fx)]
        n_eval = 1
        if float(g.abs().sum()) <= self.tolFun:
            return x, f_hist
        old_dirs, old_stps = [], []
        d = -g.clone()
        t = min(1.0, 1.0 / float(g.abs().sum())) * self.learningRate
        ro = []
        Hdiag = 1.0
        g_prev = g.clone()
        for it in range(int(self.maxIter)):
            if it > 0:
                y = g - g_prev
                s = d * t
                ys = float((y * s).sum())
                if ys > 1e-10:
                    if len(old_dirs) == self.nCorrection:
                        old_dirs.pop(0)
                        old_stps.pop(0)
                        ro.pop(0)
                    old_dirs.append(s)
                    old_stps.append(y)
                    ro.append(1.0 / ys)
                    Hdiag = ys / float((y * y).sum())
                q = -g.clone()
                al = [0.0] * len(old_dirs)
                for i in range(len(old_dirs) - 1, -1, -1):
                    al[i] = float((old_dirs[i] * q).sum()) * ro[i]
                    q.add_(old_stps[i], alpha=-al[i])
                d = q * Hdiag
                for i in range(len(old_dirs)):
                    be = float((old_stps[i] * d).sum()) * ro[i]
                    d.add_(old_dirs[i], alpha=al[i] - be)
                t = self.learningRate
            g_prev = g.clone()
            gtd = float((g * d).sum())
            if gtd > -self.tolX:
                break
            if self.lineSearch is not None:
                # strong-Wolfe search along d (LineSearch.scala); it evaluates feval itself
                f_new, g_new, x_new, t, ls_evals = self.lineSearch.apply(
                    lambda xx: feval(xx), x, t, d, float(fx), g, gtd)
                x.copy_(x_new)
                fx, g = f_new, g_new
                n_eval += ls_evals
                f_hist.append(float(fx))
            else:
                x.add_(d, alpha=t)
                if it != self.maxIter - 1:
                    fx, g = feval(x)
                    n_eval += 1
                    f_hist.append(float(fx))
            if n_eval >= self.maxEval or float((d * t).abs().sum()) <= self.tolX:
                break
            if len(f_hist) > 1 and abs(f_hist[-1] - f_hist[-2]) < self.tolFun:
                break
        self.state["evalCounter"] = self.state.get("evalCounter", 0) + 1
        _sync_shadow(self, x)
        return x, f_hist


class LarsSGD(SGD):
    """Layer-wise adaptive rate scaling (``LarsSGD.scala:47``): per-layer trust ratio
    ‖w‖ / (‖g‖ + wd·‖w‖) × trust, computed per parameter slice.  The ratio needs whole-layer norms, so
    the DistriOptimizer runs it replicated (a rank's shard can split a layer)."""

    supports_slices = False

    def __init__(self, lr_schedule=None, learningrate=1e-3, learningrate_decay=0.01, weightdecay=5e-4,
                 momentum=0.5, trust=1.0, bigdl_type="float"):
        super().__init__(learningrate, learningrate_decay, weightdecay, momentum, leaningrate_schedule=lr_schedule)
        self.trust = trust
        self.slices = None  # list of (offset, length) set by the optimizer driver

    def optimize(self, feval, x):
        self.updateHyperParameter()
        fx, g = feval(x)
        g = g * self.grad_scale
        clr = -self.learningRateSchedule.currentRate
        buf = self._state_tensor("dfdx", x)
        slices = self.slices or [(0, x.numel())]
        for off, n in slices:
            w, gg, b = x[off:off + n], g[off:off + n], buf[off:off + n]
            wn = float(w.norm())
            gn = float(gg.norm())
            ratio = self.trust * wn / (gn + self.weightDecay * wn + 1e-12) if wn > 0 and gn > 0 else 1.0
            upd = (gg + self.weightDecay * w) * (ratio * clr)
            b.mul_(self.momentum).add_(upd)
            w.sub_(b)
        _sync_shadow(self, x)
        return x, [fx]


def _sync_shadow(method, x):
    if method.shadow is not None:
        ops.cast_copy(method.shadow, x)
