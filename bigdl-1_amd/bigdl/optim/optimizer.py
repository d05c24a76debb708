"""Training drivers: ``Optimizer`` builder, ``LocalOptimizer``.

Reference: ``DL/optim/Optimizer.scala:47-699`` (builder setters 93-470; ``apply`` 602-681),
``AbstractOptimizer.scala:30-286`` (summary 47-91, validate 93-191, checkpoint 205-231),
``LocalOptimizer.scala:45-295`` and the retry loop of ``DistriOptimizer.scala:881-963``.

Loop per iteration (one device, or one rank of :class:`bigdl.parallel.DistriOptimizer`)::

    zero grads (one memset of the flat grad arena)
    forward → criterion forward/backward → backward       (explicit Module contract)
    gradient hooks: bucketed reduce-scatter (distributed only, overlapped with backward)
    clipping (constant / global L2 norm, X9)
    OptimMethod update(s) on the flat arena or this rank's shard (fused HIP kernel, K22)
    all-gather of updated weights (distributed only; waited for lazily by the next forward)

The hot loop never synchronises the host with the device: the loss stays on the GPU and is read
back one iteration late through a pinned buffer, so the host enqueues step i+1 while step i runs.
The canonical log line (``DistriOptimizer.scala:411-416``) is kept.
"""
from __future__ import annotations

import glob
import os
import time
from typing import Dict, List, Optional

import torch

from ..dataset.core import (AbstractDataSet, DataSet, DevicePrefetcher, MiniBatch, SampleToMiniBatch,
                            TransformedDataSet)
from ..nn.abstractnn import AbstractModule, AbstractCriterion, to_torch
from ..utils import config
from ..utils.engine import Engine
from ..utils.logger import get_logger, iteration_line
from ..utils.table import Table
from .metrics import Metrics
from .optim_method import OptimMethod, SGD
from .trigger import Trigger, MaxEpoch
from .validation import ValidationMethod, allreduce_results

log = get_logger("bigdl.optim")


class _LazyScalar:
    """Device scalar read back asynchronously (pinned host copy + event)."""

    def __init__(self, t: torch.Tensor):
        if isinstance(t, torch.Tensor) and t.is_cuda:
            self.host = torch.empty((), dtype=torch.float32, pin_memory=True)
            self.host.copy_(t.detach().float(), non_blocking=True)
            self.ev = torch.cuda.Event()
            self.ev.record()
            self.v = None
        else:
            self.ev = None
            self.v = float(t)

    def ready(self) -> bool:
        return self.ev is None or self.ev.query()

    def value(self) -> float:
        if self.v is None:
            self.ev.synchronize()
            self.v = float(self.host)
        return self.v


class BaseOptimizer:
    """Builder + loop shared by the local and distributed drivers."""

    def __init__(self, model: AbstractModule, dataset, criterion: AbstractCriterion, batch_size: int = 32):
        self.model = model
        self.criterion = criterion
        self.batch_size = batch_size
        self.dataset = self._as_dataset(dataset, batch_size)
        self.optim_methods: Dict[str, OptimMethod] = {model.get_name(): SGD()}
        self.end_when: Trigger = MaxEpoch(1)
        self.state = {"epoch": 1, "neval": 1, "recordsProcessedThisEpoch": 0, "Loss": float("nan"),
                      "score": 0.0}
        self.validation_trigger = None
        self.validation_set = None
        self.validation_methods: List[ValidationMethod] = []
        self.checkpoint_trigger = None
        self.checkpoint_path = None
        self.is_overwrite = False
        self.train_summary = None
        self.validation_summary = None
        self.constant_clip = None
        self.l2_clip = None
        self.drop_percentage = 0.0
        self.max_drop_percentage = 0.0
        self.reserve_optim_state = False
        self.metrics = Metrics()
        self.log_interval = 1
        self.device = Engine.device()
        self.compute_dtype = Engine.compute_dtype()
        self._pending_loss: Optional[_LazyScalar] = None
        self._skipped = False

    # ------------------------------------------------------------------------------ data helpers
    @staticmethod
    def _as_dataset(ds, batch_size):
        if ds is None:
            return None
        if isinstance(ds, AbstractDataSet):
            return ds
        if isinstance(ds, (list, tuple)):
            items = list(ds)
            if items and isinstance(items[0], MiniBatch):
                return DataSet.array(items)
            return DataSet.array(items).transform(SampleToMiniBatch(batch_size))
        if callable(getattr(ds, "data", None)) and callable(getattr(ds, "size", None)):
            return ds  # a batch source with the data-set protocol (runtime.NativeBatchLoader)
        raise TypeError(f"unsupported training data {type(ds)}")

    # ------------------------------------------------------------------------------ builder setters
    def setValidation(self, trigger, dataset, vmethods, batch_size=None):
        self.validation_trigger = trigger
        self.validation_set = self._as_dataset(dataset, batch_size or self.batch_size)
        self.validation_methods = list(vmethods)
        return self

    def set_validation(self, batch_size, val_rdd, trigger, val_method=None):
        """pyspark signature: ``set_validation(batch_size, val_rdd, trigger, val_method)``."""
        from .validation import Top1Accuracy
        return self.setValidation(trigger, val_rdd, val_method or [Top1Accuracy()], batch_size)

    def setCheckpoint(self, path, trigger, is_overwrite=False):
        stamp = time.strftime("%Y%m%d_%H%M%S")
        self.checkpoint_path = os.path.join(path, stamp) if not os.environ.get("BIGDL_CKPT_FLAT") else path
        self.checkpoint_trigger = trigger
        self.is_overwrite = is_overwrite
        if Engine.rank() == 0:
            os.makedirs(self.checkpoint_path, exist_ok=True)
        return self

    def set_checkpoint(self, checkpoint_trigger, checkpoint_path, isOverWrite=True):
        return self.setCheckpoint(checkpoint_path, checkpoint_trigger, isOverWrite)

    def overWriteCheckpoint(self):
        self.is_overwrite = True
        return self

    def setTrainSummary(self, summary):
        self.train_summary = summary
        return self

    set_train_summary = setTrainSummary

    def setValidationSummary(self, summary):
        self.validation_summary = summary
        return self

    set_val_summary = setValidationSummary

    def setModel(self, model):
        self.model = model
        return self

    def setTrainData(self, dataset, batch_size=None):
        self.dataset = self._as_dataset(dataset, batch_size or self.batch_size)
        return self

    set_traindata = setTrainData

    def setCriterion(self, criterion):
        self.criterion = criterion
        return self

    set_criterion = setCriterion

    def setState(self, state):
        self.state.update(dict(state.items()) if isinstance(state, Table) else dict(state))
        return self

    def setOptimMethod(self, method: OptimMethod):
        self.optim_methods = {self.model.get_name(): method}
        return self

    def setOptimMethods(self, methods: Dict[str, OptimMethod]):
        self.optim_methods = dict(methods)
        return self

    def setModelAndOptimMethods(self, model, methods):
        self.model = model
        return self.setOptimMethods(methods)

    def setEndWhen(self, trigger: Trigger):
        self.end_when = trigger
        return self

    set_end_when = setEndWhen

    def set_gradclip_const(self, min_value, max_value):
        return self.setConstantGradientClipping(min_value, max_value)

    def set_gradclip_l2norm(self, clip_norm):
        return self.setGradientClippingByl2Norm(clip_norm)

    def disable_gradclip(self):
        return self.disableGradientClipping()

    def set_model(self, model):
        return self.setModel(model)

    def prepare_input(self):
        return self.prepareInput()

    def setDropModuleProperty(self, drop_percentage, max_drop_percentage, batchsize=100, warmup_iteration=200):
        """Straggler handling (P5, ``DistriOptimizer.scala:240-280,343-345,421-449,510-515``).  With
        ``drop_percentage > 0`` the DistriOptimizer times every rank's forward + backward; every
        ``batchsize`` iterations after ``warmup_iteration`` the ranks all-gather those times and the
        threshold becomes ``Util.kthLargest`` at k = drop_percentage · batchsize · world minus the
        ranks already dropped in the window.  A rank over the threshold contributes a zero gradient
        and a finished-count of 0; the update averages over the finished ranks, and an iteration
        where fewer than ``(1 − max_drop_percentage)·world`` ranks finished is discarded (see
        :mod:`bigdl.parallel.distri_optimizer`)."""
        self.drop_percentage = float(drop_percentage)
        self.max_drop_percentage = float(max_drop_percentage)
        self._straggler_window = int(batchsize)
        self._straggler_warmup = int(warmup_iteration)
        return self

    def disableGradientClipping(self):
        self.constant_clip = None
        self.l2_clip = None
        return self

    disable_gradient_clipping = disableGradientClipping

    def setConstantGradientClipping(self, min_value, max_value):
        self.constant_clip = (min_value, max_value)
        return self

    set_gradclip_const = setConstantGradientClipping

    def setGradientClippingByl2Norm(self, clip_norm):
        self.l2_clip = clip_norm
        return self

    set_gradclip_l2norm = setGradientClippingByl2Norm

    def reserveOptim(self, reserve: bool):
        self.reserve_optim_state = reserve
        return self

    def prepareInput(self):
        return self

    # ------------------------------------------------------------------------------ setup
    def _make_tracer(self):
        from ..utils.tracing import StepTracer
        self.tracer = StepTracer(self.metrics, Engine.rank(), Engine.world_size())
        if self.drop_percentage > 0:
            # the straggler monitor needs device-side step times
            self.tracer.window = getattr(self, "_straggler_window", self.tracer.window)
            self.tracer.device = torch.cuda.is_available() and self.device.type == "cuda"
            self.tracer.host_timers = True
            self.tracer.enabled = True
        return self.tracer

    def _setup_model(self):
        from ..nn.fusion import fuse
        self._make_tracer()
        m = self.model
        m.to(self.device)
        m.training()
        fuse(m)
        from ..nn.fusion import mark_input_no_grad
        mark_input_no_grad(m)
        flat_w, flat_g = m.getParameters()
        self.flat = m.flat_parameters()
        if self.flat is not None and self.device.type == "cuda" and self.compute_dtype != torch.float32:
            self.flat.enable_shadow(self.compute_dtype)
        self._method_slices = self._compute_method_slices()
        for name, meth in self.optim_methods.items():
            for k in ("epoch", "neval"):
                meth.state.setdefault(k, self.state[k])
        reg = self._fold_regularizers()
        if reg is not None:
            for name, meth in self.optim_methods.items():
                off, n = self._method_slices[name]
                meth._reg_decay = reg[off:off + n]

    def _fold_regularizers(self):
        """Fold every pure-L2 ``wRegularizer``/``bRegularizer`` (``Regularizer.scala``: g += λ·w
        inside accGradParameters) into a per-element decay vector over the arena, applied by the
        fused SGD kernel — one elementwise pass per layer per step less.  Only when every
        OptimMethod is SGD (the kernel that takes per-element decays).  Returns the vector or None."""
        from .optim_method import SGD
        from .regularizer import L1L2Regularizer
        for mod in self.model.flattened_modules():  # undo a previous optimizer's folding
            for r in (mod.wRegularizer, mod.bRegularizer):
                if isinstance(r, L1L2Regularizer):
                    r._folded = False
        if self.flat is None or not config.get_property("bigdl.optim.foldRegularizers"):
            return None
        if not all(type(m) is SGD for m in self.optim_methods.values()):
            return None
        reg_full = None
        for (m, wname, gname, off, n, shape) in self.flat.slices:
            reg = m.wRegularizer if wname == "weight" else (m.bRegularizer if wname == "bias" else None)
            if not (isinstance(reg, L1L2Regularizer) and reg.l1 == 0 and reg.isRegualrized):
                continue
            if reg_full is None:
                reg_full = torch.zeros(self.flat.numel, dtype=torch.float32, device=self.flat.weight.device)
            scale = m.scale_b if wname == "bias" else m.scale_w
            reg_full[off:off + n] = reg.l2 * scale
            reg._folded = True
        return reg_full

    def _compute_method_slices(self):
        """Map each OptimMethod to the (offset, length) of its sub-module's parameters in the
        flat arena (``Optimizer.scala:492-522`` checkSubModules)."""
        if self.flat is None:
            return {}
        slices = {}
        root = self.model.get_name()
        for name in self.optim_methods:
            if name == root:
                slices[name] = (0, self.flat.numel)
                continue
            sub = [m for m in self.model.flattened_modules() if m.get_name() == name]
            if not sub:
                raise ValueError(f"optimMethod names a sub-module '{name}' that does not exist")
            ents = sub[0]._param_entries()
            offs = [o for (m, w, g, o, n, s) in self.flat.slices for (mm, ww, gg) in ents if m is mm and w == ww]
            lens = [n for (m, w, g, o, n, s) in self.flat.slices for (mm, ww, gg) in ents if m is mm and w == ww]
            lo = min(offs)
            hi = max(o + n for o, n in zip(offs, lens))
            slices[name] = (lo, hi - lo)
        covered = sum(l for _, l in slices.values())
        if covered != self.flat.numel:
            raise ValueError("optimMethods must cover every trainable parameter exactly once")
        return slices

    # ------------------------------------------------------------------------------ per-iteration hooks
    def _before_backward(self):
        pass

    def _sync_and_update(self, loss_t: torch.Tensor, batch_size: int):
        """Gradient aggregation + clipping + optimizer update (local: no aggregation)."""
        from ..ops import native_ops as NO
        NO.join_wgrad()  # weight gradients computed on the side stream
        self._clip(self.flat.grad, self.flat.grad)
        with self.tracer.phase("compute weight"):
            for name, meth in self.optim_methods.items():
                off, n = self._method_slices[name]
                w = self.flat.weight[off:off + n]
                g = self.flat.grad[off:off + n]
                meth.shadow = self.flat.shadow[off:off + n] if self.flat.shadow is not None else None
                meth.optimize(lambda _x, g=g: (loss_t, g), w)
        if self.flat.shadow is not None:
            self.flat.mark_shadow_fresh()

    def parameter_processors(self):
        """The gradient processors of this optimizer, in application order
        (``Optimizer.scala:76`` ``parameterProcessors``): constant clipping, then L2-norm clipping."""
        from ..parameters import ConstantClippingProcessor, L2NormClippingProcessor
        procs = []
        if self.constant_clip is not None:
            procs.append(ConstantClippingProcessor(*self.constant_clip))
        if self.l2_clip is not None:
            procs.append(L2NormClippingProcessor(self.l2_clip))
        return procs

    def _clip(self, grad: torch.Tensor, local_shard: torch.Tensor):
        from ..parameters import run_processors
        # ``grad`` is this rank's gradient shard (the whole arena on one process); the norm of a
        # sharded gradient is completed by ``_global_sum`` (one all-reduce per processor)
        run_processors(self.parameter_processors(), None, grad, self._global_sum)

    def _global_sum(self, t: torch.Tensor) -> torch.Tensor:
        return t

    def _reduce_scalar(self, t: torch.Tensor) -> torch.Tensor:
        return t

    # ------------------------------------------------------------------------------ main loop
    def optimize(self) -> AbstractModule:
        retry = int(config.get_property("bigdl.failure.retryTimes"))
        interval = float(config.get_property("bigdl.failure.retryTimeInterval"))
        failures: List[float] = []
        self._setup_model()
        self._maybe_resume()
        while True:
            try:
                self._train_loop()
                break
            except (ValueError, KeyboardInterrupt):
                raise
            except Exception as e:  # noqa: BLE001 - retry loop (DistriOptimizer.scala:881-963)
                if Engine.world_size() > 1:
                    # after a collective failure / watchdog abort the RCCL communicator is dead: a
                    # distributed rank must not retry in-process (a restore would broadcast over the
                    # broken group).  Exit non-zero; ``python -m bigdl.launch --max-restarts N``
                    # relaunches every rank and they resume from the latest checkpoint
                    # (``_maybe_resume``), the reference's retry-from-checkpoint semantics.
                    log.error(f"rank {Engine.rank()} failed ({e!r}); exiting so the launcher restarts all ranks")
                    raise
                now = time.time()
                failures = [t for t in failures if now - t < retry * interval] + [now]
                if self.checkpoint_path is None or len(failures) > retry:
                    raise
                log.warning(f"training failed ({e!r}); retry {len(failures)}/{retry} from the latest checkpoint")
                self._restore_latest()
        self._finish()
        return self.model

    def _global_epoch_size(self, local_epoch_size: int) -> int:
        """Records per epoch across all ranks: a rank-sharded dataset reports the local shard."""
        if hasattr(self.dataset, "local_size") and Engine.world_size() > 1:
            return local_epoch_size * Engine.world_size()
        return local_epoch_size

    def _finish(self):
        from ..serialization.checkpoint import wait_checkpoints
        wait_checkpoints()
        if self.device.type == "cuda":
            torch.cuda.synchronize()
        if getattr(self, "tracer", None) is not None:
            self.tracer.flush()
        self.metrics.resolve()

    def _batches(self):
        it = self.dataset.data(train=True)
        if self.device.type == "cuda":
            return DevicePrefetcher(it, self.device)
        return it

    def _epoch_size(self) -> int:
        """Records per epoch on this rank.  A data set of ready-made MiniBatches counts their
        records (the reference sums ``batch.size()`` over one pass, LocalOptimizer.scala:93-96)."""
        ds = self.dataset
        buf = getattr(ds, "buffer", None)
        if buf and isinstance(buf[0], MiniBatch) and type(ds).__name__ == "LocalArrayDataSet":
            return max(1, sum(b.size() for b in buf))
        n = getattr(ds, "local_size", None)
        n = n() if callable(n) else ds.size()
        return max(1, n)

    def _train_loop(self):
        m, crit = self.model, self.criterion
        epoch_size = self._epoch_size()
        batches = self._batches()
        wall0 = time.perf_counter()
        for meth in self.optim_methods.values():
            meth.state["epoch"] = self.state["epoch"]
            meth.state["neval"] = self.state["neval"]
        while not self.end_when(self.state):
            t0 = time.perf_counter()
            batch = next(batches)
            bs = batch.size()
            it = self.state["neval"]
            loss_t = self._step(batch)
            if self._skipped:
                # straggler drop discarded this iteration's gradients: it does not count
                # (DistriOptimizer.scala:510-515 — neval / records do not advance)
                self._skipped = False
                continue
            # bookkeeping (no device sync: the loss is read one iteration late)
            if not (isinstance(loss_t, torch.Tensor) and loss_t.is_cuda) or self._needs_loss():
                # host tensor, or a consumer (summary / MinLoss trigger) needs this iteration's value
                self._pending_loss = None
                self.state["Loss"] = float(loss_t)
            else:
                prev = self._pending_loss
                self._pending_loss = _LazyScalar(loss_t)
                if prev is not None:
                    self.state["Loss"] = prev.value() if prev.ready() else self.state["Loss"]
            global_bs = bs * Engine.world_size()
            self.state["recordsProcessedThisEpoch"] += global_bs
            dt = time.perf_counter() - t0
            self.metrics.add("computing time", dt)
            if it % self.log_interval == 0 and Engine.rank() == 0:
                log.info(iteration_line(self.state["epoch"], self.state["recordsProcessedThisEpoch"],
                                        self._global_epoch_size(epoch_size), it, time.perf_counter() - wall0,
                                        global_bs, dt, self.state["Loss"], self._hyper_str()))
            self.state["neval"] = it + 1
            if self.state["recordsProcessedThisEpoch"] >= self._global_epoch_size(epoch_size):
                self.state["epoch"] += 1
                self.state["recordsProcessedThisEpoch"] = 0
                self.dataset.shuffle()
            for meth in self.optim_methods.values():
                meth.state["epoch"] = self.state["epoch"]
                meth.state["neval"] = self.state["neval"]
            self._observe_straggler(it, dt)
            self._save_summary(global_bs, dt)
            self._maybe_validate()
            self._maybe_checkpoint()
        if self._pending_loss is not None:
            self.state["Loss"] = self._pending_loss.value()

    def prepare(self):
        """Set the model up for stepping without running the loop (used by bench/smoke)."""
        self._setup_model()
        return self

    def _step(self, batch: MiniBatch) -> torch.Tensor:
        """One iteration of the optimize loop: HIP-graph replay when ``bigdl.graph.capture`` is on
        and the batch has the captured shape (LocalOptimizer on a GPU), else eager."""
        if (type(self) is LocalOptimizer and self.device.type == "cuda"
                and config.get_property("bigdl.graph.capture")):
            from .graph_step import graphed_train_step
            g = getattr(self, "_graphed", None)
            x = batch.getInput()
            if g is None or (isinstance(x, torch.Tensor) and x.shape == g.sx.shape and x.dtype == g.sx.dtype):
                return graphed_train_step(self, batch)
        return self.train_step(batch)

    def train_step(self, batch: MiniBatch) -> torch.Tensor:
        """One synchronous-SGD iteration.  The FIRST iteration on a GPU is also the training compile
        phase (``bigdl.compile.trainAutotune``; the reference compiles ``TrainingPhase`` per replica,
        ``DL/optim/DistriOptimizer.scala:600-609``): its forward / backward-data / weight-gradient
        launches are recorded, and once it has finished each distinct geometry is re-timed under
        every kernel candidate and the fastest pinned (``nn.compiled.autotune_training_step``)."""
        if (not getattr(self, "_kernels_selected", False) and self.device.type == "cuda"
                and not torch.cuda.is_current_stream_capturing()):
            self._kernels_selected = True
            # bigdl.deterministic: no timing-based kernel choice (two runs could pin different tiles
            # for the same geometry, i.e. different accumulation orders, and lose bit reproducibility)
            if config.get_property("bigdl.compile.trainAutotune") and not config.get_property("bigdl.deterministic"):
                from ..nn.compiled import autotune_training_step
                loss, chosen = autotune_training_step(lambda: self._train_step_run(batch))
                self.selected_kernels = chosen
                if Engine.rank() == 0:
                    log.info(f"training compile phase: {len(chosen)} launch geometries re-tiled")
                return loss
        return self._train_step_run(batch)

    def _train_step_run(self, batch: MiniBatch) -> torch.Tensor:
        """One synchronous-SGD iteration on ``batch`` (see :meth:`_train_step_impl`).  On a GPU with
        ``bigdl.step.highPriority`` the iteration runs on a high-priority HIP stream, so the
        backward-data / BatchNorm chain wins the CUs over the side-stream weight-gradient kernels
        it overlaps with (``bigdl.conv.asyncWgrad``); the caller's stream waits for it at the end."""
        # Both stream tricks cost host time per step (stream switches, per-conv stream waits);
        # they pay only when the GPU, not the host, bounds the step: enable them once the measured
        # step period exceeds bigdl.step.overlapMinMs (ResNet-50 at batch 256: yes; VGG-CIFAR /
        # PTB, which are launch-bound: no)
        now = time.perf_counter()
        last = getattr(self, "_last_step_t", None)
        self._last_step_t = now
        if last is not None:
            dt = now - last
            ew = getattr(self, "_step_ewma", None)
            self._step_ewma = dt if ew is None else 0.7 * ew + 0.3 * dt
        knobs = getattr(self, "_step_knobs", None)
        if knobs is None:  # read once: config lookups cost microseconds a launch-bound step cannot spare
            knobs = self._step_knobs = (float(config.get_property("bigdl.step.overlapMinMs")),
                                        bool(config.get_property("bigdl.step.highPriority")),
                                        int(config.get_property("bigdl.step.maxInflight")))
        big = (getattr(self, "_step_ewma", None) or 0.0) * 1e3 >= knobs[0]
        self._overlap_now = big
        if self.device.type != "cuda" or torch.cuda.is_current_stream_capturing():
            return self._train_step_impl(batch)
        # bounded run-ahead: at most maxInflight iterations queued on the device (the host waits on
        # the end event of the oldest one); the reference's iteration ends on the host anyway
        inflight = getattr(self, "_inflight", None)
        if inflight is None:
            import collections
            inflight = self._inflight = collections.deque()
        while knobs[2] > 0 and len(inflight) >= knobs[2]:
            inflight.popleft().synchronize()
        if not big or not knobs[1]:
            loss = self._train_step_impl(batch)
            self._note_inflight(inflight)
            return loss
        hs = getattr(self, "_hp_stream", None)
        if hs is None:
            hs = self._hp_stream = torch.cuda.Stream(device=self.device, priority=-1)
        cur = torch.cuda.current_stream(self.device)
        hs.wait_stream(cur)
        for t in (batch.getInput(), batch.getTarget()):
            if isinstance(t, torch.Tensor) and t.is_cuda:
                t.record_stream(hs)
        with torch.cuda.stream(hs):
            loss = self._train_step_impl(batch)
        cur.wait_stream(hs)
        if isinstance(loss, torch.Tensor) and loss.is_cuda:
            loss.record_stream(cur)
        self._note_inflight(inflight)
        return loss

    def _note_inflight(self, inflight):
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        inflight.append(ev)

    def _train_step_impl(self, batch: MiniBatch) -> torch.Tensor:
        """One synchronous-SGD iteration on ``batch``; returns the (rank-averaged) loss as a
        device scalar without synchronising the host.  Phases (roctx ranges / HIP-event timers /
        JSON metrics per ``bigdl.roctx`` / ``bigdl.metrics.*``): forward, backward, then the
        optimizer's own (local: "compute weight"; distributed: "aggregate gradient",
        "compute weight", "send weights")."""
        m, crit = self.model, self.criterion
        tr = getattr(self, "tracer", None) or self._make_tracer()
        x, y = batch.getInput(), batch.getTarget()
        self._before_forward()
        m.zeroGradParameters()
        with tr.phase("forward"):
            out = m.forward(x)
            loss = crit.forward(out, y)
        with tr.phase("backward"):
            gout = crit.backward(out, y)
            self._before_backward()
            if getattr(self, "_overlap_now", False) and self.device.type == "cuda":
                from ..ops import native_ops as NO
                NO.async_wgrad(True)
                try:
                    m.backward(x, gout)
                finally:
                    NO.async_wgrad(False)
            else:
                m.backward(x, gout)
        loss_t = loss if isinstance(loss, torch.Tensor) else torch.tensor(float(loss))
        loss_t = self._reduce_scalar(loss_t.detach().float().reshape(()))
        self._sync_and_update(loss_t, batch.size())
        if tr.enabled:
            tr.end_iteration(self.state["neval"], {"epoch": self.state["epoch"], "batch": batch.size(),
                                                   "global_batch": batch.size() * Engine.world_size(),
                                                   "loss_prev": self.state.get("Loss")})
        return loss_t

    def _observe_straggler(self, it, host_dt):
        if self.drop_percentage <= 0 or it < getattr(self, "_straggler_warmup", 0):
            return
        tr = self.tracer
        ph = tr.last_phases
        # the rank's own computing time (forward + backward), like the reference's per-model
        # moduleTimeList: a synchronous collective makes every rank's wall time the slowest's
        dt = (ph.get("forward", 0.0) + ph.get("backward", 0.0)) if ph else host_dt
        from ..utils.tracing import allgather_floats
        tr.observe_step_time(it, dt, self.drop_percentage,
                             allgather_floats if Engine.world_size() > 1 else None)

    def _needs_loss(self) -> bool:
        from .trigger import MinLoss, TriggerAnd, TriggerOr

        def uses(t):
            if isinstance(t, MinLoss):
                return True
            if isinstance(t, (TriggerAnd, TriggerOr)):
                return any(uses(s) for s in t.triggers)
            return False
        return uses(self.end_when) or self.train_summary is not None

    def _hyper_str(self):
        return "".join(m.getHyperParameter() for m in self.optim_methods.values())

    def _before_forward(self):
        pass

    # ------------------------------------------------------------------------------ summary / validation / checkpoint
    def _save_summary(self, batch, dt):
        s = self.train_summary
        if s is None or Engine.rank() != 0:
            return
        it = self.state["neval"] - 1
        if s.should_write("Loss", self.state):
            s.add_scalar("Loss", float(self.state["Loss"]), it)
        if s.should_write("Throughput", self.state):
            s.add_scalar("Throughput", batch / dt if dt > 0 else 0.0, it)
        if s.should_write("LearningRate", self.state):
            lr = list(self.optim_methods.values())[0].getLearningRate()
            s.add_scalar("LearningRate", -lr if lr < 0 else lr, it)
        if s.should_write("Parameters", self.state):
            for mod in self.model.flattened_modules():
                p = mod.parameters() if not mod.children() else None
                if p:
                    for (w, g), wt, gt in zip(mod._param_slots, p[0], p[1]):
                        s.add_histogram(f"{mod.get_name()}/{w}", wt, it)
                        s.add_histogram(f"{mod.get_name()}/{g}", gt, it)

    def _maybe_validate(self):
        if self.validation_trigger is None or self.validation_set is None:
            return
        if not self.validation_trigger(self.state):
            return
        results = self.validate()
        if results:
            self.state["score"] = results[0][1].result()[0]
            for meth in self.optim_methods.values():
                meth.state["score"] = self.state["score"]
                for vm, r in results:
                    meth.state[vm.format()] = r.result()[0]

    def validate(self):
        self._flush_weights()
        m = self.model
        m.evaluate()
        results = None
        it = self.validation_set.data(train=False)
        with torch.no_grad():
            for b in it:
                b = b.to(self.device) if self.device.type == "cuda" else b
                out = m.forward(b.getInput())
                rs = [vm(out, b.getTarget()) for vm in self.validation_methods]
                results = rs if results is None else [a + r for a, r in zip(results, rs)]
        m.training()
        if results is None:
            return []
        results = allreduce_results(results)
        pairs = list(zip(self.validation_methods, results))
        if Engine.rank() == 0:
            for vm, r in pairs:
                log.info(f"{vm.format()} is {r}")
            if self.validation_summary is not None:
                for vm, r in pairs:
                    self.validation_summary.add_scalar(vm.format(), r.result()[0], self.state["neval"] - 1)
        return pairs

    def _flush_weights(self):
        """Make sure the fp32 weights in the arena are current (distributed overrides)."""

    def _maybe_checkpoint(self):
        if self.checkpoint_trigger is None or self.checkpoint_path is None:
            return
        if not self.checkpoint_trigger(self.state):
            return
        self.checkpoint(asynchronous=bool(config.get_property("bigdl.checkpoint.async")))

    def checkpoint(self, asynchronous: bool = False):
        """Write ``model.<neval>`` / ``optimMethod-*`` / ``state``; ``asynchronous`` returns after
        the host snapshot and leaves serialisation + file writes to the checkpoint writer thread."""
        from ..serialization.checkpoint import save_checkpoint
        self._flush_weights()
        if Engine.rank() == 0:
            save_checkpoint(self.checkpoint_path, self.model, self.optim_methods, self.state, self.is_overwrite,
                            asynchronous=asynchronous, slices=getattr(self, "_method_slices", None))

    def _maybe_resume(self):
        """Resume from the latest checkpoint when this process is a launcher restart
        (``BIGDL_RESTART_COUNT`` > 0, set by ``bigdl.launch --max-restarts``) or when
        ``bigdl.failure.resume`` is set, and a checkpoint exists under the checkpoint path."""
        import os
        from ..serialization.checkpoint import has_checkpoint
        restart = int(os.environ.get("BIGDL_RESTART_COUNT", "0") or 0) > 0
        if not (restart or config.get_property("bigdl.failure.resume")):
            return False
        if self.checkpoint_path is None or not has_checkpoint(self.checkpoint_path):
            return False
        log.info(f"resuming from the latest checkpoint under {self.checkpoint_path}")
        self._restore_latest()
        return True

    def _restore_latest(self):
        from ..serialization.checkpoint import load_latest_checkpoint
        model, methods, state = load_latest_checkpoint(
            self.checkpoint_path, world_size=Engine.world_size(), sharded=bool(getattr(self, "sharded", False)))
        if model is not None:
            p_dst = self.model.parameters()
            p_src = model.parameters()
            if p_dst is not None and p_src is not None:
                for a, b in zip(p_dst[0], p_src[0]):
                    a.copy_(b.to(a.device))
            ex_dst, ex_src = self.model.getExtraParameter(), model.getExtraParameter()
            if ex_dst and ex_src:
                for a, b in zip(ex_dst, ex_src):
                    a.copy_(b.to(a.device))
        if methods:
            # copy only the restored STATE into the live method objects: the per-run installation
            # (grad_scale = 1/W, folded L2 decay vectors, shard-space lr/decay vectors) lives on
            # those objects and is not part of a checkpoint.  Tensors are copied IN PLACE so a
            # captured HIP graph keeps pointing at the live state; when that is impossible (a
            # state tensor appears, disappears or changes shape) the graph is dropped and recaptured.
            graph_stale = False
            for cur, v in self._match_restored_methods(methods):
                for sk, sv in v.state.items():
                    old = cur.state.get(sk)
                    if isinstance(sv, torch.Tensor):
                        sv = sv.to(self.device)
                        if (isinstance(old, torch.Tensor) and old.shape == sv.shape and old.dtype == sv.dtype
                                and old.device == sv.device):
                            old.copy_(sv)
                            continue
                        graph_stale = True
                    cur.state[sk] = sv
                for sk in [k for k, t in cur.state.items() if isinstance(t, torch.Tensor) and k not in v.state]:
                    if sk == "_dev_n":
                        continue  # re-derived from evalCounter below
                    del cur.state[sk]
                    graph_stale = True
                cur.sync_device_counter()
            if graph_stale and getattr(self, "_graphed", None) is not None:
                log.info("optimizer state layout changed by the restore: the HIP-graph step will be recaptured")
                self._graphed = None
                self._graph_failed = False
        if state:
            self.state.update(state)
        if self.flat is not None and self.flat.shadow is not None:
            self.flat.refresh_shadow()
        self._on_restore()

    def _on_restore(self):
        pass

    def _match_restored_methods(self, methods):
        """Pair restored OptimMethods with the live ones: by the arena slice each owns when the
        checkpoint recorded it, else by key, else (one method on each side) directly.  Anything
        else is ambiguous and raises instead of guessing."""
        by_slice = {tuple(v): k for k, v in getattr(self, "_method_slices", {}).items()}
        pairs = []
        for k, v in methods.items():
            sl = getattr(v, "_arena_slice", None)
            if sl is not None and tuple(sl) in by_slice:
                pairs.append((self.optim_methods[by_slice[tuple(sl)]], v))
            elif k in self.optim_methods:
                pairs.append((self.optim_methods[k], v))
            elif len(methods) == 1 and len(self.optim_methods) == 1:
                pairs.append((next(iter(self.optim_methods.values())), v))
            else:
                raise ValueError(f"checkpointed OptimMethod '{k}' matches no live OptimMethod "
                                 f"({sorted(self.optim_methods)}) by arena slice or name")
        return pairs


class LocalOptimizer(BaseOptimizer):
    """Single-device trainer (``LocalOptimizer.scala:45-295``).  The reference clones one replica
    per core and sums their gradients; a GPU is one replica, so the loop is direct."""

    def __init__(self, model, training_set, criterion, optim_method=None, end_trigger=None, batch_size=32,
                 bigdl_type="float"):
        super().__init__(model, training_set, criterion, batch_size)
        if optim_method is not None:
            if isinstance(optim_method, dict):
                self.setOptimMethods(optim_method)
            else:
                self.setOptimMethod(optim_method)
        if end_trigger is not None:
            self.setEndWhen(end_trigger)


class Optimizer:
    """Factory mirroring ``object Optimizer`` and pyspark ``Optimizer.create``."""

    def __new__(cls, model, training_rdd=None, criterion=None, end_trigger=None, batch_size=32, optim_method=None,
                bigdl_type="float", **kw):
        return Optimizer.create(model, training_rdd, criterion, end_trigger, batch_size, optim_method)

    @staticmethod
    def create(model, training_set, criterion, end_trigger=None, batch_size=32, optim_method=None,
               cores=None, bigdl_type="float", distributed: Optional[bool] = None):
        if distributed is None:
            distributed = Engine.is_distributed() or (
                hasattr(training_set, "world") and getattr(training_set, "world", 1) > 1)
        if distributed:
            from ..parallel.distri_optimizer import DistriOptimizer
            opt = DistriOptimizer(model, training_set, criterion, optim_method, end_trigger, batch_size)
        else:
            opt = LocalOptimizer(model, training_set, criterion, optim_method, end_trigger, batch_size)
        return opt


# ---- pyspark ``bigdl.optim.optimizer`` namespace: every optimizer-side class in one module ----
from .optim_method import *  # noqa: E402,F401,F403
from .trigger import *  # noqa: E402,F401,F403
from .validation import *  # noqa: E402,F401,F403
from .regularizer import L1L2Regularizer, L1Regularizer, L2Regularizer  # noqa: E402,F401
from ..visualization import TrainSummary, ValidationSummary  # noqa: E402,F401


class ActivityRegularization(L1L2Regularizer):
    """pyspark ``ActivityRegularization(l1, l2)`` — L1 and L2 together."""


def DistriOptimizer(*args, **kwargs):  # noqa: N802 - pyspark class name
    from ..parallel.distri_optimizer import DistriOptimizer as _D
    return _D(*args, **kwargs)
