"""Module / Criterion base classes.

Reference: ``DL/nn/abstractnn/AbstractModule.scala:59-1200``.

Contract kept from the reference
--------------------------------
* ``forward(input)`` = (lazy parameter update hook) + ``updateOutput`` with a wall-clock timer
  (``AbstractModule.scala:255-270``).
* ``backward(input, gradOutput)`` = ``updateGradInput`` + ``accGradParameters`` + gradient-ready
  hook (``:282-297``; the hook is where the ParallelOptimizer pushed a layer's gradient — here the
  bucketed RCCL reduce-scatter of :mod:`bigdl.parallel` attaches).
* ``accGradParameters`` ACCUMULATES ``scale * dL/dW`` into ``gradWeight``; ``zeroGradParameters``
  clears it.
* ``parameters()`` returns ``([weights], [grads])``; ``getParameters()`` compacts every weight
  and gradient into ONE contiguous storage and re-points the layers at views of it
  (``:988-1000`` and ``DL/nn/Module.scala:113-166``).  That flat arena is what the optimizer and
  the collectives operate on (zero-copy buckets).

Device / precision design (MI355X-first)
----------------------------------------
Weights and gradients are fp32 master tensors.  When the engine's compute dtype is bf16,
layers read their weights through :meth:`cw` which returns a bf16 *shadow* — a view into the
arena's bf16 copy, refreshed once per optimizer step by the fused optimizer kernel (or lazily by
a single cast when the fp32 arena changed behind its back; detected through torch's shared view
version counter).
"""
from __future__ import annotations

import functools
import inspect
import time
from collections import OrderedDict
from typing import Any, Callable, List, Optional, Tuple

import numpy as np

import torch

from ..utils.engine import Engine
from ..utils.table import Table
from ..utils import config

_DEV_TIMERS = [bool(config.get_property("bigdl.profile.deviceTimers"))]
config.on_change("bigdl.profile.deviceTimers", lambda v: _DEV_TIMERS.__setitem__(0, bool(v)))
# read on every module forward / backward: cached, refreshed by config.set_property listeners
_PROFILE_SYNC = [bool(config.get_property("bigdl.profile.sync"))]
config.on_change("bigdl.profile.sync", lambda v: _PROFILE_SYNC.__setitem__(0, bool(v)))


class LayerException(RuntimeError):
    """Wraps a failure with the module path (``DL/utils/LayerException.scala``)."""

    def __init__(self, layer_msg: str, cause: BaseException):
        super().__init__(f"{layer_msg}: {cause}")
        self.layer_msg = layer_msg
        self.cause = cause


# ----------------------------------------------------------------------------------------------
# activity helpers
# ----------------------------------------------------------------------------------------------

def flatten_activity(a) -> List[torch.Tensor]:
    if isinstance(a, torch.Tensor):
        return [a]
    if isinstance(a, Table):
        out = []
        for k in sorted(a.keys(), key=lambda k: (not isinstance(k, int), str(k) if not isinstance(k, int) else k)):
            out.extend(flatten_activity(a[k]))
        return out
    if isinstance(a, (list, tuple)):
        out = []
        for v in a:
            out.extend(flatten_activity(v))
        return out
    return []


def unflatten_like(template, flat: List, pos: int = 0):
    if isinstance(template, torch.Tensor):
        return flat[pos], pos + 1
    if isinstance(template, Table):
        t = Table()
        for k in sorted(template.keys(), key=lambda k: (not isinstance(k, int), str(k) if not isinstance(k, int) else k)):
            v, pos = unflatten_like(template[k], flat, pos)
            t[k] = v
        return t, pos
    if isinstance(template, (list, tuple)):
        vals = []
        for v in template:
            r, pos = unflatten_like(v, flat, pos)
            vals.append(r)
        return type(template)(vals), pos
    return template, pos


def map_activity(a, fn):
    if isinstance(a, torch.Tensor):
        return fn(a)
    if isinstance(a, Table):
        t = Table()
        for k, v in a.items():
            t[k] = map_activity(v, fn)
        return t
    if isinstance(a, (list, tuple)):
        return type(a)(map_activity(v, fn) for v in a)
    return a


def to_torch(x, device=None, dtype=None):
    """Accept numpy / torch / bigdl Tensor / Table / list and return torch (Table for lists)."""
    from ..tensor.tensor import Tensor as BTensor
    if isinstance(x, BTensor):
        x = x.data
    if isinstance(x, np.ndarray):
        x = torch.from_numpy(np.ascontiguousarray(x))
    if isinstance(x, torch.Tensor):
        if device is not None and x.device != torch.device(device):
            x = x.to(device, non_blocking=True)
        if dtype is not None and x.is_floating_point() and x.dtype != dtype:
            x = x.to(dtype)
        return x
    if isinstance(x, Table):
        t = Table()
        for k, v in x.items():
            t[k] = to_torch(v, device, dtype)
        return t
    if isinstance(x, (list, tuple)):
        return Table(*[to_torch(v, device, dtype) for v in x])
    if isinstance(x, (int, float)):
        return torch.tensor(x)
    return x


# ----------------------------------------------------------------------------------------------
# flat parameter arena
# ----------------------------------------------------------------------------------------------

#: process-wide mutation epoch: bumped by every training-mode forward and every native weight write
#: (ops.fp32x3.mark_dirty); caches of weight-derived state compare it (AbstractModule._cached_predictor)
_MUTATION = [0]


class FlatParameters:
    """One contiguous fp32 weight storage, one fp32 grad storage, optional bf16 shadow.

    ``slices`` records (module, weight_attr, grad_attr, offset, numel, shape) for every
    parameter in ``parameters()`` order, so buckets and shards map back to layers.
    """

    def __init__(self, weight: torch.Tensor, grad: torch.Tensor, slices):
        self.weight = weight
        self.grad = grad
        self.slices = slices
        self.shadow: Optional[torch.Tensor] = None
        self.shadow_version = -1
        #: bumped whenever the shadow's contents change (refresh / optimizer update): caches derived
        #: from the bf16 weights (the dgrad weight transforms, ops/native_ops.py) key on it
        self.shadow_gen = 0
        self.buckets = [(0, weight.numel())]

    @property
    def numel(self) -> int:
        return self.weight.numel()

    def enable_shadow(self, dtype=torch.bfloat16):
        if self.shadow is None or self.shadow.dtype != dtype:
            self.shadow = torch.empty(self.weight.numel(), dtype=dtype, device=self.weight.device)
            for (m, wname, gname, off, n, shape) in self.slices:
                m._shadow_views[wname] = m._view_param(self.shadow[off:off + n], wname, shape)
                m._arena = self
            if self.shadow.is_cuda:
                from ..ops import native_ops
                native_ops.register_shadow_arena(self)
        self.refresh_shadow()

    def refresh_shadow(self):
        if self.shadow is not None:
            from .. import ops
            ops.cast_copy(self.shadow, self.weight)
            self.shadow_version = self.weight._version
            self.shadow_gen += 1

    def mark_shadow_fresh(self):
        self.shadow_version = self.weight._version
        self.shadow_gen += 1

    def shadow_is_fresh(self) -> bool:
        return self.shadow is not None and self.shadow_version == self.weight._version


# ----------------------------------------------------------------------------------------------
# module base
# ----------------------------------------------------------------------------------------------

def _record_ctor(init):
    @functools.wraps(init)
    def wrapper(self, *args, **kwargs):
        outer = not getattr(self, "_in_ctor", False)
        if outer:
            object.__setattr__(self, "_in_ctor", True)
            try:
                sig = inspect.signature(init)
                bound = sig.bind(self, *args, **kwargs)
                bound.apply_defaults()
                ctor = OrderedDict((k, v) for k, v in bound.arguments.items() if k != "self")
                # flatten **kwargs / *args parameters
                for pname, p in sig.parameters.items():
                    if p.kind == inspect.Parameter.VAR_KEYWORD and pname in ctor:
                        ctor.update(ctor.pop(pname))
                object.__setattr__(self, "_ctor_args", ctor)
            except TypeError:
                object.__setattr__(self, "_ctor_args", OrderedDict())
        try:
            init(self, *args, **kwargs)
        finally:
            if outer:
                object.__setattr__(self, "_in_ctor", False)
    wrapper._bigdl_wrapped = True
    return wrapper


class AbstractModule:
    """Base of every layer (``AbstractModule.scala:59``)."""

    #: Scala class name used by the .bigdl serializer; subclasses may override.
    SCALA_PACKAGE = "com.intel.analytics.bigdl.nn"

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        init = cls.__dict__.get("__init__")
        if init is not None and not getattr(init, "_bigdl_wrapped", False):
            cls.__init__ = _record_ctor(init)

    def __init__(self):
        self.output: Any = torch.empty(0)
        self.gradInput: Any = torch.empty(0)
        self.train = True
        self._name: Optional[str] = None
        self.forward_time = 0.0
        self.backward_time = 0.0
        self.scale_w = 1.0
        self.scale_b = 1.0
        self.wRegularizer = None
        self.bRegularizer = None
        self._param_slots: List[Tuple[str, str]] = []
        self._param_layouts: dict = {}
        self._buffer_names: List[str] = []
        self._frozen = False
        self._shadow_views: dict = {}
        self._shadow_cache: dict = {}
        self._arena: Optional[FlatParameters] = None
        self._pre_forward_hooks: List[Callable] = []
        self._grad_ready_hooks: List[Callable] = []
        self._init_weight_method = None
        self._init_bias_method = None
        self._input_shape = None
        self._output_shape = None
        if not hasattr(self, "_ctor_args"):
            self._ctor_args = OrderedDict()

    # ---- naming ---------------------------------------------------------------------------
    def set_name(self, name: str):
        self._name = name
        return self

    setName = set_name

    def get_name(self) -> str:
        if self._name is None:
            self._name = f"{type(self).__name__}{id(self) & 0xFFFFFF:x}"
        return self._name

    getName = get_name

    def name(self) -> str:
        return self.get_name()

    @classmethod
    def scala_class_name(cls) -> str:
        return f"{cls.SCALA_PACKAGE}.{getattr(cls, 'SCALA_NAME', cls.__name__)}"

    def __repr__(self):
        return f"{type(self).__name__}[{self.get_name()}]"

    def __str__(self):
        return self.__repr__()

    # ---- parameters -------------------------------------------------------------------------
    def register_parameter(self, wname: str, weight: torch.Tensor, gname: Optional[str] = None,
                           layout: Optional[Tuple[Tuple[int, ...], Tuple[int, ...]]] = None):
        """Register a trainable tensor.  ``layout=(phys_shape, perm)`` stores it physically as
        ``phys_shape`` and exposes ``phys.permute(perm)`` as the logical (BigDL-shaped) tensor —
        used for conv weights kept KRSC for the NHWC implicit-GEMM kernels."""
        gname = gname or ("grad" + wname[0].upper() + wname[1:])
        if layout is not None:
            self._param_layouts[wname] = layout
            w = torch.empty(layout[0], dtype=weight.dtype, device=weight.device).permute(layout[1])
            w.copy_(weight)
            weight = w
            g = torch.zeros(layout[0], dtype=weight.dtype, device=weight.device).permute(layout[1])
        else:
            g = torch.zeros_like(weight)
        setattr(self, wname, weight)
        setattr(self, gname, g)
        self._param_slots.append((wname, gname))

    def _view_param(self, flat: torch.Tensor, wname: str, shape) -> torch.Tensor:
        lay = self._param_layouts.get(wname)
        if lay is None:
            return flat.view(shape)
        return flat.view(lay[0]).permute(lay[1])

    def register_buffer(self, name: str, value: torch.Tensor):
        setattr(self, name, value)
        if name not in self._buffer_names:
            self._buffer_names.append(name)

    def parameters(self) -> Optional[Tuple[List[torch.Tensor], List[torch.Tensor]]]:
        if not self._param_slots:
            return None
        return ([getattr(self, w) for w, _ in self._param_slots],
                [getattr(self, g) for _, g in self._param_slots])

    def _param_entries(self) -> List[Tuple["AbstractModule", str, str]]:
        return [(self, w, g) for w, g in self._param_slots]

    def getParametersTable(self) -> Table:
        t = Table()
        p = self.parameters()
        if p is not None:
            inner = Table()
            for (w, g), wt, gt in zip(self._param_slots, p[0], p[1]):
                inner[w] = wt
                inner[g] = gt
            t[self.get_name()] = inner
        return t

    def getExtraParameter(self) -> Optional[List[torch.Tensor]]:
        """Non-trainable state (e.g. BN running stats), ``AbstractModule.scala:358``."""
        if not self._buffer_names:
            return None
        return [getattr(self, b) for b in self._buffer_names]

    def setExtraParameter(self, extra: List[torch.Tensor]):
        mine = self.getExtraParameter() or []
        for a, b in zip(mine, extra):
            a.copy_(b)
        return self

    def zeroGradParameters(self):
        p = self.parameters()
        if p is not None:
            if self._arena is not None:
                pass  # arena owner zeros once
            for g in p[1]:
                g.zero_()

    zero_grad_parameters = zeroGradParameters

    def getParameters(self) -> Tuple[torch.Tensor, torch.Tensor]:
        """Compact all weights and grads into one storage each; return the flat views."""
        entries = self._param_entries()
        if not entries:
            e = torch.empty(0)
            return e, e
        dev = getattr(entries[0][0], entries[0][1]).device
        # already compact?
        if self._arena is not None and self._arena.slices and len(self._arena.slices) == len(entries) and all(
                m is sm and w == sw and getattr(m, w).data_ptr() == self._arena.weight[off:].data_ptr()
                for (m, w, g), (sm, sw, _, off, _, _) in zip(entries, self._arena.slices)):
            return self._arena.weight, self._arena.grad
        total = sum(getattr(m, w).numel() for m, w, _ in entries)
        flat_w = torch.empty(total, dtype=torch.float32, device=dev)
        flat_g = torch.zeros(total, dtype=torch.float32, device=dev)
        slices = []
        off = 0
        seen = {}
        for m, w, g in entries:
            wt = getattr(m, w)
            n = wt.numel()
            shape = wt.shape
            wv = m._view_param(flat_w[off:off + n], w, shape)
            gv = m._view_param(flat_g[off:off + n], w, shape)
            wv.copy_(wt)
            gt = getattr(m, g)
            if gt is not None and gt.numel() == n:
                gv.copy_(gt.reshape(shape))
            setattr(m, w, wv)
            setattr(m, g, gv)
            slices.append((m, w, g, off, n, shape))
            off += n
        arena = FlatParameters(flat_w, flat_g, slices)
        for m, *_ in slices:
            m._arena = arena
            m._shadow_views = {}
        self._set_arena_recursive(arena)
        return flat_w, flat_g

    def compactParametersBucketed(self, bucket_bytes: int, multiple: int):
        """Re-lay the flat arena so gradient buckets are contiguous, start on 256-B boundaries and
        have a length divisible by ``multiple`` (= world size × 64): every bucket is then directly a
        reduce-scatter input / all-gather output with equal per-rank shards.  Buckets are cut at
        parameter boundaries, in arena order (backward produces them last-to-first).  The padding
        gaps hold zeros in weights and grads.  Returns the arena with ``buckets=[(lo, hi), ...]``."""
        self.getParameters()
        old = self._arena
        if old is None:
            return None
        groups, cur, cur_bytes = [], [], 0
        for s in old.slices:
            cur.append(s)
            cur_bytes += s[4] * 4
            if cur_bytes >= bucket_bytes:
                groups.append(cur)
                cur, cur_bytes = [], 0
        if cur:
            groups.append(cur)
        align = 64
        total = 0
        layout = []
        for g in groups:
            lo = total
            off = lo
            placed = []
            for s in g:
                placed.append((s, off))
                off += s[4]
            n = off - lo
            n_pad = ((n + multiple - 1) // multiple) * multiple
            hi = lo + n_pad
            layout.append((placed, lo, hi))
            total = ((hi + align - 1) // align) * align
        dev = old.weight.device
        flat_w = torch.zeros(total, dtype=torch.float32, device=dev)
        flat_g = torch.zeros(total, dtype=torch.float32, device=dev)
        slices, buckets = [], []
        for placed, lo, hi in layout:
            for (m, w, g, _, n, shape), off in placed:
                wv = m._view_param(flat_w[off:off + n], w, shape)
                gv = m._view_param(flat_g[off:off + n], w, shape)
                wv.copy_(getattr(m, w))
                gv.copy_(getattr(m, g))
                setattr(m, w, wv)
                setattr(m, g, gv)
                m._shadow_views = {}
                slices.append((m, w, g, off, n, shape))
            buckets.append((lo, hi))
        arena = FlatParameters(flat_w, flat_g, slices)
        arena.buckets = buckets
        for m, *_ in slices:
            m._arena = arena
        self._set_arena_recursive(arena)
        return arena

    def _set_arena_recursive(self, arena):
        self._arena = arena

    def flat_parameters(self) -> Optional[FlatParameters]:
        return self._arena

    # ---- compute-dtype weights ---------------------------------------------------------------
    def cw(self, name: str, dtype: Optional[torch.dtype] = None) -> torch.Tensor:
        """Weight ``name`` in the compute dtype (bf16 shadow when enabled)."""
        w = getattr(self, name)
        dt = dtype or self.compute_dtype_for(w)
        if w.dtype == dt:
            return w
        arena = self._arena
        if arena is not None and name in self._shadow_views and arena.shadow is not None and arena.shadow.dtype == dt:
            if not arena.shadow_is_fresh():
                arena.refresh_shadow()
            return self._shadow_views[name]
        key = (w.data_ptr(), w._version, dt)
        c = self._shadow_cache.get(name)
        if c is None or c[0] != key:
            c = (key, w.to(dt))
            self._shadow_cache[name] = c
        return c[1]

    def compute_dtype_for(self, t: torch.Tensor) -> torch.dtype:
        if t.device.type == "cuda":
            return Engine.compute_dtype()
        # host: fp32 like the reference's Float models; a module cast to float64 (the gradient
        # checker, nn/gradient_checker.py) keeps computing in float64
        return torch.float64 if t.dtype == torch.float64 else torch.float32

    # ---- device ----------------------------------------------------------------------------------
    def _tensors_attrs(self):
        names = []
        for w, g in self._param_slots:
            names += [w, g]
        names += self._buffer_names
        return names

    def to(self, device=None, dtype=None):
        for n in self._tensors_attrs():
            t = getattr(self, n, None)
            if isinstance(t, torch.Tensor):
                t2 = t
                if device is not None and n in self._param_layouts and t2.device != torch.device(device):
                    lay = self._param_layouts[n]
                    inv = [0] * len(lay[1])
                    for i, p in enumerate(lay[1]):
                        inv[p] = i
                    t2 = t2.permute(inv).contiguous().to(device).permute(lay[1])
                elif device is not None:
                    t2 = t2.to(device)
                if dtype is not None and t2.is_floating_point():
                    t2 = t2.to(dtype)
                setattr(self, n, t2)
        self._arena = None
        self._shadow_views = {}
        self._shadow_cache = {}
        for c in self.children():
            c.to(device, dtype)
        return self

    def cuda(self, device=None):
        return self.to(device or Engine.device())

    def cpu(self):
        return self.to("cpu")

    def children(self) -> List["AbstractModule"]:
        return []

    # ---- train / eval ------------------------------------------------------------------------------
    def training(self, is_training: bool = True):
        self.train = is_training
        for c in self.children():
            c.training(is_training)
        return self

    def evaluate(self, *args, **kwargs):
        """``evaluate()`` → eval mode; with arguments → model evaluation (AbstractModule.scala:637-918)."""
        if not args and not kwargs:
            return self.training(False)
        from ..optim.evaluator import evaluate_model
        return evaluate_model(self, *args, **kwargs)

    def isTraining(self) -> bool:
        return self.train

    is_training = isTraining

    def freeze(self, *names):
        if not names:
            self._frozen = True
            self.scale_w = 0.0
            self.scale_b = 0.0
            for c in self.children():
                c.freeze()
        else:
            for n in names:
                for m in self.flattened_modules():
                    if m.get_name() == n:
                        m.freeze()
        return self

    def unFreeze(self, *names):
        if not names:
            self._frozen = False
            self.scale_w = 1.0
            self.scale_b = 1.0
            for c in self.children():
                c.unFreeze()
        else:
            for n in names:
                for m in self.flattened_modules():
                    if m.get_name() == n:
                        m.unFreeze()
        return self

    unfreeze = unFreeze

    def setScaleW(self, w: float):
        self.scale_w = w
        return self

    def setScaleB(self, b: float):
        self.scale_b = b
        return self

    def flattened_modules(self) -> List["AbstractModule"]:
        out = [self]
        for c in self.children():
            out.extend(c.flattened_modules())
        return out

    # ---- forward / backward -------------------------------------------------------------------------
    def updateOutput(self, input):
        raise NotImplementedError(type(self).__name__)

    def updateGradInput(self, input, gradOutput):
        raise NotImplementedError(type(self).__name__)

    def accGradParameters(self, input, gradOutput):
        pass

    # HIP-event per-module timers (bigdl.profile.deviceTimers): events are recorded around
    # forward / backward on the current stream and resolved only when getDeviceTimes() asks, so
    # timing never synchronises the step (SURVEY §2.12 "HIP-event per-module timers")
    def _dev_start(self, x):
        if not _DEV_TIMERS[0]:
            return None
        t = x if isinstance(x, torch.Tensor) else next((v for v in (x.values() if isinstance(x, Table) else ())
                                                         if isinstance(v, torch.Tensor)), None)
        if t is None or not t.is_cuda or torch.cuda.is_current_stream_capturing():
            return None
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    def _dev_stop(self, start, which):
        if start is None:
            return
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        pend = self.__dict__.setdefault("_dev_pending", [])
        pend.append((start, e, which))

    def _dev_resolve(self):
        pend = self.__dict__.get("_dev_pending")
        acc = self.__dict__.setdefault("_dev_times", [0.0, 0.0])
        if pend:
            for s, e, which in pend:
                e.synchronize()
                acc[which] += s.elapsed_time(e) / 1e3
            pend.clear()
        return acc

    def getDeviceTimes(self):
        """[(module, forward_s, backward_s)] measured on the device by HIP events (requires
        ``bigdl.profile.deviceTimers``); containers include their children's time."""
        f, b = self._dev_resolve()
        out = [(self, f, b)]
        for c in self.children():
            out.extend(c.getDeviceTimes())
        return out

    def _sync_for_timing(self):
        if _PROFILE_SYNC[0] and torch.cuda.is_available():
            torch.cuda.synchronize()

    def forward(self, input):
        conv_back = None
        if self.train:
            _MUTATION[0] += 1  # a training forward may update buffers (BN running statistics) natively
        if not isinstance(input, (torch.Tensor, Table)):
            conv_back = type(input)
            input = to_torch(input)
        for h in self._pre_forward_hooks:
            h(self)
        self._sync_for_timing()
        t0 = time.perf_counter()
        ev = self._dev_start(input)
        try:
            self.output = self.updateOutput(input)
        except LayerException:
            raise
        except Exception as e:  # noqa: BLE001 - wrap with the layer path as the reference does
            raise LayerException(f"Layer info: {self}", e) from e
        self._dev_stop(ev, 0)
        self._sync_for_timing()
        self.forward_time += time.perf_counter() - t0
        if conv_back is np.ndarray:
            return _to_numpy(self.output)
        return self.output

    def backward(self, input, gradOutput):
        conv_back = None
        from ..ops.reference import BNGrad  # a deferred BN input gradient passes through as is
        if not isinstance(input, (torch.Tensor, Table)):
            conv_back = type(gradOutput)
            input = to_torch(input)
            gradOutput = to_torch(gradOutput)
        elif not isinstance(gradOutput, (torch.Tensor, Table, BNGrad)):
            conv_back = type(gradOutput)
            gradOutput = to_torch(gradOutput)
        self._sync_for_timing()
        t0 = time.perf_counter()
        ev = self._dev_start(gradOutput)
        self.gradInput = self.updateGradInput(input, gradOutput)
        self.accGradParameters(input, gradOutput)
        self._dev_stop(ev, 1)
        self._sync_for_timing()
        self.backward_time += time.perf_counter() - t0
        for h in self._grad_ready_hooks:
            h(self)
        if conv_back is np.ndarray:
            return _to_numpy(self.gradInput)
        return self.gradInput

    def __call__(self, *nodes):
        """Graph construction: ``layer(node1, node2)`` → ModuleNode (``inputs``, AbstractModule.scala:773)."""
        from .graph import ModuleNode
        return ModuleNode.create(self, list(nodes))

    def inputs(self, *nodes):
        return self.__call__(*nodes)

    # ---- update helpers ------------------------------------------------------------------------------
    def updateParameters(self, learning_rate: float):
        p = self.parameters()
        if p is not None:
            for w, g in zip(*p):
                w.add_(g, alpha=-learning_rate)

    update_parameters = updateParameters

    def reset(self):
        return self

    def resetTimes(self):
        self.forward_time = 0.0
        self.backward_time = 0.0
        self.__dict__.pop("_dev_pending", None)
        self.__dict__.pop("_dev_times", None)
        for c in self.children():
            c.resetTimes()

    def getTimes(self):
        """[(module, forwardTime, backwardTime)] in seconds (``AbstractModule.scala:168-190``)."""
        out = [(self, self.forward_time, self.backward_time)]
        for c in self.children():
            out.extend(c.getTimes())
        return out

    def getTimesGroupByModuleType(self):
        agg = OrderedDict()
        for m, f, b in self.getTimes():
            k = type(m).__name__
            a = agg.get(k, (0.0, 0.0))
            agg[k] = (a[0] + f, a[1] + b)
        return [(k, f, b) for k, (f, b) in agg.items()]

    def clearState(self):
        self.output = torch.empty(0)
        self.gradInput = torch.empty(0)
        for c in self.children():
            c.clearState()
        return self

    def __getstate__(self):
        d = dict(self.__dict__)
        d.pop("_predictor_cache", None)  # compiled forms (HIP graphs) of this module: rebuilt on demand
        return d

    def cloneModule(self):
        import copy
        return copy.deepcopy(self)

    clone_module = cloneModule

    def setWRegularizer(self, r):
        self.wRegularizer = r
        return self

    def setBRegularizer(self, r):
        self.bRegularizer = r
        return self

    def setInitMethod(self, weight_init_method=None, bias_init_method=None):
        if weight_init_method is not None:
            self._init_weight_method = weight_init_method
        if bias_init_method is not None:
            self._init_bias_method = bias_init_method
        self.reset()
        return self

    set_init_method = setInitMethod

    # ---- pyspark-style weight access ----------------------------------------------------------------
    def get_weights(self):
        p = self.parameters()
        if p is None:
            return None
        return [w.detach().float().cpu().numpy() for w in p[0]]

    def set_weights(self, weights):
        p = self.parameters()
        if p is None:
            raise ValueError("module has no weights")
        if len(weights) != len(p[0]):
            raise ValueError(f"expected {len(p[0])} weight tensors, got {len(weights)}")
        for dst, src in zip(p[0], weights):
            src = to_torch(src)
            if tuple(src.shape) != tuple(dst.shape):
                src = src.reshape(dst.shape)
            dst.copy_(src)
        return self

    setWeightsBias = set_weights

    def getWeightsBias(self):
        p = self.parameters()
        return None if p is None else list(p[0])

    def is_with_weights(self) -> bool:
        return self.parameters() is not None

    # ---- save / load (implemented in bigdl.serialization) -------------------------------------------
    def saveModule(self, path: str, weight_path: Optional[str] = None, over_write: bool = False):
        from ..serialization.module_serializer import save_module
        save_module(self, path, weight_path, over_write)
        return self

    save_module = saveModule

    def saveModel(self, model_path, weight_path=None, over_write=False):
        return self.saveModule(model_path, weight_path, over_write)

    def save(self, path: str, over_write: bool = False):
        return self.saveModule(path, None, over_write)

    def saveDefinition(self, path: str, over_write: bool = False):
        from ..serialization.module_serializer import save_definition
        save_definition(self, path, over_write)
        return self

    def saveTorch(self, path: str, over_write: bool = False):
        from ..serialization.torch_file import save_torch
        save_torch(self, path, over_write)
        return self

    def saveCaffe(self, prototxt_path: str, model_path: str, use_v2: bool = True, over_write: bool = False):
        from ..serialization.caffe_persister import save_caffe
        save_caffe(self, prototxt_path, model_path, use_v2, over_write)
        return self

    save_caffe = saveCaffe

    # ---- inference helpers ----------------------------------------------------------------------------
    def _cached_predictor(self, batch_size: int):
        """One LocalPredictor per (model, batch size), so repeated ``predict`` calls reuse its lowered
        / compiled forms; refreshed when any weight or buffer may have changed since it compiled: a
        torch in-place write (version counters), a native optimizer update / weight collective, or a
        training-mode forward (BN running statistics) anywhere in the process (:data:`_MUTATION`)."""
        from ..optim.predictor import LocalPredictor
        ps = self.parameters()
        bufs = [getattr(m, n, None) for m in self.flattened_modules() for n in getattr(m, "_buffer_names", ())]
        sig = (_MUTATION[0], tuple(t._version for t in (list(ps[0]) if ps else []) + bufs
                                   if isinstance(t, torch.Tensor)))
        c = self.__dict__.get("_predictor_cache")  # dropped by __getstate__: clones / pickles never carry it
        if c is None or c[0] != batch_size:
            c = self.__dict__["_predictor_cache"] = [batch_size, LocalPredictor(self, batch_size=batch_size), sig]
        elif c[2] != sig:
            c[1].refresh()
            c[2] = sig
        return c[1]

    def predict(self, features, batch_size: int = -1):
        return self._cached_predictor(batch_size).predict(features)

    def predictClass(self, features, batch_size: int = -1):
        return self._cached_predictor(batch_size).predict_class(features)

    predict_class = predictClass
    predict_local = predict
    predict_class_local = predictClass

    def quantize(self):
        from .quantized.quantizer import quantize
        return quantize(self)

    def toGraph(self, *start_nodes):
        from .graph import to_graph
        return to_graph(self)

    def setInputShape(self, s):
        self._input_shape = s
        return self


def _to_numpy(a):
    if isinstance(a, torch.Tensor):
        return a.detach().float().cpu().numpy() if a.is_floating_point() else a.detach().cpu().numpy()
    if isinstance(a, Table):
        return [_to_numpy(v) for v in a]
    return a


class TensorModule(AbstractModule):
    """Tensor → Tensor module (``AbstractModule.scala:48``)."""


# ----------------------------------------------------------------------------------------------
# autograd-backed module: explicit forward, backward derived by reverse-mode AD
# ----------------------------------------------------------------------------------------------

class AutogradModule(TensorModule):
    """Layers whose forward is a composition of torch device ops.

    The long tail of cold layers (≈150 of the ≈190 reference layers) is defined only by a
    forward function here; ``updateGradInput``/``accGradParameters`` are derived from the
    recorded graph.  Hot-path layers (conv, BN, linear, pooling, activations, softmax, LSTM…)
    override all three methods with explicit HIP kernels instead.
    """

    def _forward(self, input):  # pragma: no cover - abstract
        raise NotImplementedError

    def P(self, name: str) -> torch.Tensor:
        leaves = getattr(self, "_leaves", None)
        if leaves is not None and name in leaves:
            return leaves[name]
        return getattr(self, name)

    def _diff_inputs(self, input):
        flat = flatten_activity(input)
        leaves = []
        for t in flat:
            if t.is_floating_point():
                leaves.append(t.detach().requires_grad_(True))
            else:
                leaves.append(t)
        rebuilt, _ = unflatten_like(input, leaves)
        return rebuilt, leaves

    def _build_graph(self, input):
        xin, xleaves = self._diff_inputs(input)
        self._leaves = OrderedDict()
        for w, _ in self._param_slots:
            self._leaves[w] = getattr(self, w).detach().requires_grad_(True)
        try:
            with torch.enable_grad():
                out = self._forward(xin)
        finally:
            pleaves = self._leaves
            self._leaves = None
        self._graph = (id(input), xleaves, pleaves, out)
        self._pgrads = None
        return out

    def updateOutput(self, input):
        if self.train:
            out = self._build_graph(input)
            return map_activity(out, lambda t: t.detach())
        self._graph = None
        with torch.no_grad():
            return self._forward(input)

    def _run_backward(self, input, gradOutput):
        g = getattr(self, "_graph", None)
        if g is None or g[0] != id(input):
            self._build_graph(input)
            g = self._graph
        _, xleaves, pleaves, out = g
        outs = flatten_activity(out)
        gos = flatten_activity(gradOutput)
        pairs = [(o, go) for o, go in zip(outs, gos) if o.requires_grad]
        targets = [x for x in xleaves if x.requires_grad] + list(pleaves.values())
        if pairs and targets:
            grads = torch.autograd.grad([o for o, _ in pairs], targets,
                                        [go.to(o.dtype) for o, go in pairs], allow_unused=True)
        else:
            grads = [None] * len(targets)
        gi = []
        k = 0
        for x in xleaves:
            if x.requires_grad:
                gx = grads[k]
                k += 1
                gi.append(torch.zeros_like(x) if gx is None else gx)
            else:
                gi.append(torch.zeros_like(x, dtype=torch.float32) if x.is_floating_point() else x)
        self._pgrads = OrderedDict()
        for name in pleaves:
            self._pgrads[name] = grads[k]
            k += 1
        self._graph = None
        grad_input, _ = unflatten_like(input, gi)
        return grad_input

    def updateGradInput(self, input, gradOutput):
        return self._run_backward(input, gradOutput)

    def accGradParameters(self, input, gradOutput):
        if not self._param_slots:
            return
        if getattr(self, "_pgrads", None) is None:
            self._run_backward(input, gradOutput)
        for w, gname in self._param_slots:
            gw = self._pgrads.get(w)
            scale = self.scale_b if w == "bias" else self.scale_w
            if gw is not None and scale != 0:
                getattr(self, gname).add_(gw.to(getattr(self, gname).dtype), alpha=scale)
            reg = self.bRegularizer if w == "bias" else self.wRegularizer
            if reg is not None and scale != 0:
                reg.accRegularization(getattr(self, w), getattr(self, gname), scale)
        self._pgrads = None


class AbstractCriterion:
    """``DL/nn/abstractnn/AbstractCriterion.scala:50-138``."""

    SCALA_PACKAGE = "com.intel.analytics.bigdl.nn"

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        init = cls.__dict__.get("__init__")
        if init is not None and not getattr(init, "_bigdl_wrapped", False):
            cls.__init__ = _record_ctor(init)

    def __init__(self, size_average: bool = True):
        self.output = 0.0
        self.gradInput: Any = torch.empty(0)
        self.sizeAverage = size_average
        if not hasattr(self, "_ctor_args"):
            self._ctor_args = OrderedDict()

    def forward(self, input, target):
        numpy_out = isinstance(input, np.ndarray)
        input = to_torch(input)
        target = to_torch(target)
        out = self.updateOutput(input, target)
        if isinstance(out, torch.Tensor) and out.dtype != torch.float64:
            out = out.float()
        self.output = out
        if numpy_out:
            return float(out)
        return self.output

    def backward(self, input, target):
        numpy_out = isinstance(input, np.ndarray)
        input = to_torch(input)
        target = to_torch(target)
        self.gradInput = self.updateGradInput(input, target)
        if numpy_out:
            return _to_numpy(self.gradInput)
        return self.gradInput

    def updateOutput(self, input, target):
        raise NotImplementedError

    def updateGradInput(self, input, target):
        raise NotImplementedError

    def cloneCriterion(self):
        import copy
        return copy.deepcopy(self)

    @classmethod
    def scala_class_name(cls) -> str:
        return f"{cls.SCALA_PACKAGE}.{getattr(cls, 'SCALA_NAME', cls.__name__)}"

    def __repr__(self):
        return type(self).__name__


class AutogradCriterion(AbstractCriterion):
    """Criterion whose gradient is derived by AD from ``_loss(input, target)``."""

    def _loss(self, input, target):  # pragma: no cover
        raise NotImplementedError

    def updateOutput(self, input, target):
        with torch.no_grad():
            return self._loss(input, target)

    def updateGradInput(self, input, target):
        flat = flatten_activity(input)
        leaves = [t.detach().float().requires_grad_(True) if t.is_floating_point() else t for t in flat]
        xin, _ = unflatten_like(input, leaves)
        with torch.enable_grad():
            loss = self._loss(xin, target)
        targets = [l for l in leaves if l.requires_grad]
        grads = torch.autograd.grad(loss, targets, allow_unused=True)
        it = iter(grads)
        gi = []
        for l in leaves:
            if l.requires_grad:
                g = next(it)
                gi.append(torch.zeros_like(l) if g is None else g)
            else:
                gi.append(torch.zeros_like(l, dtype=torch.float32))
        out, _ = unflatten_like(input, gi)
        return out


class Activity:
    """Marker namespace (``DL/nn/abstractnn/Activity.scala``)."""

    @staticmethod
    def allocate(is_table: bool):
        return Table() if is_table else torch.empty(0)


class EmptyGradInput(Activity):
    """``gradInput`` placeholder of a module that never propagates a gradient to its input
    (``Activity.scala`` ``EmptyGradInput``): any use as a tensor raises, naming the module."""

    def __init__(self, module_name: str = ""):
        self.module_name = module_name

    def __getattr__(self, item):
        raise RuntimeError(f"{self.module_name or 'module'} does not compute a gradInput "
                           f"(EmptyGradInput.{item} accessed)")

    def __repr__(self):
        return f"EmptyGradInput({self.module_name})"
