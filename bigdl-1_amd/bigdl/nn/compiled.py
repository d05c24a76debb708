"""Two-phase execution: plan a model once for a fixed input shape, then run it repeatedly.

The reference compiles its MKL-DNN graphs in a separate phase (``nn/mkldnn/DnnGraph.scala``
``compile(phase)`` → ``initFwdPrimitives`` / ``initBwdPrimitives``: input formats fixed, memory
descriptors chosen, reorders inserted, buffers allocated) before the first iteration.  Here the
same split is:

* **plan** (:func:`plan`): one forward at the target shape with every leaf module instrumented —
  per-layer input/output shapes, dtypes and memory layout (NCHW vs the NHWC device layout the
  conv path switches to: the "reorder" points), the activation buffers (by storage, so views are
  one buffer), their live ranges in execution order, the peak live bytes and a first-fit offset
  assignment of every buffer into one workspace (what an arena allocator for this shape needs);
* **select kernels** (:func:`autotune`, ``bigdl.compile.autotune``): every distinct conv geometry of
  the planned forward is timed under each implicit-GEMM tile candidate and the winner pinned;
* **execute** (:class:`CompiledModule`): on a GPU and in the inference phase the forward is
  captured once into a HIP graph with a static input buffer — every kernel and every workspace
  allocation of the forward is then fixed (the graph's private memory pool, reserved up front as one
  slab of the plan's first-fit arena size), and each call is a copy-in plus one graph replay, with
  no per-layer host dispatch.  Models whose forward syncs with
  the host (data-dependent shapes, ``.item()``) cannot be captured and run eagerly with a warning.

``compile(model, example, phase)`` does both.
"""
from __future__ import annotations

import logging
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch

from ..utils.table import Table

_log = logging.getLogger("bigdl.nn.compiled")


def _leaves(m) -> List:
    from ..utils.intermediate import IRGraph
    if isinstance(m, IRGraph):  # a lowered model: plan the device graph it executes
        return _leaves(m._need())
    subs = getattr(m, "modules", None)
    if isinstance(subs, list) and subs and all(hasattr(s, "updateOutput") for s in subs):
        out = []
        for s in subs:
            out.extend(_leaves(s))
        return out
    return [m]


def _tensors(a) -> List[torch.Tensor]:
    if isinstance(a, torch.Tensor):
        return [a]
    if isinstance(a, Table):
        return [t for v in a.values() for t in _tensors(v)]
    if isinstance(a, (list, tuple)):
        return [t for v in a for t in _tensors(v)]
    return []


def _layout(t: torch.Tensor) -> str:
    if t.dim() == 4:
        if t.is_contiguous():
            return "NCHW"
        if t.is_contiguous(memory_format=torch.channels_last):
            return "NHWC"
    return "dense" if t.is_contiguous() else "strided"


@dataclass
class LayerRecord:
    index: int
    name: str
    kind: str
    in_shapes: List[tuple]
    out_shapes: List[tuple]
    out_dtype: str
    in_layout: str
    out_layout: str
    out_bytes: int


@dataclass
class Buffer:
    key: int
    nbytes: int
    first: int
    last: int
    offset: int = -1


@dataclass
class Plan:
    phase: str
    input_shape: tuple
    layers: List[LayerRecord] = field(default_factory=list)
    buffers: List[Buffer] = field(default_factory=list)
    reorders: List[int] = field(default_factory=list)   # layer indices whose output layout differs from their input's
    peak_bytes: int = 0
    arena_bytes: int = 0
    total_bytes: int = 0

    def summary(self) -> str:
        mb = 1 / 2 ** 20
        lines = [f"plan ({self.phase}) input {self.input_shape}: {len(self.layers)} layers, "
                 f"{len(self.buffers)} activation buffers, total {self.total_bytes * mb:.1f} MiB, "
                 f"peak live {self.peak_bytes * mb:.1f} MiB, arena {self.arena_bytes * mb:.1f} MiB, "
                 f"{len(self.reorders)} layout changes"]
        for r in self.layers:
            lines.append(f"  {r.index:4d} {r.kind:28s} {str(r.in_shapes[:1]):24s} -> {str(r.out_shapes[:1]):24s} "
                         f"{r.in_layout}->{r.out_layout} {r.out_dtype}")
        return "\n".join(lines)


def _assign_offsets(bufs: List[Buffer], align: int = 256) -> int:
    """First-fit placement, largest first, of buffers whose live ranges overlap in time."""
    placed: List[Buffer] = []
    top = 0
    for b in sorted(bufs, key=lambda x: (-x.nbytes, x.first)):
        size = (b.nbytes + align - 1) // align * align
        busy = sorted((p.offset, p.offset + (p.nbytes + align - 1) // align * align) for p in placed
                      if not (p.last < b.first or b.last < p.first))
        off = 0
        for lo, hi in busy:
            if off + size <= lo:
                break
            off = max(off, hi)
        b.offset = off
        placed.append(b)
        top = max(top, off + size)
    return top


def plan(model, example, phase: str = "inference") -> Plan:
    """Run one forward of ``model`` on ``example`` with instrumented leaf modules and build the
    shape / layout / workspace plan (``phase``: "inference" frees a buffer after its last use,
    "training" keeps every activation for the backward)."""
    if phase not in ("inference", "training"):
        raise ValueError(phase)
    was_training = model.isTraining()
    if phase == "inference" and was_training:
        model.evaluate()  # first: an IRGraph re-folds its device graph on the switch
    leaves = _leaves(model)
    records: List[LayerRecord] = []
    uses: Dict[int, List[int]] = {}
    sizes: Dict[int, int] = {}
    first: Dict[int, int] = {}
    in_keys = set()

    def key(t):
        return t.untyped_storage().data_ptr()

    for t in _tensors(example):
        in_keys.add(key(t))

    def wrap(m):
        orig = m.updateOutput

        def rec(inp):
            out = orig(inp)
            i = len(records)
            ins, outs = _tensors(inp), _tensors(out)
            for t in ins + outs:
                k = key(t)
                uses.setdefault(k, []).append(i)
                sizes[k] = max(sizes.get(k, 0), t.untyped_storage().nbytes())
                first.setdefault(k, i)
            il = _layout(ins[0]) if ins else "-"
            ol = _layout(outs[0]) if outs else "-"
            records.append(LayerRecord(i, getattr(m, "getName", lambda: type(m).__name__)(), type(m).__name__,
                                       [tuple(t.shape) for t in ins], [tuple(t.shape) for t in outs],
                                       str(outs[0].dtype).replace("torch.", "") if outs else "-", il, ol,
                                       sum(t.untyped_storage().nbytes() for t in outs)))
            return out
        m.updateOutput = rec

    for m in leaves:
        wrap(m)
    try:
        with torch.no_grad():
            out = model.forward(example)
    finally:
        for m in leaves:
            m.__dict__.pop("updateOutput", None)
        if was_training:
            model.training()
    n = len(records)
    out_keys = {key(t) for t in _tensors(out)}
    bufs = []
    for k, idx in uses.items():
        if k in in_keys:
            continue  # the caller's input, not a workspace
        last = n if (k in out_keys or phase == "training") else max(idx)
        bufs.append(Buffer(k, sizes[k], first[k], last))
    p = Plan(phase, tuple(_tensors(example)[0].shape) if _tensors(example) else (), records, bufs)
    p.reorders = [r.index for r in records if r.in_layout in ("NCHW", "NHWC") and r.out_layout in ("NCHW", "NHWC")
                  and r.in_layout != r.out_layout]
    p.total_bytes = sum(b.nbytes for b in bufs)
    live = [0] * (n + 1)
    for b in bufs:
        for i in range(b.first, min(b.last, n) + 1):
            live[i] += b.nbytes
    p.peak_bytes = max(live) if live else 0
    p.arena_bytes = _assign_offsets(bufs)
    return p


#: tile candidates (BN output channels, BK k-tile depth, BM output pixels) of the implicit-GEMM
#: forward; (0, 0, 0) is the launcher's shape heuristic.  BK = 1 is the 8-wave 32x32x16 / LDS-DMA
#: family (ops/csrc/conv_mfma32.hip), which wins on the deep reductions (C ≥ 256 3×3, C ≥ 1024 1×1).
TILE_CANDIDATES = ((0, 0, 0), (64, 32, 128), (64, 64, 128), (128, 32, 128), (128, 64, 128), (64, 64, 256),
                   (128, 64, 256), (128, 1, 128), (64, 1, 256), (128, 1, 256), (256, 1, 256))

#: weight-gradient candidates (target blocks of the pixel split, k-tile pixel depth); 0 = heuristic
WGRAD_CANDIDATES = ((0, 0), (0, 32), (0, 64), (256, 0), (768, 0), (1024, 0), (256, 32), (768, 64))
#: a wider split-count grid, on by default (BIGDL_WGRAD_EXTRA=0 drops it): ResNet-50 step 20.77-20.86
#: vs 20.86-20.90 ms, 3 interleaved repeats (profiles/r5_wgrad_candidates_ab.txt)
WGRAD_EXTRA = ((512, 32), (512, 64), (1536, 0), (2048, 32), (2048, 0))


#: fp32 direct-operand conv (ops/csrc/conv_x3.hip) tiles (BM, BN | wave-layout bits): (0, 0) = the
#: launcher's heuristic; bn | 256 = waves over pixels only, | 512 = 2-deep ring (2-3 blocks per CU)
X3_CANDIDATES = ((0, 0), (256, 128), (256, 64), (128, 128), (256, 128 | 256), (256, 64 | 256), (128, 128 | 256),
                 (128, 128 | 512), (128, 128 | 768), (128, 64 | 768))


#: fp32 weight-gradient (conv_wgrad.hip F32): split-M block targets (0 = heuristic ≈512 blocks)
WGRAD32_CANDIDATES = ((0,), (-256,), (-1024,), (-2048,), (-4096,))


def _candidates(key):
    if isinstance(key, tuple) and key and key[0] == "wg":
        import os
        return WGRAD_CANDIDATES + (() if os.environ.get("BIGDL_WGRAD_EXTRA") == "0" else WGRAD_EXTRA)
    if isinstance(key, tuple) and key and key[0] == "wg32":
        return WGRAD32_CANDIDATES
    if isinstance(key, tuple) and key and key[0] == "x3":
        return X3_CANDIDATES
    return TILE_CANDIDATES


def _time_candidates(key, fn, iters, lib):
    import torch
    times = {}
    for cand in _candidates(key):
        if len(cand) == 3 and lib.bigdl_conv_tile_ok(*cand) != 0:
            continue
        try:
            fn(cand)  # warm-up (and validity: an unsupported combination raises)
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record()
            for _ in range(iters):
                fn(cand)
            t1.record()
            t1.synchronize()
            times[cand] = t0.elapsed_time(t1) / iters
        except RuntimeError:
            continue
    return times


def select_kernels(records, iters: int = 5, min_gain: float = 0.03) -> Dict[tuple, tuple]:
    """Time every candidate of every distinct recorded launch geometry (``records`` = the
    (key, relaunch-with-tile) pairs a recorded pass left in ``native_ops._TILE["record"]``) and pin
    the fastest one when it beats the launcher's heuristic by more than ``min_gain``.  Forward /
    backward-data launches (conv geometry keys) take :data:`TILE_CANDIDATES`, weight-gradient
    launches (``("wg", ...)`` keys) :data:`WGRAD_CANDIDATES`."""
    from ..ops import native_ops as NO
    lib = NO._lib()
    table = NO._TILE["table"]
    chosen = {}
    seen = {}
    for key, fn in (records.items() if isinstance(records, dict) else records):
        seen.setdefault(key, fn)
    NO._TILE["retiming"] = True
    try:
        for key, fn in seen.items():
            _select_one(key, fn, iters, min_gain, lib, table, chosen)
    finally:
        NO._TILE["retiming"] = False
    return chosen


def _select_one(key, fn, iters, min_gain, lib, table, chosen):
    if key in table:
        # already pinned by an earlier compile in this process (a predictor per batch shape, a serving
        # replica, a second optimizer): keep it instead of re-timing (clear the table to re-select)
        chosen[key] = table[key]
        return
    times = _time_candidates(key, fn, iters, lib)
    base = times.get(_candidates(key)[0])
    if base is None or not times:
        return
    best = min(times, key=times.get)
    if best != _candidates(key)[0] and times[best] < base * (1.0 - min_gain):
        table[key] = best
        chosen[key] = best
        _log.info("kernel %s: %s %.1f us (heuristic %.1f us)", key, best, times[best] * 1e3, base * 1e3)


def autotune_training_step(step_fn, iters: int = 5, min_gain: float = 0.03) -> Dict[tuple, tuple]:
    """The training compile phase (the reference compiles ``TrainingPhase`` per replica,
    ``DL/optim/DistriOptimizer.scala:600-609``, ``DL/nn/mkldnn/DnnBase.scala:321-366``): run one real
    training iteration ``step_fn()`` with launch recording on — forward (with its BN-statistics
    epilogues), backward-data and weight-gradient convolutions exactly as training issues them —
    then, once that iteration has finished (its collectives included), re-time each recorded launch
    under every candidate and pin the winners per geometry.  Re-running a launch only rewrites that
    iteration's outputs (activations, partials) or adds into gradient buffers the next iteration
    zeroes, so the optimizer state is untouched.  Returns ``(step result, {key: choice})``."""
    import torch
    from ..ops import native_ops as NO
    rec = NO._TILE["record"] = {}  # geometry → first launch (dedup while recording)
    try:
        out = step_fn()
    finally:
        NO._TILE["record"] = None
    torch.cuda.synchronize()
    chosen = select_kernels(rec, iters, min_gain)
    rec.clear()
    torch.cuda.synchronize()
    return out, chosen


def autotune(model, example, iters: int = 5, min_gain: float = 0.03) -> Dict[tuple, tuple]:
    """Kernel selection for the planned shape (the reference's compile step creates its MKL-DNN
    primitives per layer, ``DL/nn/mkldnn/DnnBase.scala:321-366``): run one forward recording every
    implicit-GEMM conv launch, time each distinct conv geometry under every tile candidate
    (HIP events, ``iters`` launches after a warm-up) and pin the fastest one for that geometry when
    it beats the shape heuristic by more than ``min_gain``.  The choice is process-wide, keyed by
    geometry (``ops.native_ops.conv_tile_table()``), like a cuDNN benchmark-mode cache.  Returns
    {geometry: (BN, BK, BM)} of the pinned entries (empty off the GPU)."""
    from ..ops import native_ops as NO
    ex = _tensors(example)
    if not ex or not ex[0].is_cuda:
        return {}
    was_training = model.isTraining() if hasattr(model, "isTraining") else False
    model.evaluate()
    rec = NO._TILE["record"] = {}
    try:
        with torch.no_grad():
            model.forward(example)
    finally:
        NO._TILE["record"] = None
        if was_training:
            model.training()
    return select_kernels(rec, iters, min_gain)


class CompiledModule:
    """``model`` planned for ``example``'s shape; in the inference phase on a GPU the forward is a
    captured HIP graph (``graph=False`` forces eager execution).  The returned output tensor is the
    graph's static output buffer: it is overwritten by the next call (clone it to keep it)."""

    def __init__(self, model, example, phase: str = "inference", graph: Optional[bool] = None, warmup: int = 2,
                 tune: Optional[bool] = None, lower: Optional[bool] = None):
        self.source, self.phase = model, phase
        # inference: lower through the IR first (BN folded into the convs / Linears, ReLU and the
        # residual sum in the conv epilogues) — the reference's predictors always convert
        # (LocalPredictor.scala:66, Predictor.scala:131,165 → ConversionUtils.convert)
        self.lowered = False
        if phase == "inference":
            model = _lower(model, lower)
            self.lowered = model is not self.source
        self.model = model
        self.plan = plan(model, example, phase)
        ex = _tensors(example)
        self.graph = None
        self.tiles = {}
        if tune is None:
            from ..utils import config
            tune = bool(config.get_property("bigdl.compile.autotune"))
        if tune and phase == "inference" and bool(ex) and ex[0].is_cuda:
            self.tiles = autotune(model, example)
        want = graph if graph is not None else (phase == "inference" and bool(ex) and ex[0].is_cuda)
        if want and isinstance(example, torch.Tensor) and example.is_cuda:
            try:
                self._capture(example, warmup)
            except Exception as e:  # noqa: BLE001 - host-synchronising forward: stay eager
                _log.warning("HIP graph capture of %s failed (%s); running eagerly", type(model).__name__, e)
                self.graph = None

    def _capture(self, example, warmup):
        m = self.model
        m.evaluate()
        self.static_in = example.detach().clone()
        side = torch.cuda.Stream(device=example.device)
        side.wait_stream(torch.cuda.current_stream(example.device))
        with torch.cuda.stream(side), torch.no_grad():
            for _ in range(max(1, warmup)):
                m.forward(self.static_in)
        torch.cuda.current_stream(example.device).wait_stream(side)
        # the planned workspace: the graph's private pool is reserved up front as ONE segment of
        # the first-fit arena size (plan.arena_bytes, plus kernel-side temporaries the leaf-level
        # plan does not see), so the captured forward's activations are carved from one slab —
        # the arena the plan laid out — rather than grown segment by segment during capture
        pool = torch.cuda.graph_pool_handle()
        self.arena_reserved = 0
        if self.plan.arena_bytes > 0:
            g0 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g0, pool=pool, capture_error_mode="thread_local"):
                slab = torch.empty(int(self.plan.arena_bytes * 1.25) + (1 << 20), dtype=torch.uint8,
                                   device=example.device)
                slab[:1].zero_()  # (a capture with no kernel at all is reported as an empty graph)
                self.arena_reserved = slab.numel()
                del slab
            del g0
        g = torch.cuda.CUDAGraph()
        with torch.no_grad(), torch.cuda.graph(g, pool=pool, capture_error_mode="thread_local"):
            self.static_out = m.forward(self.static_in)
        self.graph = g

    @property
    def captured(self) -> bool:
        return self.graph is not None

    def forward(self, x):
        if self.graph is None:
            if self.phase == "inference":
                self.model.evaluate()
                with torch.no_grad():
                    return self.model.forward(x)
            return self.model.forward(x)
        if tuple(x.shape) != tuple(self.static_in.shape):
            raise ValueError(f"compiled for input {tuple(self.static_in.shape)}, got {tuple(x.shape)}")
        self.static_in.copy_(x)
        self.graph.replay()
        return self.static_out

    __call__ = forward


def _model_device(model):
    for p in (model.parameters() or ([], []))[0]:
        return p.device
    return torch.device("cpu")


def _lower(model, lower: Optional[bool]):
    """The IR-lowered inference form of ``model`` (``utils/intermediate.ConversionUtils.convert``), on
    the model's device, or ``model`` itself when lowering is off (``bigdl.compile.lower``) or the model
    cannot be expressed in the IR."""
    from ..utils import config
    if lower is None:
        lower = bool(config.get_property("bigdl.compile.lower"))
    if not lower:
        return model
    from ..utils.intermediate import ConversionUtils, IRGraph
    if isinstance(model, IRGraph):
        return model
    was_training = model.isTraining() if hasattr(model, "isTraining") else False
    was_fused = bool(getattr(model, "_fused", False))
    try:
        model.evaluate()
        ir = ConversionUtils.convert(model)
        dev = _model_device(model)
        if dev.type == "cuda":
            ir.to(dev)
        ir.evaluate()
    except Exception as e:  # noqa: BLE001 - a layer the IR does not cover: compile the model as is
        _log.warning("IR lowering of %s failed (%s); compiling it unlowered", type(model).__name__, e)
        return model
    finally:
        if was_training:
            model.training()
        if was_fused and _model_device(model).type == "cuda":
            from .fusion import fuse, unfuse
            unfuse(model)
            fuse(model)  # the conversion cleared the source's execution-fusion flags: restore them
    return ir


def compile(model, example, phase: str = "inference", graph: Optional[bool] = None,  # noqa: A001
            tune: Optional[bool] = None, lower: Optional[bool] = None) -> CompiledModule:
    """Plan ``model`` for ``example``'s shape, select conv kernels (``autotune``) and return the
    executor (see module docstring).  In the inference phase the model is first lowered through the
    IR (``lower``; default ``bigdl.compile.lower``): BN folding and conv+sum+ReLU epilogues, then
    kernel selection and a HIP graph of the lowered forward.  The lowered graph holds folded copies
    of the weights taken now: compile again after the weights change."""
    # one compilation at a time per process: kernel selection swaps the process-wide tile table's
    # record / retiming state and graph capture must not interleave with another thread's launches
    # (PredictionService replicas compile lazily inside concurrent request threads)
    with _COMPILE_LOCK:
        return CompiledModule(model, example, phase, graph, tune=tune, lower=lower)


_COMPILE_LOCK = __import__("threading").RLock()


__all__ = ["plan", "autotune", "compile", "CompiledModule", "Plan", "LayerRecord", "Buffer", "TILE_CANDIDATES",
           "WGRAD_CANDIDATES", "select_kernels", "autotune_training_step"]
