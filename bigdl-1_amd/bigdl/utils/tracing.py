"""Per-iteration phase tracing for the training loops.

The reference times each synchronous-SGD iteration in named phases ("computing time", "aggregate
gradient time", "compute weight average", "send weights average" — ``DL/optim/DistriOptimizer.scala:
188-196``) and logs ``metrics.summary()``.  Here one :class:`StepTracer` per optimizer provides

* ``phase(name)`` — a context manager that, depending on the config, opens a **roctx range**
  (``bigdl.roctx``; visible in ``rocprofv3 --marker-trace`` timelines next to the kernels) and/or
  records a pair of **HIP events** on the current stream (``bigdl.metrics.deviceTimers``).  Events
  are resolved lazily: an iteration's phase times are read only once its last event has completed
  (``Event.query()``), so tracing adds no host↔device synchronisation to the hot loop;
* ``end_iteration(...)`` — closes the iteration, appends its resolved phases to the optimizer's
  :class:`~bigdl.optim.metrics.Metrics`, and writes one JSON line per iteration per rank to
  ``<bigdl.metrics.jsonPath>.rank<r>.jsonl`` (``bigdl.metrics.jsonPath``; off when empty);
* the **straggler monitor** (P5, ``DistriOptimizer.scala:246-278,421-449``): every
  ``bigdl.straggler.window`` iterations the ranks all-gather their per-iteration step times, the
  threshold is ``Util.kthLargest`` of that list at k = dropPercentage · window · world (the
  reference's formula), and ranks whose mean computing time (forward + backward) exceeds ``factor`` ×
  the lower median are logged
  as slow.  Synchronous RCCL collectives cannot drop a late rank's gradient the way the reference's
  thread pool cancels a late model replica (the reduce-scatter waits for every rank), so on MI355X
  the mechanism detects and reports stragglers rather than discarding their work.

When every switch is off ``phase`` returns a shared no-op context, so the default loop pays one
attribute lookup per phase.
"""
from __future__ import annotations

import contextlib
import ctypes
import json
import os
import time
from typing import Dict, List, Optional

import torch

from . import config
from .logger import get_logger

log = get_logger("bigdl.tracing")

_NULL = contextlib.nullcontext()
_roctx_lib = None
_roctx_tried = False


def _roctx():
    """The roctx marker API via ctypes.  ``librocprofiler-sdk-roctx`` first: that is the library
    rocprofv3 ``--marker-trace`` intercepts (the legacy ``libroctx64`` belongs to roctracer)."""
    global _roctx_lib, _roctx_tried
    if not _roctx_tried:
        _roctx_tried = True
        for name in ("librocprofiler-sdk-roctx.so.1", "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1",
                     "libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                _roctx_lib = lib
                break
            except OSError:
                continue
    return _roctx_lib


@contextlib.contextmanager
def roctx_range(name: str):
    lib = _roctx()
    if lib is None:
        yield
        return
    lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        lib.roctxRangePop()


def roctx_mark(name: str) -> None:
    lib = _roctx()
    if lib is not None:
        lib.roctxMarkA(name.encode())


class _Phase:
    __slots__ = ("tr", "name", "s", "t")

    def __init__(self, tr, name):
        self.tr, self.name = tr, name

    def __enter__(self):
        tr = self.tr
        if tr.roctx:
            lib = _roctx()
            if lib is not None:
                lib.roctxRangePushA(self.name.encode())
        if tr.device:
            self.s = torch.cuda.Event(enable_timing=True)
            self.s.record()
        else:
            self.t = time.perf_counter()
        return self

    def __exit__(self, *exc):
        tr = self.tr
        if tr.device:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            tr._cur.append((self.name, self.s, e))
        else:
            tr._cur_host[self.name] = tr._cur_host.get(self.name, 0.0) + time.perf_counter() - self.t
        if tr.roctx:
            lib = _roctx()
            if lib is not None:
                lib.roctxRangePop()
        return False


class StepTracer:
    def __init__(self, metrics, rank: int = 0, world: int = 1):
        self.metrics = metrics
        self.rank, self.world = rank, world
        self.roctx = bool(config.get_property("bigdl.roctx"))
        dev_timers = bool(config.get_property("bigdl.metrics.deviceTimers"))
        path = str(config.get_property("bigdl.metrics.jsonPath") or "")
        self.json_path = f"{path}.rank{rank}.jsonl" if path else None
        self.device = (dev_timers or bool(self.json_path)) and torch.cuda.is_available()
        self.host_timers = dev_timers or bool(self.json_path)
        self.enabled = self.roctx or self.device or self.host_timers
        self._cur: List = []          # (name, start, end) events of the open iteration
        self._cur_host: Dict[str, float] = {}
        self._pending: List = []      # closed iterations whose events are not resolved yet
        self._json = None
        self._steps = 0  # iterations closed by this tracer (train_step driven outside optimize())
        self.last_phases: Dict[str, float] = {}
        # straggler monitor
        self.window = max(1, int(config.get_property("bigdl.straggler.window")))
        self.factor = float(config.get_property("bigdl.straggler.factor"))
        self._times: List[float] = []
        self.threshold: Optional[float] = None
        self.slow_ranks: List[int] = []

    def phase(self, name: str):
        if not self.enabled:
            return _NULL
        if self.device and torch.cuda.is_current_stream_capturing():
            return _NULL  # a HIP-graph capture replays without host-side timing
        return _Phase(self, name)

    # -------------------------------------------------------------------------- iteration close
    def end_iteration(self, it: int, record: Dict):
        """Close iteration ``it``; ``record`` holds host-side facts (loss may be None if not yet
        read).  Returns the phase dict of the most recent iteration resolved so far."""
        self._steps += 1
        record = dict(record, step=self._steps)
        if self.device:
            marker = torch.cuda.Event()
            marker.record()
            self._pending.append((it, self._cur, dict(self._cur_host), record, marker))
        else:
            self._emit(it, dict(self._cur_host), record)
        self._cur, self._cur_host = [], {}
        self._drain(block=False)
        return self.last_phases

    def _drain(self, block: bool):
        while self._pending:
            it, evs, host, record, marker = self._pending[0]
            if not block and not marker.query():
                break
            if block:
                marker.synchronize()
            self._pending.pop(0)
            ph = dict(host)
            for name, s, e in evs:
                ph[name] = ph.get(name, 0.0) + s.elapsed_time(e) / 1000.0
            self._emit(it, ph, record)

    def _emit(self, it, ph, record):
        self.last_phases = ph
        for k, v in ph.items():
            self.metrics.add(k, v)
        if self.json_path is not None:
            if self._json is None:
                os.makedirs(os.path.dirname(os.path.abspath(self.json_path)), exist_ok=True)
                self._json = open(self.json_path, "a", buffering=1)
            line = {"iteration": it, "rank": self.rank, "world": self.world, "time": time.time()}
            line.update({k: v for k, v in record.items() if v is not None})
            line["phases_s"] = {k: round(v, 6) for k, v in ph.items()}
            self._json.write(json.dumps(line) + "\n")

    def flush(self):
        self._drain(block=True)
        if self._json is not None:
            self._json.flush()

    def close(self):
        self.flush()
        if self._json is not None:
            self._json.close()
            self._json = None

    # -------------------------------------------------------------------------- straggler monitor
    def observe_step_time(self, it: int, seconds: float, drop_percentage: float, allgather=None):
        """Collect this rank's step time; every ``window`` iterations all-gather the window's times
        of every rank (``allgather(list_of_floats) -> list of per-rank lists``), compute the
        reference's kthLargest threshold and log ranks whose mean is > factor × the median."""
        self._times.append(float(seconds))
        if len(self._times) < self.window:
            return None
        mine, self._times = self._times, []
        per_rank = allgather(mine) if (allgather is not None and self.world > 1) else [mine]
        flat = [t for r in per_rank for t in r]
        k = int(drop_percentage * self.window * len(per_rank))
        from .util import kthLargest
        if k > 0:
            us = [int(t * 1e6) for t in flat]
            self.threshold = kthLargest(us, 0, len(us) - 1, min(k, len(us))) / 1e6
        means = [sum(r) / max(1, len(r)) for r in per_rank]
        med = sorted(means)[(len(means) - 1) // 2]  # lower median: with two ranks, the faster one
        self.slow_ranks = [i for i, m in enumerate(means) if med > 0 and m > self.factor * med]
        self.metrics.set("straggler threshold", self.threshold or 0.0)
        self.metrics.set("slow ranks", len(self.slow_ranks))
        if self.slow_ranks and self.rank == 0:
            log.warning(f"iteration {it}: slow ranks {self.slow_ranks} (mean step "
                        f"{[round(means[i], 4) for i in self.slow_ranks]} s vs median {med:.4f} s"
                        + (f", drop threshold {self.threshold:.4f} s" if self.threshold else "") + ")")
        return self.slow_ranks


def allgather_floats(values: List[float]) -> List[List[float]]:
    """All-gather a short list of floats from every rank (one small collective on the default
    group; a CPU tensor under gloo, a device tensor under RCCL)."""
    import torch.distributed as dist
    dev = torch.device("cuda", torch.cuda.current_device()) if (
        torch.cuda.is_available() and dist.get_backend() == "nccl") else torch.device("cpu")
    t = torch.tensor(values, dtype=torch.float64, device=dev)
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [o.cpu().tolist() for o in out]


__all__ = ["StepTracer", "roctx_range", "roctx_mark", "allgather_floats"]
