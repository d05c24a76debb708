"""Named phase timers (``DL/optim/Metrics.scala:31-123``).

The reference accumulates "get weights", "computing time", "aggregate gradient time", "put
gradient", "compute weight", "send weights" per iteration (``DistriOptimizer.scala:188-196``).
Device phases are timed with HIP events on the stream that runs them (no host sync in the hot
loop); ``summary()`` resolves them lazily.
"""
from __future__ import annotations

import time
from collections import OrderedDict, defaultdict

import torch


class Metrics:
    def __init__(self):
        self._host = defaultdict(float)
        self._events = defaultdict(list)
        self._counts = defaultdict(int)

    def set(self, name, value):
        self._host[name] = float(value)
        return self

    def add(self, name, value):
        self._host[name] += float(value)
        self._counts[name] += 1
        return self

    def get(self, name):
        return self._host.get(name, 0.0)

    def timer(self, name):
        m = self

        class _T:
            def __enter__(self_):
                self_.t = time.perf_counter()

            def __exit__(self_, *a):
                m.add(name, time.perf_counter() - self_.t)
        return _T()

    def device_timer(self, name, stream=None):
        """Record start/end HIP events around a device phase."""
        m = self

        class _E:
            def __enter__(self_):
                if torch.cuda.is_available():
                    self_.s = torch.cuda.Event(enable_timing=True)
                    self_.e = torch.cuda.Event(enable_timing=True)
                    self_.s.record(stream)
                else:
                    self_.t = time.perf_counter()

            def __exit__(self_, *a):
                if torch.cuda.is_available():
                    self_.e.record(stream)
                    m._events[name].append((self_.s, self_.e))
                else:
                    m.add(name, time.perf_counter() - self_.t)
        return _E()

    def resolve(self):
        for name, evs in self._events.items():
            for s, e in evs:
                e.synchronize()
                self._host[name] += s.elapsed_time(e) / 1000.0
                self._counts[name] += 1
        self._events.clear()

    def summary(self, unit="s", scale=1.0):
        self.resolve()
        out = OrderedDict()
        for k, v in self._host.items():
            out[k] = v * scale
        return "========== Metrics Summary ==========\n" + "\n".join(
            f"{k} : {v} {unit}" for k, v in out.items()) + "\n====================================="

    def reset(self):
        self._host.clear()
        self._events.clear()
        self._counts.clear()
