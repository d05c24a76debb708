"""Logging setup (``DL/utils/LoggerFilter.scala:34-134``).

``redirect_logs()`` routes framework INFO logs to ``bigdl.log`` (configurable with
``bigdl.utils.LoggerFilter.logFile``) and keeps WARN+ on the console; the per-iteration
training line keeps the reference format (``DistriOptimizer.scala:411-416``) because tools grep it.
"""
from __future__ import annotations

import logging
import os
import sys

from . import config

_configured = False


def get_logger(name: str = "bigdl") -> logging.Logger:
    global _configured
    if not _configured:
        _configured = True
        root = logging.getLogger("bigdl")
        if not root.handlers:
            h = logging.StreamHandler(sys.stdout)
            h.setFormatter(logging.Formatter("%(asctime)s %(levelname)s %(name)s: %(message)s"))
            root.addHandler(h)
        root.setLevel(logging.INFO if os.environ.get("RANK", "0") == "0" else logging.WARNING)
        root.propagate = False
    return logging.getLogger(name)


def redirect_logs(log_file: str | None = None):
    if config.get_property("bigdl.utils.LoggerFilter.disable"):
        return
    log_file = log_file or config.get_property("bigdl.utils.LoggerFilter.logFile")
    root = get_logger()
    fh = logging.FileHandler(log_file)
    fh.setLevel(logging.INFO)
    fh.setFormatter(logging.Formatter("%(asctime)s %(levelname)s %(name)s: %(message)s"))
    root.addHandler(fh)


def iteration_line(epoch, processed, total, iteration, wall_clock_s, batch, seconds, loss, extra="") -> str:
    """The canonical per-iteration line (``DistriOptimizer.scala:411-416``)."""
    thr = batch / seconds if seconds > 0 else float("inf")
    return (f"[Epoch {epoch} {processed}/{total}][Iteration {iteration}][Wall Clock {wall_clock_s:.3f}s] "
            f"Trained {batch} records in {seconds:.4f} seconds. Throughput is {thr:.2f} records/second. "
            f"Loss is {loss:.6f}. {extra}").rstrip()
