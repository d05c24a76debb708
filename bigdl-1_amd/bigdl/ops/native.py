"""ctypes bindings to ``libbigdl_kernels.so`` (hand-written HIP/CDNA4 kernels, gfx950).

The library is built in-tree by ``bigdl/ops/build.py`` (``hipcc --offload-arch=gfx950``) into
``bigdl/ops/lib/``.  Kernels take raw device pointers plus the current HIP stream of the torch
caching allocator, so they interleave with torch ops and are capturable in HIP graphs.

Each Python wrapper validates shapes/strides on the host BEFORE launching (a mis-shaped launch
must never reach the GPU), and returns ``NotImplemented`` for a configuration the kernel does not
cover so the dispatcher can fall back explicitly.
"""
from __future__ import annotations

import ctypes
import logging
import os
from typing import Optional

import torch

from ..utils import config

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libbigdl_kernels.so")

_lib: Optional[ctypes.CDLL] = None
_load_error: Optional[str] = None
_ops_available: set = set()


def _load():
    global _lib, _load_error
    if _lib is not None or _load_error is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        _load_error = f"{LIB_PATH} not built (run python -m bigdl.ops.build)"
        return None
    try:
        _lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    except OSError as e:  # pragma: no cover - depends on box
        _load_error = str(e)
        return None
    _declare(_lib)
    _push_deterministic(config.get_property("bigdl.deterministic"))
    return _lib


def _push_deterministic(on) -> None:
    if _lib is not None:
        _lib.bigdl_set_deterministic(1 if on else 0)


config.on_change("bigdl.deterministic", _push_deterministic)


def _declare(lib):
    # every exported symbol returns int (hipError_t) and takes void*/int64/float args
    names = []
    try:
        lib.bigdl_op_name.restype = ctypes.c_char_p
        n = lib.bigdl_num_ops()
        for i in range(n):
            names.append(lib.bigdl_op_name(i).decode())
    except AttributeError:
        pass
    _ops_available.update(names)


def status() -> dict:
    _load()
    return {"library": LIB_PATH, "loaded": _lib is not None, "error": _load_error,
            "ops": sorted(_ops_available)}


class _TracedLib:
    """``BIGDL_TRACE_NATIVE=1``: print every native entry point before it runs (stderr, flushed);
    ``=2``: also synchronize after it and print ``ok`` — a GPU fault is then attributed to the last
    name printed without its ``ok`` (fault triage without a debugger)."""

    def __init__(self, l, sync):
        self._l, self._sync = l, sync

    def __getattr__(self, name):
        f = getattr(self._l, name)
        if not callable(f) or not name.startswith("bigdl_"):
            return f
        import sys

        def call(*a):
            print(f"[native] {name}", file=sys.stderr, flush=True)
            r = f(*a)
            if self._sync and torch.cuda.is_available():
                torch.cuda.synchronize()
                print(f"[native] {name} ok rc={r}", file=sys.stderr, flush=True)
            return r
        return call


_TRACE = os.environ.get("BIGDL_TRACE_NATIVE", "")


def lib():
    l = _load()
    if l is None and torch.cuda.is_available() and config.get_property("bigdl.native.require"):
        raise RuntimeError(f"bigdl native HIP kernels are required on a GPU but not loaded: {_load_error}")
    if _TRACE and l is not None:
        return _TracedLib(l, _TRACE == "2")
    return l


# asked on every op dispatch: cached, refreshed by config.set_property listeners
_ENABLED = [bool(config.get_property("bigdl.native.enable"))]
config.on_change("bigdl.native.enable", lambda v: _ENABLED.__setitem__(0, bool(v)))


def has(opname: str) -> bool:
    if not _ENABLED[0]:
        return False
    l = _load()
    if l is None:
        if torch.cuda.is_available() and config.get_property("bigdl.native.require"):
            raise RuntimeError(f"bigdl native HIP kernels are required on a GPU but not loaded: {_load_error}")
        return False
    return opname in _PY_OPS


# Python-level op wrappers registered below (populated by kernels.py once written)
_PY_OPS: dict = {}


def register(name):
    def deco(fn):
        _PY_OPS[name] = fn
        globals()[name] = fn
        return fn
    return deco


# ---------------------------------------------------------------------------- fallback accounting
# Every device-tensor call of a dispatched op that does NOT reach a HIP kernel is counted here and
# warned about once per (op, reason, signature); ``bigdl.native.strict`` turns it into an error.
# Tests assert zero fallbacks over the flagship training steps (tests/test_no_fallback.py).
_FALLBACKS: dict = {}
_log = logging.getLogger("bigdl.ops")


def _sig(args) -> str:
    parts = []
    for a in args:
        if isinstance(a, torch.Tensor):
            parts.append(f"{str(a.dtype).replace('torch.', '')}{list(a.shape)}")
            if len(parts) == 3:
                break
    return ",".join(parts)


def note_fallback(opname: str, reason: str, args=()) -> None:
    key = (opname, reason, _sig(args))
    n = _FALLBACKS.get(key, 0)
    _FALLBACKS[key] = n + 1
    if n == 0:
        msg = f"bigdl op {opname} fell back to the torch reference on a device tensor ({reason}: {key[2]})"
        if config.get_property("bigdl.native.strict"):
            raise RuntimeError(msg)
        _log.warning(msg)


def fallback_counts() -> dict:
    return dict(_FALLBACKS)


def reset_fallbacks() -> None:
    _FALLBACKS.clear()


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_ptr() -> int:
    """The current HIP stream of the current device (raw handle; called once per kernel launch, so it
    skips the torch.cuda.Stream object that ``current_stream()`` builds)."""
    if _RAW_STREAM is not None:
        return _RAW_STREAM(torch._C._cuda_getDevice())
    return torch.cuda.current_stream().cuda_stream


def ptr(t: Optional[torch.Tensor]) -> ctypes.c_void_p:
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def check(rc: int, what: str):
    if rc != 0:
        raise RuntimeError(f"bigdl HIP kernel {what} failed with hipError {rc}")


from . import native_ops  # noqa: E402,F401  (registers wrappers)
