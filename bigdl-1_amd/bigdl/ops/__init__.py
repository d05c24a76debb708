"""Hot-op library.

Every op has a plain-torch reference (``reference.py``: CPU path + test oracle) and, for device
tensors, a hand-written HIP/CDNA4 kernel in ``csrc/`` (``native.py`` binds them).  Selection is
by tensor device only — there is no backend registry: a CUDA(HIP) tensor goes to the native
kernel, and if the compiled library is missing on a GPU box the op raises (set
``BIGDL_NATIVE_REQUIRE=0`` to allow the reference path for debugging).
"""
from __future__ import annotations

from . import reference
from .dispatch import *  # noqa: F401,F403
from .dispatch import native_status, native_has, __all__ as _dispatch_all  # noqa: F401
from .dispatch import fallback_counts, reset_fallbacks  # noqa: F401
from . import native_ops  # noqa: F401  (fused entry points beyond the dispatch table)
from . import native  # noqa: F401

__all__ = list(_dispatch_all) + ["reference", "native_status", "native_has", "native_ops", "native",
                                 "fallback_counts", "reset_fallbacks"]
