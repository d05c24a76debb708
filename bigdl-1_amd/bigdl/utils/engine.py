"""Global engine: topology, device, precision policy and process group.

Reference: ``DL/utils/Engine.scala:41-600`` (``init`` 106-119, ``coreNumber/nodeNumber``
279-320, ``initThreadPool`` 349-380).  BigDL discovers executors×cores from a SparkConf and
runs one model replica per core.  Here the unit of parallelism is one process per GPU:
``RANK/WORLD_SIZE/LOCAL_RANK/MASTER_ADDR`` come from the launcher (``torch.distributed.run`` or
``bigdl.parallel.launcher``), each rank owns ``cuda:LOCAL_RANK`` and joins an RCCL process group
(backend ``nccl`` is RCCL on ROCm) — or ``gloo`` when no GPU is present, which is how the
distributed paths are tested on CPU.
"""
from __future__ import annotations

import os
import threading
from concurrent.futures import ThreadPoolExecutor

import torch

from . import config
from .logger import get_logger

log = get_logger("bigdl.engine")


class _EngineState:
    def __init__(self):
        self.inited = False
        self.node_number = 1
        self.core_number = 1
        self.rank = 0
        self.world_size = 1
        self.local_rank = 0
        self.device = torch.device("cpu")
        self.compute_dtype = torch.float32
        self.process_group_owned = False
        self.default_pool: ThreadPoolExecutor | None = None
        self.lock = threading.Lock()


_S = _EngineState()

_DTYPES = {"fp32": torch.float32, "float": torch.float32, "float32": torch.float32,
           "bf16": torch.bfloat16, "bfloat16": torch.bfloat16,
           "fp16": torch.float16, "half": torch.float16}


class Engine:
    """Static facade mirroring ``object Engine``."""

    @staticmethod
    def init(node_number: int | None = None, core_number: int | None = None, on_spark: bool = False,
             device: str | torch.device | None = None, dist: bool | None = None, backend: str | None = None):
        with _S.lock:
            env_world = int(os.environ.get("WORLD_SIZE", "1"))
            _S.rank = int(os.environ.get("RANK", "0"))
            _S.world_size = env_world
            _S.local_rank = int(os.environ.get("LOCAL_RANK", str(_S.rank)))
            _S.node_number = node_number if node_number is not None else max(1, env_world)
            cores = core_number or config.get_property("bigdl.coreNumber") or (os.cpu_count() or 1)
            _S.core_number = int(cores)
            if device is not None:
                _S.device = torch.device(device)
            elif torch.cuda.is_available():
                n = torch.cuda.device_count()
                _S.device = torch.device("cuda", _S.local_rank % max(1, n))
            else:
                _S.device = torch.device("cpu")
            if _S.device.type == "cuda":
                torch.cuda.set_device(_S.device)
            want = str(config.get_property("bigdl.compute.dtype")).lower()
            if want == "auto":
                # device compute is bf16 with fp32 master weights (the HIP conv/GEMM kernels are
                # bf16 MFMA); host compute stays fp32 like the reference
                want = "bf16" if _S.device.type == "cuda" else "fp32"
            _S.compute_dtype = _DTYPES[want]
            want_dist = dist if dist is not None else env_world > 1
            if want_dist:
                import torch.distributed as tdist
                if not tdist.is_initialized():
                    # BIGDL_DIST_BACKEND=gloo rehearses the multi-rank device path with several ranks
                    # on one card (RCCL refuses two ranks on the same GPU)
                    be = backend or os.environ.get("BIGDL_DIST_BACKEND") or ("nccl" if _S.device.type == "cuda" else "gloo")
                    import datetime
                    # collective watchdog: a hung collective becomes an error after
                    # this many seconds, which the optimizer's retry loop / the launcher can handle
                    kw = {"timeout": datetime.timedelta(seconds=float(config.get_property("bigdl.comm.timeout")))}
                    if be == "nccl":
                        kw["device_id"] = _S.device
                        apply_comm_env()
                    tdist.init_process_group(backend=be, **kw)
                    _S.process_group_owned = True
                    # tear the group down before interpreter exit: a live gloo / RCCL group's
                    # threads destroyed by the C++ runtime at exit abort the process (SIGABRT)
                    import atexit
                    atexit.register(_shutdown_at_exit)
                _S.rank = tdist.get_rank()
                _S.world_size = tdist.get_world_size()
            if _S.default_pool is None:
                _S.default_pool = ThreadPoolExecutor(max_workers=max(1, min(16, _S.core_number)))
            _S.inited = True
        return Engine

    @staticmethod
    def is_inited() -> bool:
        return _S.inited

    @staticmethod
    def _ensure():
        if not _S.inited:
            Engine.init()

    @staticmethod
    def device() -> torch.device:
        Engine._ensure()
        return _S.device

    @staticmethod
    def set_device(dev):
        Engine._ensure()
        _S.device = torch.device(dev)

    @staticmethod
    def compute_dtype() -> torch.dtype:
        Engine._ensure()
        return _S.compute_dtype

    @staticmethod
    def set_compute_dtype(dt):
        Engine._ensure()
        _S.compute_dtype = _DTYPES[dt] if isinstance(dt, str) else dt

    @staticmethod
    def node_number() -> int:
        Engine._ensure()
        return _S.node_number

    nodeNumber = node_number

    @staticmethod
    def core_number() -> int:
        Engine._ensure()
        return _S.core_number

    coreNumber = core_number

    @staticmethod
    def set_node_and_core(nodes: int, cores: int):
        Engine._ensure()
        _S.node_number, _S.core_number = int(nodes), int(cores)

    setNodeAndCore = set_node_and_core

    @staticmethod
    def rank() -> int:
        Engine._ensure()
        return _S.rank

    @staticmethod
    def world_size() -> int:
        Engine._ensure()
        return _S.world_size

    @staticmethod
    def local_rank() -> int:
        Engine._ensure()
        return _S.local_rank

    @staticmethod
    def is_distributed() -> bool:
        import torch.distributed as tdist
        return tdist.is_available() and tdist.is_initialized() and tdist.get_world_size() > 1

    @staticmethod
    def default_pool() -> ThreadPoolExecutor:
        Engine._ensure()
        return _S.default_pool

    @staticmethod
    def engine_type() -> str:
        return "hip" if Engine.device().type == "cuda" else "cpu"

    getEngineType = engine_type

    @staticmethod
    def shutdown():
        import torch.distributed as tdist
        if _S.process_group_owned and tdist.is_initialized():
            tdist.destroy_process_group()
            _S.process_group_owned = False
        _S.inited = False

    @staticmethod
    def reset():
        Engine.shutdown()
        _S.__init__()


def _shutdown_at_exit():
    try:
        Engine.shutdown()
    except Exception:  # noqa: BLE001 — best effort at interpreter exit
        pass


def apply_comm_env(env=None) -> dict:
    """RCCL knobs that must be in the environment before the first communicator is created
    (SURVEY §5.8): ``bigdl.comm.channels`` caps the channels — and with them the CUs — a collective
    takes from compute (``NCCL_MIN_NCHANNELS`` / ``NCCL_MAX_NCHANNELS``).  Values the user already
    exported win.  ``env`` defaults to ``os.environ`` (the launcher passes the child env)."""
    env = os.environ if env is None else env
    ch = int(config.get_property("bigdl.comm.channels") or 0)
    if ch > 0:
        env.setdefault("NCCL_MIN_NCHANNELS", str(ch))
        env.setdefault("NCCL_MAX_NCHANNELS", str(ch))
    return env


def init_engine(*args, **kwargs):
    """pyspark ``init_engine`` (``PY/util/common.py:420``)."""
    return Engine.init(*args, **kwargs)
