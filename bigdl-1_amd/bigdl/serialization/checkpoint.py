"""Checkpoint / resume.

Reference: on trigger ``getModel`` gathers shards and saves ``model.<neval>`` plus one
``optimMethod-<name>.<neval>`` per OptimMethod (``DL/optim/AbstractOptimizer.scala:205-231``,
``Optimizer.scala:548-586``), overwriting fixed names with ``overWriteCheckpoint``; resume takes the
latest files by mtime (``DistriOptimizer.scala:986-1003``).  The reference writes those with Java
serialisation, which is not reproducible outside a JVM, so here:

* ``model.<neval>`` is a ``.bigdl`` protobuf (loadable with ``Module.loadModule``);
* ``optimMethod-<name>.<neval>`` is a BigDLModule-schema protobuf whose ``moduleType`` is the
  OptimMethod's Scala class name, hyper-parameters are attrs and every state tensor / scalar
  (momentum buffer, ``epoch``, ``neval``, ``evalCounter`` …) lives under the ``state`` attr;
* with sharded (ZeRO-1) optimiser state each rank also writes ``….rank<r>`` with its shard's state.
"""
from __future__ import annotations

import glob
import json
import os
from typing import Dict, Optional, Tuple

import torch

from . import bigdl_pb as pb
from .module_serializer import (_SerCtx, _DeCtx, _set_attr, _get_attr, _storage_from_pb, save_module, load_module,
                                fill_global_storage, module_snapshot, module_snapshot_bytes)

_SKIP = {"state", "shadow", "grad_scale", "slices", "_first", "_clr", "_t"}


def optim_to_pb(method, defer: bool = False):
    """OptimMethod → protobuf; ``defer`` returns ``(proto, ctx)`` with the state tensors
    snapshotted but not yet merged (finish with ``fill_global_storage(proto, ctx, "global_storage")``)."""
    ctx = _SerCtx()
    ctx.defer = defer
    mp = pb.BigDLModule()
    mp.moduleType = method.scala_class_name()
    mp.name = type(method).__name__
    for k, v in vars(method).items():
        if k in _SKIP or k.startswith("_"):
            continue
        if isinstance(v, (int, float, bool, str)) or v is None:
            _set_attr(ctx, mp.attr[k], v)
        elif isinstance(v, torch.Tensor):
            _set_attr(ctx, mp.attr[k], v)
        else:
            # schedules etc.: store their simple fields
            try:
                _set_attr(ctx, mp.attr[k], json.dumps({"type": type(v).__name__, **{a: b for a, b in vars(v).items()
                                                                                     if isinstance(b, (int, float, str, bool, list))}}))
            except TypeError:
                pass
    st = mp.attr["state"]
    st.dataType = pb.DataType["NAME_ATTR_LIST"]
    st.nameAttrListValue.name = "state"
    for k, v in method.state.items():
        if isinstance(v, (torch.Tensor, int, float, bool, str)):
            _set_attr(ctx, st.nameAttrListValue.attr[k], v)
    # storages inline (optimizer state is never shared with a model)
    if defer:
        return mp, ctx
    fill_global_storage(mp, ctx, "global_storage")
    return mp


def optim_from_pb(mp):
    from .. import optim as O
    name = mp.moduleType.rsplit(".", 1)[-1]
    cls = getattr(O, name)
    storages = {}
    if "global_storage" in mp.attr:
        for _, av in mp.attr["global_storage"].nameAttrListValue.attr.items():
            sp = av.tensorValue.storage
            flat = _storage_from_pb(sp)
            if flat is not None:
                storages[sp.id] = flat
    ctx = _DeCtx(storages)
    m = cls.__new__(cls)
    O.OptimMethod.__init__(m)
    proto = cls()
    m.__dict__.update(proto.__dict__)
    for k, av in mp.attr.items():
        if k in ("state", "global_storage"):
            continue
        v = _get_attr(ctx, av)
        if isinstance(v, str) and v.startswith("{"):
            try:
                d = json.loads(v)
                sched_cls = getattr(O, d.pop("type"), None)
                if sched_cls is not None:
                    obj = sched_cls.__new__(sched_cls)
                    O.LearningRateSchedule.__init__(obj)
                    obj.__dict__.update(d)
                    v = obj
            except (ValueError, TypeError):
                pass
        setattr(m, k, v)
    m.state = {}
    if "state" in mp.attr:
        for k, av in mp.attr["state"].nameAttrListValue.attr.items():
            v = _get_attr(ctx, av)
            m.state[k] = v.clone() if isinstance(v, torch.Tensor) else v
    return m


def save_optim_method(method, path: str, over_write: bool = False):
    if os.path.exists(path) and not over_write:
        raise FileExistsError(path)
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "wb") as f:
        f.write(optim_to_pb(method).SerializeToString())


def load_optim_method(path: str):
    mp = pb.BigDLModule()
    with open(path, "rb") as f:
        mp.ParseFromString(f.read())
    return optim_from_pb(mp)


def _suffix(state, overwrite):
    return "" if overwrite else f".{state['neval'] - 1}"


# ------------------------------------------------------------------------------------------ async writer
# checkpoints are written asynchronously from a host snapshot.  The calling (training)
# thread only walks the model / optimizer state and copies the tensors to host memory; merging the
# payloads into the protobufs, serialising and writing run on one background thread.  Files appear
# by atomic rename, the ``state`` file last, so a crash mid-write never leaves a torn file behind.
_WRITER = {"queue": None, "thread": None, "error": None}


def _atomic_write(path: str, data, mode: str = "wb"):
    tmp = f"{path}.tmp{os.getpid()}"
    with open(tmp, mode) as f:
        f.write(data)
    os.replace(tmp, path)


def _worker(q):
    while True:
        job = q.get()
        try:
            if job is None:
                return
            job()
        except BaseException as e:  # noqa: BLE001 - surfaced by the next wait_checkpoints()
            _WRITER["error"] = e
        finally:
            q.task_done()


def wait_checkpoints():
    """Block until every queued checkpoint write has finished; re-raise a writer error."""
    q = _WRITER["queue"]
    if q is not None:
        q.join()
    err, _WRITER["error"] = _WRITER["error"], None
    if err is not None:
        raise RuntimeError("asynchronous checkpoint write failed") from err


def _submit(job):
    import queue
    import threading
    q = _WRITER["queue"]
    if q is None or not _WRITER["thread"].is_alive():
        q = _WRITER["queue"] = queue.Queue()
        _WRITER["thread"] = threading.Thread(target=_worker, args=(q,), name="bigdl-checkpoint-writer", daemon=True)
        _WRITER["thread"].start()
    if q.unfinished_tasks >= 4:  # bound the host snapshots held in flight
        q.join()
    q.put(job)


def save_checkpoint(path: str, model, methods: Dict, state: Dict, overwrite: bool = False, world_size: int = 1,
                    sharded: bool = False, asynchronous: bool = False, slices: Optional[Dict] = None):
    """``slices`` = {method key: (arena offset, length)}: recorded in the state file so a resume
    matches optimizer methods by the parameters they own (keys built from default module names
    differ in every process)."""
    os.makedirs(path, exist_ok=True)
    sfx = _suffix(state, overwrite)
    msnap = module_snapshot(model)
    osnaps = []
    for name, m in methods.items():
        m.state.update({k: state[k] for k in ("epoch", "neval", "recordsProcessedThisEpoch") if k in state})
        osnaps.append((name, optim_to_pb(m, defer=True)))
    meta = {k: (float(v) if isinstance(v, (int, float)) else v) for k, v in state.items()
            if isinstance(v, (int, float, str))}
    # how the optimizer state was laid out: a sharded (ZeRO-1) run's un-suffixed optimMethod file
    # holds only rank 0's shard, so a resume must find its own ``.rank<r>`` file at the same world size
    meta["_world_size"] = int(world_size)
    meta["_sharded"] = bool(sharded)
    if slices:
        meta["_slices"] = {name: [int(o), int(n)] for name, (o, n) in slices.items()}

    def job():
        # model and optimizer files first, the state file LAST: a state file names a complete set
        _atomic_write(os.path.join(path, "model" + sfx), module_snapshot_bytes(msnap))
        for name, (mp, ctx) in osnaps:
            fill_global_storage(mp, ctx, "global_storage")
            _atomic_write(os.path.join(path, f"optimMethod-{name}" + sfx), mp.SerializeToString())
        _atomic_write(os.path.join(path, "state" + sfx), json.dumps(meta), "w")
    if asynchronous:
        _submit(job)
    else:
        wait_checkpoints()
        job()


def _shard_key(i: int, name: str, slices: Optional[Dict]) -> str:
    """File key of a method's per-rank shard: its arena offset when known (stable across processes
    and restarts), else its position in sorted key order."""
    if slices and name in slices:
        return f"@{int(slices[name][0])}"
    return f"#{i}"


def save_shard_state(path: str, methods: Dict, state: Dict, rank: int, overwrite: bool = False,
                     asynchronous: bool = False, slices: Optional[Dict] = None):
    """Each rank's shard of the optimizer state, keyed by the method's arena offset (see
    :func:`_shard_key`) — a key derived from a default module name is random per process (the
    reference's ``getName`` postfix), so rank 1 — and a restarted process — could never find a file
    named after rank 0's key."""
    sfx = _suffix(state, overwrite)
    snaps = [(_shard_key(i, name, slices), optim_to_pb(methods[name], defer=True))
             for i, name in enumerate(sorted(methods))]

    def job():
        for key, (mp, ctx) in snaps:
            fill_global_storage(mp, ctx, "global_storage")
            _atomic_write(os.path.join(path, f"optimMethod-{key}{sfx}.rank{rank}"), mp.SerializeToString())
    if asynchronous:
        _submit(job)
    else:
        wait_checkpoints()
        job()


def _latest(pattern: str) -> Optional[str]:
    files = [f for f in glob.glob(pattern) if ".rank" not in f and ".tmp" not in f]
    if not files:
        return None
    return max(files, key=os.path.getmtime)


def has_checkpoint(path: str) -> bool:
    return _latest(os.path.join(path, "model*")) is not None


def load_latest_checkpoint(path: str, world_size: Optional[int] = None,
                           sharded: Optional[bool] = None) -> Tuple[Optional[object], Dict, Dict]:
    """Latest COMPLETE checkpoint under ``path``: the newest ``state<sfx>`` file (written last by
    :func:`save_checkpoint`) fixes the suffix, and the model / optimMethod files of that same suffix
    are loaded — never a newer model with older optimizer state from an interrupted write.  With
    ``world_size`` given, a checkpoint whose optimizer state was sharded is only accepted by a
    sharded run of the SAME world size that finds its own ``.rank<r>`` state file.  Loaded methods
    carry ``_arena_slice`` (offset, length) when the checkpoint recorded it."""
    wait_checkpoints()
    # newest first; a checkpoint whose sharded optimizer files are incomplete (a crash between the
    # state file and another rank's shard write) is skipped for the next-newest complete one
    states = sorted((f for f in glob.glob(os.path.join(path, "state*")) if ".rank" not in f and ".tmp" not in f),
                    key=os.path.getmtime, reverse=True)
    last_err = None
    for sfile in states or [None]:
        try:
            return _load_checkpoint_at(path, sfile, world_size, sharded)
        except FileNotFoundError as e:
            last_err = e
            continue
    raise last_err


def _load_checkpoint_at(path, sfile, world_size, sharded):
    meta = {}
    sfx = None
    if sfile:
        with open(sfile) as fh:
            meta = json.load(fh)
        sfx = os.path.basename(sfile)[len("state"):]
    ck_sharded = bool(meta.get("_sharded", False))
    ck_world = int(meta.get("_world_size", 1))
    if world_size is not None and ck_sharded and (not sharded or ck_world != world_size):
        raise ValueError(f"checkpoint under {path} holds sharded optimizer state for world size {ck_world}; "
                         f"this run is world size {world_size} ({'sharded' if sharded else 'replicated'}) — "
                         "resume with the same world size and bigdl.comm.sharded")
    mfile = os.path.join(path, "model" + sfx) if sfx is not None else None
    if mfile is None or not os.path.exists(mfile):
        mfile = _latest(os.path.join(path, "model*"))
    model = load_module(mfile) if mfile else None
    methods = {}
    for f in glob.glob(os.path.join(path, "optimMethod-*")):
        b = os.path.basename(f)
        if ".rank" in f or ".tmp" in f or b.startswith("optimMethod-#") or b.startswith("optimMethod-@"):
            continue
        base = b[len("optimMethod-"):]
        if sfx is not None:
            if sfx and not base.endswith(sfx):
                continue
            name = base[:len(base) - len(sfx)] if sfx else base
            if not sfx and base.rsplit(".", 1)[-1].isdigit():
                continue
            methods[name] = (os.path.getmtime(f), f)
            continue
        name = base.rsplit(".", 1)[0] if base.rsplit(".", 1)[-1].isdigit() else base
        cur = methods.get(name)
        if cur is None or os.path.getmtime(f) > cur[0]:
            methods[name] = (os.path.getmtime(f), f)
    slices = meta.get("_slices") or {}
    loaded = {}
    rank = int(os.environ.get("RANK", "0"))
    for i, name in enumerate(sorted(methods)):
        f = methods[name][1]
        fsfx = f[len(os.path.join(path, "optimMethod-" + name)):]
        shard = os.path.join(path, f"optimMethod-{_shard_key(i, name, slices)}{fsfx}.rank{rank}")
        if ck_sharded:
            # every rank's shard must be there (not only this rank's), so all ranks agree on which
            # checkpoint is complete and resume from the same one
            for r in range(ck_world):
                sr = os.path.join(path, f"optimMethod-{_shard_key(i, name, slices)}{fsfx}.rank{r}")
                if not os.path.exists(sr):
                    raise FileNotFoundError(f"sharded checkpoint: missing rank {r}'s optimizer state {sr}")
        m = load_optim_method(shard if ck_sharded else f)
        if name in slices:
            m._arena_slice = tuple(slices[name])
        loaded[name] = m
    state = {k: v for k, v in meta.items() if not k.startswith("_")}
    for k in ("epoch", "neval", "recordsProcessedThisEpoch"):
        if k in state:
            state[k] = int(state[k])
    return model, loaded, state
