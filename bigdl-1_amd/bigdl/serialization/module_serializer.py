"""``.bigdl`` model persistence (protobuf), compatible with the reference format.

Reference: ``DL/utils/serializer/ModuleSerializable.scala:44-533`` (moduleType = JVM class name,
attrs = primary-constructor parameter names, ``module_tags``/``module_numerics``, parameters in
``parameters()`` order, version), ``ModuleLoader.scala:37-363`` (single file with a top-level
``global_storage`` NameAttrList holding every storage once — flat parameter arenas share one storage
and tensors carry 1-based offsets/strides; two-file mode with a weight file
``int32 MAGIC=3721, int32 count, {int32 id, int32 dataType, int32 size, data}*, int32 digestLen,
MD5`` written big-endian as Java's DataOutputStream does), ``Types.scala:54-60``.
Custom (de)serialisation for containers (``subModules``), graphs (``preModules`` +
``inputNames``/``outputNames``) and batch norm (``runningMean``/``runningVar``/``saveMean``/``saveStd``).
"""
from __future__ import annotations

import hashlib
import inspect
import io
import os
import struct
from collections import OrderedDict
from typing import Dict, Optional

import numpy as np
import torch

from ..version import BIGDL_VERSION
from . import bigdl_pb as pb

MAGIC_NO = 3721
GLOBAL_STORAGE = "global_storage"
MODULE_TAGS = "module_tags"
MODULE_NUMERICS = "module_numerics"
DT = pb.DataType

# python kwarg -> scala constructor parameter name, where camelCase conversion is not enough
_GLOBAL_ALIASES = {"kw": "kW", "kh": "kH", "dw": "dW", "dh": "dH", "data_format": "format", "k_w": "kW",
                   "k_h": "kH", "d_w": "dW", "d_h": "dH", "k_t": "kT", "d_t": "dT", "init_p": "initP", "ip": "ip",
                   "th": "th", "v": "v"}

_SKIP_ARGS = {"bigdl_type", "init_weight", "init_bias", "init_grad_weight", "init_grad_bias"}


def _camel(s: str) -> str:
    if s in _GLOBAL_ALIASES:
        return _GLOBAL_ALIASES[s]
    parts = s.split("_")
    return parts[0] + "".join(p[:1].upper() + p[1:] for p in parts[1:])


# ------------------------------------------------------------------------------------------------ registry
_REGISTRY: Dict[str, type] = {}


def _register_all():
    if _REGISTRY:
        return
    import bigdl.nn as nn
    from ..nn.abstractnn import AbstractModule, AbstractCriterion
    for name in dir(nn):
        obj = getattr(nn, name)
        if isinstance(obj, type) and issubclass(obj, (AbstractModule,)) and obj is not AbstractModule:
            _REGISTRY[obj.scala_class_name()] = obj
            _REGISTRY.setdefault(obj.__name__, obj)
    from ..nn.graph import _InputLayer, Graph
    _REGISTRY["com.intel.analytics.bigdl.nn.Input"] = _InputLayer
    _REGISTRY["com.intel.analytics.bigdl.nn.StaticGraph"] = Graph
    _REGISTRY["com.intel.analytics.bigdl.nn.Graph"] = Graph
    _REGISTRY["com.intel.analytics.bigdl.nn.DynamicGraph"] = Graph
    try:
        from ..nn import recurrent as rec
        for name in dir(rec):
            obj = getattr(rec, name)
            if isinstance(obj, type) and issubclass(obj, AbstractModule):
                _REGISTRY[obj.scala_class_name()] = obj
    except ImportError:
        pass
    try:  # TF op layers (nn/tf: control flow, data-flow resources, ...)
        from ..nn import tf as tfm
        for name in dir(tfm):
            obj = getattr(tfm, name)
            if isinstance(obj, type) and issubclass(obj, AbstractModule):
                _REGISTRY[obj.scala_class_name()] = obj
                _REGISTRY.setdefault(obj.__name__, obj)
    except ImportError:
        pass
    try:
        from ..nn.quantized import layers as q
        for name in dir(q):
            obj = getattr(q, name)
            if isinstance(obj, type) and issubclass(obj, AbstractModule):
                _REGISTRY[obj.scala_class_name()] = obj
    except ImportError:
        pass


def register_module(scala_name: str, cls: type):
    _register_all()
    _REGISTRY[scala_name] = cls


def lookup(module_type: str) -> type:
    _register_all()
    if module_type in _REGISTRY:
        return _REGISTRY[module_type]
    short = module_type.rsplit(".", 1)[-1]
    if short in _REGISTRY:
        return _REGISTRY[short]
    raise KeyError(f"no module class registered for {module_type}")


# ------------------------------------------------------------------------------------------------ tensors
class _SerCtx:
    def __init__(self):
        self.storages: Dict[int, pb.BigDLTensor] = OrderedDict()  # tensor id -> full tensor proto
        self.storage_ids: Dict[int, int] = {}  # untyped storage ptr -> storage id
        self.written_storages: set = set()
        self.next_id = 1
        # deferred storage payloads (tensor id → (field number, numpy snapshot)): the walk only
        # snapshots the data; the bytes are merged into the final global-storage entry afterwards,
        # so no message copy ever carries a payload (and the merge can run off the training thread)
        self.defer = False
        self.fills: Dict[int, tuple] = {}

    def _new_id(self):
        self.next_id += 1
        return self.next_id


def _storage_dtype(t: torch.Tensor) -> int:
    if t.dtype in (torch.float32, torch.bfloat16, torch.float16):
        return DT["FLOAT"]
    if t.dtype == torch.float64:
        return DT["DOUBLE"]
    if t.dtype == torch.int64:
        return DT["INT64"]
    if t.dtype == torch.bool:
        return DT["BOOL"]
    return DT["INT32"]


def _varint(v: int) -> bytes:
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        out.append(b | (0x80 if v else 0))
        if not v:
            return bytes(out)


def _merge_packed(msg, field_no: int, arr: np.ndarray) -> None:
    """Fill a packed repeated float/double field from raw little-endian bytes: the wire encoding
    (tag, length, payload) is parsed by the C protobuf runtime — a Python-level ``extend`` of 25 M
    floats (ResNet-50) took seconds, this takes milliseconds and yields the identical message."""
    payload = np.ascontiguousarray(arr).tobytes()
    if payload:
        msg.MergeFromString(_varint((field_no << 3) | 2) + _varint(len(payload)) + payload)


def _tensor_to_pb(ctx: _SerCtx, t: Optional[torch.Tensor], with_data: bool = True) -> pb.BigDLTensor:
    """Full tensor proto (storage data included the first time a storage is seen)."""
    tp = pb.BigDLTensor()
    if t is None:
        return tp
    t = t.detach()
    if t.dtype in (torch.bfloat16, torch.float16):
        t = t.float()
    st = t.untyped_storage()
    key = st.data_ptr()
    sid = ctx.storage_ids.get(key)
    if sid is None:
        sid = ctx._new_id()
        ctx.storage_ids[key] = sid
    tid = ctx._new_id()
    tp.id = tid
    tp.datatype = _storage_dtype(t)
    tp.dimension = t.dim()
    tp.nElements = t.numel()
    tp.isScalar = t.dim() == 0
    tp.tensorType = 0
    tp.offset = t.storage_offset() + 1
    tp.size.extend(list(t.shape))
    tp.stride.extend(list(t.stride()))
    sp = tp.storage
    sp.datatype = tp.datatype
    sp.id = sid
    if with_data and sid not in ctx.written_storages:
        ctx.written_storages.add(sid)
        n_el = st.nbytes() // t.element_size()
        full = torch.empty(0, dtype=t.dtype, device=t.device).set_(st, 0, (n_el,), (1,)).cpu()
        arr = full.numpy()
        if tp.datatype in (DT["FLOAT"], DT["DOUBLE"]):
            field, fmt = (2, "<f4") if tp.datatype == DT["FLOAT"] else (3, "<f8")
            snap = arr.astype(fmt)  # always a copy: a consistent snapshot even of host tensors
            if ctx.defer:
                ctx.fills[tid] = (field, snap)
            else:
                _merge_packed(sp, field, snap)
        elif tp.datatype == DT["INT64"]:
            sp.long_data.extend(arr.astype(np.int64).tolist())
        elif tp.datatype == DT["BOOL"]:
            sp.bool_data.extend(arr.astype(bool).tolist())
        else:
            sp.int_data.extend(arr.astype(np.int32).tolist())
    ctx.storages[tid] = tp
    return tp


def _reset(tp: pb.BigDLTensor) -> pb.BigDLTensor:
    r = pb.BigDLTensor()
    r.CopyFrom(tp)
    r.ClearField("storage")
    if tp.HasField("storage"):
        r.storage.datatype = tp.storage.datatype
        r.storage.id = tp.storage.id
    return r


class _DeCtx:
    def __init__(self, storages: Dict[int, torch.Tensor]):
        self.storages = storages  # storage id -> flat tensor
        self.tensors: Dict[int, torch.Tensor] = {}


def _storage_from_pb(sp) -> Optional[torch.Tensor]:
    if len(sp.float_data):
        return torch.tensor(np.asarray(sp.float_data, dtype=np.float32))
    if len(sp.double_data):
        return torch.tensor(np.asarray(sp.double_data, dtype=np.float64))
    if len(sp.long_data):
        return torch.tensor(np.asarray(sp.long_data, dtype=np.int64))
    if len(sp.int_data):
        return torch.tensor(np.asarray(sp.int_data, dtype=np.int32))
    if len(sp.bool_data):
        return torch.tensor(np.asarray(sp.bool_data, dtype=bool))
    return None


def _tensor_from_pb(ctx: _DeCtx, tp) -> Optional[torch.Tensor]:
    if tp.id in ctx.tensors:
        return ctx.tensors[tp.id]
    if tp.nElements == 0 and not tp.isScalar and not len(tp.size):
        return None
    flat = None
    if tp.HasField("storage"):
        flat = ctx.storages.get(tp.storage.id)
        if flat is None:
            flat = _storage_from_pb(tp.storage)
            if flat is not None:
                ctx.storages[tp.storage.id] = flat
    if flat is None:
        return None
    size = list(tp.size)
    stride = list(tp.stride) if len(tp.stride) else None
    if stride is None:
        stride, acc = [], 1
        for s in reversed(size):
            stride.insert(0, acc)
            acc *= s
    t = torch.as_strided(flat, size, stride, tp.offset - 1) if size else flat[tp.offset - 1].reshape(())
    ctx.tensors[tp.id] = t
    return t


# ------------------------------------------------------------------------------------------------ attrs
def _set_attr(ctx: _SerCtx, av: pb.AttrValue, v):
    from ..nn.abstractnn import AbstractModule
    from ..nn.initialization_method import (InitializationMethod, RandomUniform, RandomNormal, Zeros, Ones,
                                            ConstInitMethod, Xavier, BilinearFiller)
    from ..optim.regularizer import L1L2Regularizer, L1Regularizer, L2Regularizer
    if v is None:
        av.dataType = DT["TENSOR"]
        return
    if isinstance(v, bool):
        av.dataType = DT["BOOL"]
        av.boolValue = v
    elif isinstance(v, int):
        if -2 ** 31 <= v < 2 ** 31:
            av.dataType = DT["INT32"]
            av.int32Value = v
        else:
            av.dataType = DT["INT64"]
            av.int64Value = v
    elif isinstance(v, float):
        av.dataType = DT["DOUBLE"]
        av.doubleValue = v
    elif isinstance(v, str):
        if v in ("NCHW", "NHWC"):
            av.dataType = DT["DATA_FORMAT"]
            av.dataFormatValue = 0 if v == "NCHW" else 1
        else:
            av.dataType = DT["STRING"]
            av.stringValue = v
    elif isinstance(v, torch.Tensor):
        av.dataType = DT["TENSOR"]
        av.tensorValue.CopyFrom(_reset(_tensor_to_pb(ctx, v)))
    elif isinstance(v, L1L2Regularizer):
        av.dataType = DT["REGULARIZER"]
        rt = 1 if isinstance(v, L1Regularizer) else 2 if isinstance(v, L2Regularizer) else 0
        av.regularizerValue.regularizerType = rt
        av.regularizerValue.regularData.extend([v.l1, v.l2] if rt == 0 else [v.l1] if rt == 1 else [v.l2])
    elif isinstance(v, InitializationMethod):
        av.dataType = DT["INITMETHOD"]
        im = av.initMethodValue
        if isinstance(v, RandomUniform):
            if v.lower is None:
                im.methodType = 1
            else:
                im.methodType = 2
                im.data.extend([v.lower, v.upper])
        elif isinstance(v, RandomNormal):
            im.methodType = 3
            im.data.extend([v.mean, v.stdv])
        elif isinstance(v, Zeros):
            im.methodType = 4
        elif isinstance(v, Ones):
            im.methodType = 5
        elif isinstance(v, ConstInitMethod):
            im.methodType = 6
            im.data.append(v.value)
        elif isinstance(v, Xavier):
            im.methodType = 7
        elif isinstance(v, BilinearFiller):
            im.methodType = 8
    elif isinstance(v, AbstractModule):
        av.dataType = DT["MODULE"]
        av.bigDLModuleValue.CopyFrom(_module_to_pb(ctx, v))
    elif isinstance(v, (list, tuple)):
        av.dataType = DT["ARRAY_VALUE"]
        arr = av.arrayValue
        arr.size = len(v)
        if all(isinstance(x, bool) for x in v) and v:
            arr.datatype = DT["BOOL"]
            arr.boolean.extend(v)
        elif all(isinstance(x, int) for x in v):
            arr.datatype = DT["INT32"]
            arr.i32.extend(v)
        elif all(isinstance(x, (int, float)) for x in v):
            arr.datatype = DT["DOUBLE"]
            arr.dbl.extend([float(x) for x in v])
        elif all(isinstance(x, str) for x in v):
            arr.datatype = DT["STRING"]
            arr.str.extend(v)
        elif all(isinstance(x, AbstractModule) for x in v):
            arr.datatype = DT["MODULE"]
            for x in v:
                arr.bigDLModule.add().CopyFrom(_module_to_pb(ctx, x))
        elif all(isinstance(x, torch.Tensor) for x in v):
            arr.datatype = DT["TENSOR"]
            for x in v:
                arr.tensor.add().CopyFrom(_reset(_tensor_to_pb(ctx, x)))
        elif v and all(isinstance(x, (list, tuple)) and all(isinstance(y, int) and not isinstance(y, bool)
                                                           for y in x) for x in v):
            # an int table (Transpose permutations, crop pairs): flattened row-major like the
            # reference's Array[(Int, Int)] serializer; the constructors re-pair a flat list
            flat = [int(y) for x in v for y in x]
            arr.size = len(flat)
            arr.datatype = DT["INT32"]
            arr.i32.extend(flat)
        else:
            av.dataType = DT["STRING"]
            av.stringValue = repr(v)
    else:
        av.dataType = DT["STRING"]
        av.stringValue = repr(v)


def _get_attr(ctx: _DeCtx, av):
    from ..nn.initialization_method import RandomUniform, RandomNormal, Zeros, Ones, ConstInitMethod, Xavier, BilinearFiller
    from ..optim.regularizer import L1L2Regularizer, L1Regularizer, L2Regularizer
    which = av.WhichOneof("value")
    if which is None:
        return None
    if which in ("int32Value", "int64Value", "floatValue", "doubleValue", "stringValue", "boolValue"):
        return getattr(av, which)
    if which == "dataFormatValue":
        return "NCHW" if av.dataFormatValue == 0 else "NHWC"
    if which == "tensorValue":
        return _tensor_from_pb(ctx, av.tensorValue)
    if which == "regularizerValue":
        r = av.regularizerValue
        d = list(r.regularData)
        return L1L2Regularizer(*d) if r.regularizerType == 0 else L1Regularizer(d[0]) if r.regularizerType == 1 else L2Regularizer(d[0])
    if which == "initMethodValue":
        im = av.initMethodValue
        d = list(im.data)
        return {1: lambda: RandomUniform(), 2: lambda: RandomUniform(d[0], d[1]), 3: lambda: RandomNormal(d[0], d[1]),
                4: Zeros, 5: Ones, 6: lambda: ConstInitMethod(d[0]), 7: Xavier, 8: BilinearFiller}.get(
            im.methodType, lambda: None)()
    if which == "bigDLModuleValue":
        return _module_from_pb(ctx, av.bigDLModuleValue)
    if which == "variableFormatValue":
        return av.variableFormatValue
    if which == "arrayValue":
        a = av.arrayValue
        for f in ("i32", "i64", "flt", "dbl", "str", "boolean"):
            vals = list(getattr(a, f))
            if vals:
                return vals
        if len(a.bigDLModule):
            return [_module_from_pb(ctx, m) for m in a.bigDLModule]
        if len(a.tensor):
            return [_tensor_from_pb(ctx, t) for t in a.tensor]
        return []
    if which == "nameAttrListValue":
        return {k: _get_attr(ctx, v) for k, v in av.nameAttrListValue.attr.items()}
    if which == "shape":
        return list(av.shape.shapeValue)
    return None


# ------------------------------------------------------------------------------------------------ modules
def _ctor_items(m):
    sig = inspect.signature(type(m).__init__)
    for k, v in m._ctor_args.items():
        if k in _SKIP_ARGS or k not in sig.parameters:
            continue
        yield k, v


def _module_to_pb(ctx: _SerCtx, m) -> pb.BigDLModule:
    from ..nn.containers import Container
    from ..nn.graph import Graph
    from ..nn.layers.normalization import BatchNormalization
    mp = pb.BigDLModule()
    mp.name = m.get_name()
    mp.moduleType = m.scala_class_name()
    mp.version = BIGDL_VERSION.replace("-SNAPSHOT", "")
    mp.train = bool(m.train)
    _set_attr(ctx, mp.attr[MODULE_TAGS], ["Float"])
    _set_attr(ctx, mp.attr[MODULE_NUMERICS], ["Float"])
    for k, v in _ctor_items(m):
        from ..nn.abstractnn import AbstractModule
        if isinstance(m, Container) and (isinstance(v, AbstractModule) or (
                isinstance(v, (list, tuple)) and v and all(isinstance(x, AbstractModule) for x in v))):
            continue  # children travel as subModules
        _set_attr(ctx, mp.attr[_camel(k)], v)
    # extra state
    if hasattr(m, "ceilMode"):
        _set_attr(ctx, mp.attr["ceilMode"], bool(m.ceilMode))
    if hasattr(m, "numInputDims") and type(m).__name__ == "View":
        _set_attr(ctx, mp.attr["numInputDims"], int(m.numInputDims))
    if isinstance(m, BatchNormalization):
        for k in ("runningMean", "runningVar", "saveMean", "saveStd"):
            _set_attr(ctx, mp.attr[k], getattr(m, k))
    elif getattr(m, "_buffer_names", None):
        # other non-trainable state (e.g. the int8 weights + scales of quantized layers, the
        # reference's QuantizedTensor parameters) as extra attributes; readers that do not know
        # them ignore unknown attribute names
        for k in m._buffer_names:
            v = getattr(m, k, None)
            if isinstance(v, torch.Tensor):
                _set_attr(ctx, mp.attr[_BUF + k], v)
    st = m.__dict__.get("_int8_state")
    if st is not None and (st["in"] or st["out"] or st["w"] or st["inMask"] or st["outMask"] or st["wMask"]):
        # MklInt8Convertible state (bigdl.proto fields 17-23)
        mp.isMklInt8Enabled = True
        mp.inputDimMasks, mp.outputDimMasks, mp.weightDimMasks = st["inMask"], st["outMask"], st["wMask"]
        for field, key in ((mp.inputScales, "in"), (mp.outputScales, "out"), (mp.weightScales, "w")):
            for sc in st[key]:
                _set_attr(ctx, field.add(), [float(x) for x in sc])
    if isinstance(m, Graph):
        from ..nn.dynamic_graph import DynamicGraph
        dyn = isinstance(m, DynamicGraph)
        # a dynamic graph saves every reachable node (its execution order exists only after a run)
        order = list(reversed(m._all_nodes)) if dyn else m.forward_order
        for n in order:
            sub = _module_to_pb(ctx, n.element)
            sub.preModules.extend([p.element.get_name() for p in n.prev_nodes])
            sub.nextModules.extend([q.element.get_name() for q in n.next_nodes])
            mp.subModules.add().CopyFrom(sub)
            # the edges' output selections (Graph.scala:672-698 doSerializeModule "<name>_edges", written by
            # NameListConverter, DataConverter.scala:225-241): ONE NameAttrList named after the node whose
            # attr maps each previous node's name → INT32 1-based output index of its Table (-1 = the
            # whole activity)
            name = n.element.get_name()
            ev = mp.attr[f"{name}_edges"]
            ev.dataType = DT["NAME_ATTR_LIST"]
            ev.nameAttrListValue.name = name
            for p, idx in zip(n.prev_nodes, n.prev_index):
                _set_attr(ctx, ev.nameAttrListValue.attr[p.element.get_name()], int(idx) if idx else -1)
        _set_attr(ctx, mp.attr["inputNames"], [n.element.get_name() for n in m.inputs])
        _set_attr(ctx, mp.attr["outputNames"], [n.element.get_name() for n in m.outputs_nodes])
        if dyn:
            _set_attr(ctx, mp.attr["generateBackward"], bool(m.generate_backward))
        return mp
    from ..nn.layers.recurrent import Recurrent, Cell, MultiRNNCell
    if isinstance(m, Recurrent):
        # the preTopology (i2g) belongs to the cell; Recurrent.add rebuilds its TimeDistributed
        # wrapper (and the optional BN) from the cell on load
        if m.topology is not None:
            mp.subModules.add().CopyFrom(_module_to_pb(ctx, m.topology))
        return mp
    if isinstance(m, Cell) and not isinstance(m, MultiRNNCell):
        # a cell rebuilds its gate layers in its constructor: store it as a leaf holding every
        # weight it owns (preTopology first, as Recurrent.parameters() orders them)
        mp.hasParameters = True
        for w in _cell_params(m):
            mp.parameters.add().CopyFrom(_reset(_tensor_to_pb(ctx, w)))
        return mp
    if isinstance(m, Container):
        for c in m.modules:
            mp.subModules.add().CopyFrom(_module_to_pb(ctx, c))
        return mp
    p = m.parameters()
    if p is not None:
        mp.hasParameters = True
        for w in p[0]:
            mp.parameters.add().CopyFrom(_reset(_tensor_to_pb(ctx, w)))
    return mp


_BUF = "buffer:"


def _cell_params(m):
    ps = []
    if m.preTopology is not None and not m.includePreTopology:
        p = m.preTopology.parameters()
        ps += list(p[0]) if p else []
    p = m.parameters()
    ps += list(p[0]) if p else []
    return ps


def _instantiate(cls, attrs: dict):
    sig = inspect.signature(cls.__init__)
    kwargs = {}
    for pname, prm in sig.parameters.items():
        if pname in ("self", "bigdl_type") or prm.kind in (prm.VAR_POSITIONAL, prm.VAR_KEYWORD):
            continue
        sname = _camel(pname)
        if sname in attrs:
            kwargs[pname] = attrs[sname]
        elif pname in attrs:
            kwargs[pname] = attrs[pname]
    for pname in list(kwargs):
        if pname in _SKIP_ARGS:
            kwargs.pop(pname)
    try:
        return cls(**kwargs)
    except TypeError:
        req = [p for p, prm in sig.parameters.items() if p != "self" and prm.default is prm.empty and
               prm.kind not in (prm.VAR_POSITIONAL, prm.VAR_KEYWORD)]
        raise TypeError(f"cannot rebuild {cls.__name__}: have {sorted(kwargs)} need {req}")


def _module_from_pb(ctx: _DeCtx, mp):
    from ..nn.containers import Container
    from ..nn.graph import Graph, ModuleNode
    from ..nn.layers.normalization import BatchNormalization
    cls = lookup(mp.moduleType)
    attrs = {k: _get_attr(ctx, v) for k, v in mp.attr.items() if k not in (MODULE_TAGS, MODULE_NUMERICS)}
    if cls is Graph:
        nodes = OrderedDict()
        for sub in mp.subModules:
            nodes[sub.name] = (ModuleNode(_module_from_pb(ctx, sub)), list(sub.preModules))
        for name, (node, pres) in nodes.items():
            # the decoded NameAttrList is the flat {previous node: index} map (its list name, the node's
            # own name, is dropped by _get_attr); files of the round-5 writer nested it one level deeper
            edges = attrs.get(f"{name}_edges")
            if not isinstance(edges, dict):
                edges = {}
            elif isinstance(edges.get(name), dict) and name not in pres:
                edges = edges[name]
            for p in pres:
                idx = edges.get(p, -1) if isinstance(edges, dict) else -1
                node((nodes[p][0], int(idx)) if idx is not None and int(idx) > 0 else nodes[p][0])
        ins = [nodes[n][0] for n in attrs.get("inputNames", [])]
        outs = [nodes[n][0] for n in attrs.get("outputNames", [])]
        if "generateBackward" in attrs:  # Graph.scala doLoadModule: a DynamicGraph
            from ..nn.dynamic_graph import DynamicGraph
            g = DynamicGraph(ins, outs, None, bool(attrs["generateBackward"]))
        else:
            g = Graph(ins, outs)
        g.set_name(mp.name)
        return g
    from ..nn.layers.recurrent import Cell, MultiRNNCell
    subs = None
    consumed = False
    if issubclass(cls, Container) and not (issubclass(cls, Cell) and not issubclass(cls, MultiRNNCell)):
        subs = [_module_from_pb(ctx, sub) for sub in mp.subModules]
    try:
        m = _instantiate(cls, attrs)
    except TypeError:
        # a container whose constructor takes its child module(s) (Bottle(module), MultiRNNCell(cells),
        # TableOperation(layer), ...): feed the deserialized children to the missing argument
        if not subs:
            raise
        sig = inspect.signature(cls.__init__)
        req = [p for p, prm in sig.parameters.items() if p != "self" and prm.default is prm.empty and
               prm.kind not in (prm.VAR_POSITIONAL, prm.VAR_KEYWORD) and _camel(p) not in attrs and p not in attrs]
        if len(req) != 1:
            raise
        extra = dict(attrs)
        extra[req[0]] = subs if req[0] in ("cells", "modules", "layers") else subs[0]
        m = _instantiate(cls, extra)
        consumed = True
    if mp.name:
        m.set_name(mp.name)
    if mp.isMklInt8Enabled or len(mp.inputScales) or len(mp.outputScales) or len(mp.weightScales):
        m.setInputDimMask(mp.inputDimMasks)
        m.setOutputDimMask(mp.outputDimMasks)
        m.setWeightDimMask(mp.weightDimMasks)
        m.setInputScales([list(_get_attr(ctx, a)) for a in mp.inputScales])
        m.setOutputScales([list(_get_attr(ctx, a)) for a in mp.outputScales])
        m.setWeightScales([list(_get_attr(ctx, a)) for a in mp.weightScales])
    if isinstance(m, Container) and subs is not None and not consumed:
        for sub in subs:
            m.add(sub)
    if "ceilMode" in attrs and hasattr(m, "ceilMode") and attrs["ceilMode"] is not None:
        m.ceilMode = bool(attrs["ceilMode"])
    if ("numInputDims" in attrs and type(m).__name__ == "View" and hasattr(m, "numInputDims")
            and attrs["numInputDims"] is not None):
        m.numInputDims = int(attrs["numInputDims"])
    if isinstance(m, BatchNormalization):
        for k in ("runningMean", "runningVar"):
            t = attrs.get(k)
            if isinstance(t, torch.Tensor):
                getattr(m, k).copy_(t.reshape(getattr(m, k).shape))
    for k, t in attrs.items():
        if k.startswith(_BUF) and isinstance(t, torch.Tensor):
            dst = getattr(m, k[len(_BUF):], None)
            if isinstance(dst, torch.Tensor) and dst.numel() == t.numel():
                dst.copy_(t.reshape(dst.shape).to(dst.dtype))
    if mp.hasParameters and len(mp.parameters):
        p = m.parameters()
        if isinstance(m, Cell) and not isinstance(m, MultiRNNCell):
            p = (_cell_params(m), None)
        if p is not None:
            for dst, tp in zip(p[0], mp.parameters):
                src = _tensor_from_pb(ctx, tp)
                if src is not None:
                    dst.copy_(src.reshape(dst.shape).to(dst.dtype))
    m.training(mp.train)
    return m


# ------------------------------------------------------------------------------------------------ files
def _check_path(path, over_write):
    if os.path.exists(path) and not over_write:
        raise FileExistsError(f"{path} already exists; pass over_write=True")
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)


def fill_global_storage(mp, ctx: _SerCtx, key: str = GLOBAL_STORAGE) -> None:
    """Attach every storage of ``ctx`` under ``mp.attr[key]`` and merge the deferred payloads."""
    nal = mp.attr[key]
    nal.dataType = DT["NAME_ATTR_LIST"]
    nal.nameAttrListValue.name = key
    for tid, tp in ctx.storages.items():
        av = nal.nameAttrListValue.attr[str(tid)]
        av.dataType = DT["TENSOR"]
        av.tensorValue.CopyFrom(tp)
        f = ctx.fills.get(tid)
        if f is not None:
            _merge_packed(av.tensorValue.storage, f[0], f[1])
    ctx.fills.clear()


def module_snapshot(module):
    """Phase 1 of a save: walk the module and snapshot its storages to host memory (the only part
    that must see a quiescent model).  ``module_snapshot_bytes`` finishes it, on any thread."""
    ctx = _SerCtx()
    ctx.defer = True
    return _module_to_pb(ctx, module), ctx


def module_snapshot_bytes(snap) -> bytes:
    mp, ctx = snap
    fill_global_storage(mp, ctx)
    return mp.SerializeToString()


def module_to_bytes(module) -> bytes:
    return module_snapshot_bytes(module_snapshot(module))


def module_from_bytes(data: bytes, storages: Optional[Dict[int, torch.Tensor]] = None):
    mp = pb.BigDLModule()
    mp.ParseFromString(data)
    ctx = _DeCtx(dict(storages or {}))
    if GLOBAL_STORAGE in mp.attr:
        for k, av in mp.attr[GLOBAL_STORAGE].nameAttrListValue.attr.items():
            tp = av.tensorValue
            if tp.HasField("storage") and tp.storage.id not in ctx.storages:
                flat = _storage_from_pb(tp.storage)
                if flat is not None:
                    ctx.storages[tp.storage.id] = flat
    return _module_from_pb(ctx, mp)


def save_module(module, path: str, weight_path: Optional[str] = None, over_write: bool = False):
    _check_path(path, over_write)
    if weight_path is None:
        with open(path, "wb") as f:
            f.write(module_to_bytes(module))
        return
    _check_path(weight_path, over_write)
    ctx = _SerCtx()
    mp = _module_to_pb(ctx, module)
    # storages without data in the model file; data in the weight file
    nal = mp.attr[GLOBAL_STORAGE]
    nal.dataType = DT["NAME_ATTR_LIST"]
    nal.nameAttrListValue.name = GLOBAL_STORAGE
    storages = OrderedDict()
    for tid, tp in ctx.storages.items():
        sp = tp.storage
        if len(sp.float_data) or len(sp.double_data) or len(sp.int_data) or len(sp.long_data):
            storages[sp.id] = (sp.datatype, _storage_from_pb(sp))
        av = nal.nameAttrListValue.attr[str(tid)]
        av.dataType = DT["TENSOR"]
        av.tensorValue.CopyFrom(_reset(tp))
    with open(path, "wb") as f:
        f.write(mp.SerializeToString())
    buf = io.BytesIO()
    buf.write(struct.pack(">ii", MAGIC_NO, len(storages)))
    for sid, (dtype, arr) in storages.items():
        a = arr.numpy()
        buf.write(struct.pack(">iii", sid, dtype, a.size))
        if dtype == DT["FLOAT"]:
            buf.write(a.astype(">f4").tobytes())
        elif dtype == DT["DOUBLE"]:
            buf.write(a.astype(">f8").tobytes())
        elif dtype == DT["INT64"]:
            buf.write(a.astype(">i8").tobytes())
        else:
            buf.write(a.astype(">i4").tobytes())
    body = buf.getvalue()
    digest = hashlib.md5(body).digest()
    with open(weight_path, "wb") as f:
        f.write(body)
        f.write(struct.pack(">i", len(digest)))
        f.write(digest)


def _read_weight_file(weight_path: str) -> Dict[int, torch.Tensor]:
    with open(weight_path, "rb") as f:
        data = f.read()
    magic, count = struct.unpack(">ii", data[:8])
    if magic != MAGIC_NO:
        raise ValueError(f"Magic number mismatch, expected {MAGIC_NO}, actual {magic}")
    pos = 8
    out = {}
    sizes = {DT["FLOAT"]: (">f4", np.float32), DT["DOUBLE"]: (">f8", np.float64), DT["INT64"]: (">i8", np.int64),
             DT["INT32"]: (">i4", np.int32)}
    for _ in range(count):
        sid, dtype, n = struct.unpack(">iii", data[pos:pos + 12])
        pos += 12
        fmt, native = sizes.get(dtype, (">i4", np.int32))
        w = np.dtype(fmt).itemsize
        arr = np.frombuffer(data[pos:pos + n * w], dtype=fmt).astype(native)
        pos += n * w
        out[sid] = torch.from_numpy(arr.copy())
    body_end = pos
    (dlen,) = struct.unpack(">i", data[pos:pos + 4])
    stored = data[pos + 4:pos + 4 + dlen]
    calc = hashlib.md5(data[:body_end]).digest()
    if calc != stored:
        raise ValueError("check sum error, please check weight file")
    return out


def load_module(path: str, weight_path: Optional[str] = None):
    with open(path, "rb") as f:
        data = f.read()
    storages = _read_weight_file(weight_path) if weight_path else None
    return module_from_bytes(data, storages)


def save_definition(module, path: str, over_write: bool = False):
    """Text-format definition with weights cleared (``ModulePersister.saveModelDefinitionToFile``)."""
    from google.protobuf import text_format
    _check_path(path, over_write)
    ctx = _SerCtx()
    mp = _module_to_pb(ctx, module)
    with open(path, "w") as f:
        f.write(text_format.MessageToString(mp))


def load_definition(path: str):
    from google.protobuf import text_format
    mp = pb.BigDLModule()
    with open(path) as f:
        text_format.Merge(f.read(), mp)
    return _module_from_pb(_DeCtx({}), mp)
