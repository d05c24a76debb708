"""Torch7 ``.t7`` binary reader / writer (``DL/utils/TorchFile.scala:79-1102``).

Format (little endian, torch7 ``File.lua`` binary mode): every object starts with an int32 type
tag — NIL 0, NUMBER 1 (float64), STRING 2 (int32 length + bytes), TABLE 3, TORCH 4, BOOLEAN 5.
Tables and torch objects carry an int32 reference index so shared objects are written once.
A torch object is ``version string ("V 1") + class name`` followed by its payload:

* ``torch.{Float,Double,Long,Cuda*}Tensor``: int32 nDim, int64[nDim] size, int64[nDim] stride,
  int64 1-based storage offset, then the storage object;
* ``torch.*Storage``: int64 n + raw elements;
* ``nn.*`` modules: a table of their fields (``weight``, ``bias``, ``kW``, ``modules`` …).

Modules (``cudnn.*`` read as ``nn.*``): BatchNormalization, CAddTable, Concat, ConcatTable, Dropout,
LeakyReLU, Linear, ReLU, Reshape, Sequential, SpatialMaxPooling, SpatialAveragePooling,
SpatialBatchNormalization, SpatialConvolution(MM), SpatialConvolutionMap, SpatialCrossMapLRN,
SpatialZeroPadding, Threshold, View, plus any parameter-free layer whose class name matches ours.
"""
from __future__ import annotations

import os
import struct
from typing import Any, Dict, Optional

import numpy as np
import torch

from ..utils.table import Table

TYPE_NIL, TYPE_NUMBER, TYPE_STRING, TYPE_TABLE, TYPE_TORCH, TYPE_BOOLEAN = 0, 1, 2, 3, 4, 5
TYPE_FUNCTION, LEGACY_TYPE_RECUR_FUNCTION, TYPE_RECUR_FUNCTION = 6, 7, 8

_TENSOR_DT = {
    "torch.FloatTensor": np.float32, "torch.CudaTensor": np.float32,
    "torch.DoubleTensor": np.float64, "torch.CudaDoubleTensor": np.float64,
    "torch.LongTensor": np.int64, "torch.CudaLongTensor": np.int64,
    "torch.IntTensor": np.int32, "torch.ByteTensor": np.uint8, "torch.CharTensor": np.int8,
}
_STORAGE_DT = {k.replace("Tensor", "Storage"): v for k, v in _TENSOR_DT.items()}
_STORAGE_DT["torch.CudaStorage"] = np.float32


class TorchObject:
    """A torch class instance the reader could not map (kept as class name + fields)."""

    def __init__(self, type_name: str, fields: Any):
        self.type_name = type_name
        self.fields = fields

    def __repr__(self):
        return f"TorchObject({self.type_name})"


# ------------------------------------------------------------------------------------------------ reader
class _Reader:
    def __init__(self, data: bytes):
        self.b = data
        self.p = 0
        self.objects: Dict[int, Any] = {}

    def i32(self):
        v = struct.unpack_from("<i", self.b, self.p)[0]
        self.p += 4
        return v

    def i64(self):
        v = struct.unpack_from("<q", self.b, self.p)[0]
        self.p += 8
        return v

    def f64(self):
        v = struct.unpack_from("<d", self.b, self.p)[0]
        self.p += 8
        return v

    def string(self):
        n = self.i32()
        s = self.b[self.p:self.p + n]
        self.p += n
        return s.decode("utf-8", errors="replace")

    def read(self):
        t = self.i32()
        if t == TYPE_NIL:
            return None
        if t == TYPE_NUMBER:
            v = self.f64()
            return int(v) if v.is_integer() and abs(v) < 2 ** 53 else v
        if t == TYPE_STRING:
            return self.string()
        if t == TYPE_BOOLEAN:
            return self.i32() == 1
        if t == TYPE_TABLE:
            idx = self.i32()
            if idx in self.objects:
                return self.objects[idx]
            tab = Table()
            self.objects[idx] = tab
            n = self.i32()
            for _ in range(n):
                k = self.read()
                v = self.read()
                tab[k] = v
            return tab
        if t == TYPE_TORCH:
            idx = self.i32()
            if idx in self.objects:
                return self.objects[idx]
            version = self.string()
            if version.startswith("V "):
                cls = self.string()
            else:  # pre-versioned files: the "version" is the class name
                cls = version
            if cls in _TENSOR_DT:
                obj = self._tensor(cls)
            elif cls in _STORAGE_DT:
                obj = self._storage(cls)
            else:
                self.objects[idx] = None  # placeholder against self-references
                fields = self.read()
                obj = _module_from_torch(cls, fields)
            self.objects[idx] = obj
            return obj
        if t in (TYPE_FUNCTION, TYPE_RECUR_FUNCTION, LEGACY_TYPE_RECUR_FUNCTION):
            n = self.i32()
            self.p += n  # dumped bytecode
            self.read()  # upvalues
            return None
        raise ValueError(f"unsupported t7 type id {t} at offset {self.p - 4}")

    def _tensor(self, cls):
        nd = self.i32()
        size = [self.i64() for _ in range(nd)]
        stride = [self.i64() for _ in range(nd)]
        offset = self.i64() - 1
        storage = self.read()
        if storage is None or nd == 0:
            return torch.empty(0, dtype=torch.from_numpy(np.zeros(0, _TENSOR_DT[cls])).dtype)
        return torch.as_strided(storage, size, stride, offset).clone()

    def _storage(self, cls):
        n = self.i64()
        dt = np.dtype(_STORAGE_DT[cls])
        arr = np.frombuffer(self.b, dtype=dt.newbyteorder("<"), count=n, offset=self.p).copy()
        self.p += n * dt.itemsize
        return torch.from_numpy(arr)


def load_torch_file(path: str):
    with open(path, "rb") as f:
        return _Reader(f.read()).read()


load = load_torch_file


# ------------------------------------------------------------------------------------------------ writer
class _Writer:
    def __init__(self):
        self.parts = []
        self.index = 0
        self.seen: Dict[int, int] = {}
        self._keep = []
        self._last_new = False

    def i32(self, v):
        self.parts.append(struct.pack("<i", int(v)))

    def i64(self, v):
        self.parts.append(struct.pack("<q", int(v)))

    def f64(self, v):
        self.parts.append(struct.pack("<d", float(v)))

    def string(self, s: str):
        b = s.encode("utf-8")
        self.i32(len(b))
        self.parts.append(b)

    def _new_index(self):
        self.index += 1
        return self.index

    def write(self, obj):
        if obj is None:
            self.i32(TYPE_NIL)
        elif isinstance(obj, bool):
            self.i32(TYPE_BOOLEAN)
            self.i32(1 if obj else 0)
        elif isinstance(obj, (int, float, np.integer, np.floating)):
            self.i32(TYPE_NUMBER)
            self.f64(obj)
        elif isinstance(obj, str):
            self.i32(TYPE_STRING)
            self.string(obj)
        elif isinstance(obj, torch.Tensor):
            self._tensor(obj)
        elif isinstance(obj, (Table, dict, list, tuple)):
            self._table(obj)
        elif isinstance(obj, TorchObject):
            self._torch_header(obj, obj.type_name)
            if self._last_new:
                self.write(obj.fields)
        else:
            from ..nn.abstractnn import AbstractModule
            if isinstance(obj, AbstractModule):
                name, fields = _module_to_torch(obj)
                self._torch_header(obj, name)
                if self._last_new:
                    self.write(fields)
            else:
                raise TypeError(f"cannot write {type(obj)} to t7")

    def _torch_header(self, obj, cls):
        self.i32(TYPE_TORCH)
        key = id(obj)
        if key in self.seen:
            self.i32(self.seen[key])
            self._last_new = False
            return
        idx = self._new_index()
        self.seen[key] = idx
        self._keep.append(obj)  # ids stay unique while the writer lives
        self.i32(idx)
        self.string("V 1")
        self.string(cls)
        self._last_new = True

    def _table(self, t):
        self.i32(TYPE_TABLE)
        key = id(t)
        if key in self.seen:
            self.i32(self.seen[key])
            return
        idx = self._new_index()
        self.seen[key] = idx
        self._keep.append(t)
        self.i32(idx)
        if isinstance(t, (list, tuple)):
            items = [(i + 1, v) for i, v in enumerate(t)]
        else:
            items = list(t.items())
        self.i32(len(items))
        for k, v in items:
            self.write(k)
            self.write(v)

    def _tensor(self, t0: torch.Tensor):
        t = t0.detach().cpu()
        if t.dtype in (torch.bfloat16, torch.float16):
            t = t.float()
        if t.dtype == torch.float32:
            cls, scls, np_dt = "torch.FloatTensor", "torch.FloatStorage", np.float32
        elif t.dtype == torch.float64:
            cls, scls, np_dt = "torch.DoubleTensor", "torch.DoubleStorage", np.float64
        else:
            cls, scls, np_dt = "torch.LongTensor", "torch.LongStorage", np.int64
            t = t.long()
        self._torch_header(t0, cls)
        if not self._last_new:
            return
        t = t.contiguous()
        self.i32(t.dim())
        for s in t.shape:
            self.i64(s)
        for s in t.stride():
            self.i64(s)
        self.i64(1)
        # storage object
        self.i32(TYPE_TORCH)
        self.i32(self._new_index())
        self.string("V 1")
        self.string(scls)
        self.i64(t.numel())
        self.parts.append(t.numpy().astype(np_dt).tobytes())

    def bytes(self):
        return b"".join(self.parts)


def save_torch_file(obj, path: str, over_write: bool = False):
    if os.path.exists(path) and not over_write:
        raise FileExistsError(path)
    w = _Writer()
    w.write(obj)
    with open(path, "wb") as f:
        f.write(w.bytes())


def _chain_to_sequential(module):
    """Torch7 has no graph container: a Graph whose nodes form one chain is written as the
    equivalent ``nn.Sequential`` (input placeholders dropped)."""
    from ..nn.graph import Graph, _InputLayer
    from ..nn.containers import Sequential
    if not isinstance(module, Graph) or len(module.inputs) != 1 or len(module.outputs_nodes) != 1:
        return module
    order = module.forward_order
    for a, b in zip(order, order[1:]):
        if b.prev_nodes != [a] or a.next_nodes != [b] or any(b.prev_index):
            return module
    seq = Sequential()
    seq.set_name(module.get_name())
    for n in order:
        if not isinstance(n.element, _InputLayer):
            seq.add(n.element)
    return seq


def save_torch(module, path: str, over_write: bool = False):
    save_torch_file(_chain_to_sequential(module), path, over_write)


def load_torch(path: str):
    return load_torch_file(path)


# ------------------------------------------------------------------------------------------------ modules
def _g(fields, key, default=None):
    if isinstance(fields, Table) and key in fields:
        return fields[key]
    return default


def _set_param(mod, name, value):
    if value is None or not isinstance(value, torch.Tensor) or value.numel() == 0:
        return
    dst = getattr(mod, name, None)
    if dst is None:
        return
    with torch.no_grad():
        dst.copy_(value.reshape(dst.shape).to(dst.dtype))


def _children(fields):
    mods = _g(fields, "modules")
    if mods is None:
        return []
    return [mods[k] for k in sorted(mods.keys()) if mods[k] is not None]


def _module_from_torch(cls: str, fields):
    from .. import nn
    name = cls.replace("cudnn.", "nn.")
    short = name.split(".", 1)[1] if "." in name else name
    f = fields
    if short in ("Sequential", "ConcatTable"):
        m = getattr(nn, short)()
        for c in _children(f):
            m.add(c)
    elif short == "Concat":
        m = nn.Concat(int(_g(f, "dimension")))
        for c in _children(f):
            m.add(c)
    elif short == "Linear":
        w = _g(f, "weight")
        b = _g(f, "bias")
        m = nn.Linear(w.shape[1], w.shape[0], with_bias=b is not None)
        _set_param(m, "weight", w)
        _set_param(m, "bias", b)
    elif short in ("SpatialConvolution", "SpatialConvolutionMM"):
        nin, nout = int(_g(f, "nInputPlane")), int(_g(f, "nOutputPlane"))
        b = _g(f, "bias")
        m = nn.SpatialConvolution(nin, nout, int(_g(f, "kW")), int(_g(f, "kH")), int(_g(f, "dW", 1)),
                                  int(_g(f, "dH", 1)), int(_g(f, "padW", 0)), int(_g(f, "padH", 0)),
                                  with_bias=b is not None)
        _set_param(m, "weight", _g(f, "weight"))
        _set_param(m, "bias", b)
    elif short == "SpatialConvolutionMap":
        m = nn.SpatialConvolutionMap(_g(f, "connTable"), int(_g(f, "kW")), int(_g(f, "kH")), int(_g(f, "dW", 1)),
                                     int(_g(f, "dH", 1)), int(_g(f, "padW", 0)), int(_g(f, "padH", 0)))
        _set_param(m, "weight", _g(f, "weight"))
        _set_param(m, "bias", _g(f, "bias"))
    elif short in ("BatchNormalization", "SpatialBatchNormalization"):
        rm = _g(f, "running_mean")
        rv = _g(f, "running_var")
        w = _g(f, "weight")
        n = rm.numel()
        affine = w is not None and isinstance(w, torch.Tensor) and w.numel() > 0
        m = getattr(nn, short)(n, float(_g(f, "eps", 1e-5)), float(_g(f, "momentum", 0.1)), affine)
        if rv is None and _g(f, "running_std") is not None:  # old torch stored 1/std
            std = _g(f, "running_std")
            rv = 1.0 / (std * std) - float(_g(f, "eps", 1e-5))
        with torch.no_grad():
            m.runningMean.copy_(rm.float())
            m.runningVar.copy_(rv.float())
        if affine:
            _set_param(m, "weight", w)
            _set_param(m, "bias", _g(f, "bias"))
    elif short == "SpatialMaxPooling":
        m = nn.SpatialMaxPooling(int(_g(f, "kW")), int(_g(f, "kH")), int(_g(f, "dW")), int(_g(f, "dH")),
                                 int(_g(f, "padW", 0)), int(_g(f, "padH", 0)))
        if _g(f, "ceil_mode", False):
            m.ceil()
    elif short == "SpatialAveragePooling":
        m = nn.SpatialAveragePooling(int(_g(f, "kW")), int(_g(f, "kH")), int(_g(f, "dW", 1)), int(_g(f, "dH", 1)),
                                     int(_g(f, "padW", 0)), int(_g(f, "padH", 0)),
                                     ceil_mode=bool(_g(f, "ceil_mode", False)),
                                     count_include_pad=bool(_g(f, "count_include_pad", True)),
                                     divide=bool(_g(f, "divide", True)))
    elif short == "SpatialCrossMapLRN":
        m = nn.SpatialCrossMapLRN(int(_g(f, "size", 5)), float(_g(f, "alpha", 1.0)), float(_g(f, "beta", 0.75)),
                                  float(_g(f, "k", 1.0)))
    elif short == "SpatialZeroPadding":
        m = nn.SpatialZeroPadding(int(_g(f, "pad_l", 0)), int(_g(f, "pad_r", 0)), int(_g(f, "pad_t", 0)),
                                  int(_g(f, "pad_b", 0)))
    elif short == "ReLU":
        m = nn.ReLU(bool(_g(f, "inplace", False)))
    elif short == "Threshold":
        m = nn.Threshold(float(_g(f, "threshold", 1e-6)), float(_g(f, "val", 0.0)), bool(_g(f, "inplace", False)))
    elif short == "LeakyReLU":
        m = nn.LeakyReLU(float(_g(f, "negval", 0.01)), bool(_g(f, "inplace", False)))
    elif short == "Dropout":
        m = nn.Dropout(float(_g(f, "p", 0.5)))
    elif short == "CAddTable":
        m = nn.CAddTable(bool(_g(f, "inplace", False)))
    elif short == "View":
        size = _g(f, "size")
        sizes = [int(v) for v in (size.tolist() if isinstance(size, torch.Tensor) else list(size.values()))]
        m = nn.View(sizes)
        nid = _g(f, "numInputDims")
        if nid:
            m.setNumInputDims(int(nid))
    elif short == "Reshape":
        size = _g(f, "size")
        sizes = [int(v) for v in (size.tolist() if isinstance(size, torch.Tensor) else list(size.values()))]
        bm = _g(f, "batchMode")
        m = nn.Reshape(sizes, bm if isinstance(bm, bool) else None)
    else:
        cls_obj = getattr(nn, short, None)
        if cls_obj is None:
            return TorchObject(cls, fields)
        try:
            m = cls_obj()
        except TypeError:
            return TorchObject(cls, fields)
    if isinstance(f, Table) and "train" in f and hasattr(m, "training"):
        m.training(bool(f["train"]))
    return m


def _module_to_torch(m):
    """Our module → (torch class name, field table) (the writers of ``TorchFile.scala:265-700``)."""
    from .. import nn
    t = Table()
    t["_type"] = "torch.FloatTensor"
    t["train"] = bool(m.isTraining())
    name = type(m).__name__
    if isinstance(m, (nn.Sequential, nn.ConcatTable)) and not isinstance(m, nn.Concat):
        cls = "nn.ConcatTable" if isinstance(m, nn.ConcatTable) else "nn.Sequential"
        t["modules"] = Table(*m.modules) if m.modules else Table()
        return cls, t
    if isinstance(m, nn.Concat):
        t["dimension"] = m.dimension
        t["modules"] = Table(*m.modules)
        return "nn.Concat", t
    if isinstance(m, nn.Linear):
        t["weight"] = m.weight.float()
        t["gradWeight"] = m.gradWeight.float()
        if m.bias is not None:
            t["bias"] = m.bias.float()
            t["gradBias"] = m.gradBias.float()
        return "nn.Linear", t
    if isinstance(m, nn.SpatialConvolution):
        if m.nGroup != 1:
            raise ValueError("t7 SpatialConvolution has no groups")
        for k, v in (("nInputPlane", m.nInputPlane), ("nOutputPlane", m.nOutputPlane), ("kW", m.kernelW),
                     ("kH", m.kernelH), ("dW", m.strideW), ("dH", m.strideH), ("padW", m.padW), ("padH", m.padH)):
            t[k] = v
        t["weight"] = m.weight.reshape(m.nOutputPlane, m.nInputPlane, m.kernelH, m.kernelW).float()
        if m.withBias:
            t["bias"] = m.bias.float()
        return "nn.SpatialConvolution", t
    if isinstance(m, nn.BatchNormalization):
        t["running_mean"] = m.runningMean.float()
        t["running_var"] = m.runningVar.float()
        t["eps"] = m.eps
        t["momentum"] = m.momentum
        t["affine"] = bool(m.affine)
        if m.affine:
            t["weight"] = m.weight.float()
            t["bias"] = m.bias.float()
        cls = "nn.SpatialBatchNormalization" if isinstance(m, nn.SpatialBatchNormalization) else \
            "nn.BatchNormalization"
        return cls, t
    if isinstance(m, nn.SpatialMaxPooling):
        for k, v in (("kW", m.kW), ("kH", m.kH), ("dW", m.dW), ("dH", m.dH), ("padW", m.padW), ("padH", m.padH)):
            t[k] = v
        t["ceil_mode"] = bool(getattr(m, "ceilMode", False))
        return "nn.SpatialMaxPooling", t
    if isinstance(m, nn.SpatialAveragePooling):
        for k, v in (("kW", m.kW), ("kH", m.kH), ("dW", m.dW), ("dH", m.dH), ("padW", m.padW), ("padH", m.padH)):
            t[k] = v
        t["ceil_mode"] = bool(m.ceilMode)
        t["count_include_pad"] = bool(m.countIncludePad)
        t["divide"] = bool(m.divide)
        return "nn.SpatialAveragePooling", t
    if isinstance(m, nn.SpatialCrossMapLRN):
        t["size"], t["alpha"], t["beta"], t["k"] = m.size, m.alpha, m.beta, m.k
        return "nn.SpatialCrossMapLRN", t
    if isinstance(m, nn.SpatialZeroPadding):
        t["pad_l"], t["pad_r"], t["pad_t"], t["pad_b"] = m.pads
        return "nn.SpatialZeroPadding", t
    if isinstance(m, nn.ReLU):
        t["inplace"] = bool(getattr(m, "inplace", False))
        t["threshold"], t["val"] = 0.0, 0.0
        return "nn.ReLU", t
    if isinstance(m, nn.Threshold):
        t["threshold"], t["val"], t["inplace"] = m.threshold, m.value, bool(getattr(m, "inPlace", False))
        return "nn.Threshold", t
    if isinstance(m, nn.LeakyReLU):
        t["negval"], t["inplace"] = m.negval, bool(getattr(m, "inplace", False))
        return "nn.LeakyReLU", t
    if isinstance(m, nn.Dropout):
        t["p"] = m.p
        t["v2"] = True
        return "nn.Dropout", t
    if isinstance(m, nn.View):
        t["size"] = torch.tensor(list(m.sizes), dtype=torch.int64)
        t["numInputDims"] = getattr(m, "numInputDims", 0)
        return "nn.View", t
    if isinstance(m, nn.Reshape):
        t["size"] = torch.tensor(list(m.size), dtype=torch.int64)
        if m.batchMode is not None:
            t["batchMode"] = bool(m.batchMode)
        return "nn.Reshape", t
    if isinstance(m, nn.CAddTable):
        t["inplace"] = bool(getattr(m, "inplace", False))
        return "nn.CAddTable", t
    return "nn." + name, t
