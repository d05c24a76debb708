"""TensorFlow protobuf schemas re-declared with TensorFlow's field numbers (``framework/graph.proto``,
``node_def.proto``, ``attr_value.proto``, ``tensor.proto``, ``tensor_shape.proto``, ``types.proto``,
``example/{example,feature}.proto``) — the messages the reference's loader and saver read and write
(``DL/utils/tf/TensorflowLoader.scala``, ``TensorflowSaver.scala``; generated Java classes under
``spark/dl/src/main/java/org/tensorflow/``).
"""
from __future__ import annotations

import functools

import numpy as np
import torch

from ...serialization.proto_builder import F, Msg, build

DT = [("DT_INVALID", 0), ("DT_FLOAT", 1), ("DT_DOUBLE", 2), ("DT_INT32", 3), ("DT_UINT8", 4), ("DT_INT16", 5),
      ("DT_INT8", 6), ("DT_STRING", 7), ("DT_COMPLEX64", 8), ("DT_INT64", 9), ("DT_BOOL", 10), ("DT_QINT8", 11),
      ("DT_QUINT8", 12), ("DT_QINT32", 13), ("DT_BFLOAT16", 14), ("DT_QINT16", 15), ("DT_QUINT16", 16),
      ("DT_UINT16", 17), ("DT_COMPLEX128", 18), ("DT_HALF", 19), ("DT_RESOURCE", 20), ("DT_VARIANT", 21),
      ("DT_UINT32", 22), ("DT_UINT64", 23)]
DT = DT + [(n + "_REF", v + 100) for n, v in DT[1:]]

_P = ".tensorflow."


@functools.lru_cache(None)
def graph_classes():
    msgs = [
        Msg("TensorShapeProto", [F("dim", 2, "msg", "repeated", type_name=_P + "TensorShapeProto.Dim"),
                                 F("unknown_rank", 3, "bool")],
            nested=[Msg("Dim", [F("size", 1, "int64"), F("name", 2, "string")])]),
        Msg("TensorProto", [
            F("dtype", 1, "enum", type_name=_P + "DataType"), F("tensor_shape", 2, "msg", type_name=_P + "TensorShapeProto"),
            F("version_number", 3, "int32"), F("tensor_content", 4, "bytes"),
            F("half_val", 13, "int32", "repeated", packed=True), F("float_val", 5, "float", "repeated", packed=True),
            F("double_val", 6, "double", "repeated", packed=True), F("int_val", 7, "int32", "repeated", packed=True),
            F("string_val", 8, "bytes", "repeated"), F("scomplex_val", 9, "float", "repeated", packed=True),
            F("int64_val", 10, "int64", "repeated", packed=True), F("bool_val", 11, "bool", "repeated", packed=True),
            F("dcomplex_val", 12, "double", "repeated", packed=True),
            F("uint32_val", 16, "uint32", "repeated", packed=True), F("uint64_val", 17, "uint64", "repeated", packed=True)]),
        Msg("AttrValue", [
            F("list", 1, "msg", type_name=_P + "AttrValue.ListValue", oneof="value"),
            F("s", 2, "bytes", oneof="value"), F("i", 3, "int64", oneof="value"), F("f", 4, "float", oneof="value"),
            F("b", 5, "bool", oneof="value"), F("type", 6, "enum", type_name=_P + "DataType", oneof="value"),
            F("shape", 7, "msg", type_name=_P + "TensorShapeProto", oneof="value"),
            F("tensor", 8, "msg", type_name=_P + "TensorProto", oneof="value"),
            F("placeholder", 9, "string", oneof="value"),
            F("func", 10, "msg", type_name=_P + "NameAttrList", oneof="value")],
            nested=[Msg("ListValue", [
                F("s", 2, "bytes", "repeated"), F("i", 3, "int64", "repeated", packed=True),
                F("f", 4, "float", "repeated", packed=True), F("b", 5, "bool", "repeated", packed=True),
                F("type", 6, "enum", "repeated", type_name=_P + "DataType", packed=True),
                F("shape", 7, "msg", "repeated", type_name=_P + "TensorShapeProto"),
                F("tensor", 8, "msg", "repeated", type_name=_P + "TensorProto"),
                F("func", 9, "msg", "repeated", type_name=_P + "NameAttrList")])]),
        Msg("NameAttrList", [F("name", 1, "string"), F("attr", 2, "map", type_name=("string", _P + "AttrValue"))]),
        Msg("NodeDef", [F("name", 1, "string"), F("op", 2, "string"), F("input", 3, "string", "repeated"),
                        F("device", 4, "string"), F("attr", 5, "map", type_name=("string", _P + "AttrValue"))]),
        Msg("VersionDef", [F("producer", 1, "int32"), F("min_consumer", 2, "int32"),
                           F("bad_consumers", 3, "int32", "repeated", packed=True)]),
        Msg("GraphDef", [F("node", 1, "msg", "repeated", type_name=_P + "NodeDef"), F("version", 3, "int32"),
                         F("versions", 4, "msg", type_name=_P + "VersionDef")]),
    ]
    _, classes, enums = build("bigdl_tf_graph.proto", "tensorflow", msgs, enums=[("DataType", DT)])
    return classes, enums["DataType"]


@functools.lru_cache(None)
def example_classes():
    msgs = [
        Msg("BytesList", [F("value", 1, "bytes", "repeated")]),
        Msg("FloatList", [F("value", 1, "float", "repeated", packed=True)]),
        Msg("Int64List", [F("value", 1, "int64", "repeated", packed=True)]),
        Msg("Feature", [F("bytes_list", 1, "msg", type_name=_P + "BytesList", oneof="kind"),
                        F("float_list", 2, "msg", type_name=_P + "FloatList", oneof="kind"),
                        F("int64_list", 3, "msg", type_name=_P + "Int64List", oneof="kind")]),
        Msg("Features", [F("feature", 1, "map", type_name=("string", _P + "Feature"))]),
        Msg("Example", [F("features", 1, "msg", type_name=_P + "Features")]),
    ]
    _, classes, _ = build("bigdl_tf_example.proto", "tensorflow", msgs)
    return classes


_NP = {1: np.float32, 2: np.float64, 3: np.int32, 4: np.uint8, 5: np.int16, 6: np.int8, 9: np.int64, 10: np.bool_,
       17: np.uint16, 19: np.float16, 22: np.uint32, 23: np.uint64}
_TORCH = {np.float32: torch.float32, np.float64: torch.float64, np.int32: torch.int32, np.uint8: torch.uint8,
          np.int16: torch.int16, np.int8: torch.int8, np.int64: torch.int64, np.bool_: torch.bool,
          np.float16: torch.float16}
_VAL_FIELD = {1: "float_val", 2: "double_val", 3: "int_val", 4: "int_val", 5: "int_val", 6: "int_val", 9: "int64_val",
              10: "bool_val", 17: "int_val", 19: "half_val", 22: "uint32_val", 23: "uint64_val"}


def torch_dtype(dt: int):
    return _TORCH.get(_NP.get(dt % 100, np.float32), torch.float32)


def tensor_to_torch(tp, byte_order="little"):
    """TensorProto → torch tensor (strings → list of bytes)."""
    shape = [d.size for d in tp.tensor_shape.dim]
    dt = tp.dtype % 100
    if dt == 7:
        vals = list(tp.string_val)
        return vals if shape else (vals[0] if vals else b"")
    npt = _NP[dt]
    n = int(np.prod(shape)) if shape else 1
    if tp.tensor_content:
        arr = np.frombuffer(tp.tensor_content, dtype=np.dtype(npt).newbyteorder("<" if byte_order == "little" else ">"))
        arr = arr.astype(npt)
    else:
        vals = list(getattr(tp, _VAL_FIELD[dt]))
        if dt == 19:
            arr = np.array(vals, dtype=np.uint16).view(np.float16)
        else:
            arr = np.array(vals, dtype=npt)
        if arr.size == 0:
            arr = np.zeros(n, dtype=npt)
        elif arr.size < n:  # TF repeats the last value to fill the shape
            arr = np.concatenate([arr, np.full(n - arr.size, arr[-1], dtype=npt)])
    if npt == np.uint16:
        arr = arr.astype(np.int32)
    elif npt in (np.uint32, np.uint64):
        arr = arr.astype(np.int64)
    # (np.ascontiguousarray would turn a 0-d scalar into shape [1])
    return torch.from_numpy(np.array(arr.reshape(shape), copy=True, order="C"))


_DT_OF = {torch.float32: 1, torch.float64: 2, torch.int32: 3, torch.uint8: 4, torch.int16: 5, torch.int8: 6,
          torch.int64: 9, torch.bool: 10, torch.float16: 19}


def torch_to_tensor(t: torch.Tensor):
    classes, _ = graph_classes()
    tp = classes["tensorflow.TensorProto"]()
    t = t.detach().cpu()
    if t.dtype == torch.bfloat16:
        t = t.float()
    tp.dtype = _DT_OF[t.dtype]
    for s in t.shape:
        tp.tensor_shape.dim.add().size = int(s)
    tp.tensor_content = t.contiguous().numpy().tobytes()
    return tp
