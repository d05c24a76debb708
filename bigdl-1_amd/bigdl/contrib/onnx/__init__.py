"""ONNX model loader (``pyspark/bigdl/contrib/onnx/{onnx_loader,ops_mapping,ops_converter}.py``).

The ``onnx`` package is not required: ``ModelProto`` and friends are re-declared with ONNX's field
numbers (``onnx/onnx.proto3``) through :mod:`bigdl.serialization.proto_builder`, so ``.onnx`` files
parse with the protobuf runtime alone.  ``load(path)`` returns a BigDL ``Graph``: initializers
become layer weights (``Conv`` → ``SpatialConvolution``, ``Gemm``/``MatMul`` with constant B →
``Linear``, ``BatchNormalization`` → ``SpatialBatchNormalization`` with its running statistics,
``ConvTranspose`` → ``SpatialFullConvolution``), the rest map to BigDL layers or forward-only ops.
``helper`` builds ModelProtos (the ``onnx.helper`` subset the tests and exporters need).
"""
from __future__ import annotations

import functools
import math
from typing import Dict, List

import numpy as np
import torch
import torch.nn.functional as F

from ...serialization.proto_builder import F as Fd, Msg, build
from ...utils.table import Table

_P = ".onnx."
_DT = [("UNDEFINED", 0), ("FLOAT", 1), ("UINT8", 2), ("INT8", 3), ("UINT16", 4), ("INT16", 5), ("INT32", 6),
       ("INT64", 7), ("STRING", 8), ("BOOL", 9), ("FLOAT16", 10), ("DOUBLE", 11), ("UINT32", 12), ("UINT64", 13),
       ("COMPLEX64", 14), ("COMPLEX128", 15), ("BFLOAT16", 16)]
_AT = [("UNDEFINED", 0), ("FLOAT", 1), ("INT", 2), ("STRING", 3), ("TENSOR", 4), ("GRAPH", 5), ("FLOATS", 6),
       ("INTS", 7), ("STRINGS", 8), ("TENSORS", 9), ("GRAPHS", 10)]


@functools.lru_cache(None)
def onnx_classes():
    msgs = [
        Msg("TensorProto", [
            Fd("dims", 1, "int64", "repeated", packed=True), Fd("data_type", 2, "int32"),
            Fd("float_data", 4, "float", "repeated", packed=True), Fd("int32_data", 5, "int32", "repeated", packed=True),
            Fd("string_data", 6, "bytes", "repeated"), Fd("int64_data", 7, "int64", "repeated", packed=True),
            Fd("name", 8, "string"), Fd("raw_data", 9, "bytes"), Fd("double_data", 10, "double", "repeated", packed=True),
            Fd("uint64_data", 11, "uint64", "repeated", packed=True), Fd("doc_string", 12, "string")]),
        Msg("AttributeProto", [
            Fd("name", 1, "string"), Fd("f", 2, "float"), Fd("i", 3, "int64"), Fd("s", 4, "bytes"),
            Fd("t", 5, "msg", type_name=_P + "TensorProto"), Fd("g", 6, "msg", type_name=_P + "GraphProto"),
            Fd("floats", 7, "float", "repeated", packed=True), Fd("ints", 8, "int64", "repeated", packed=True),
            Fd("strings", 9, "bytes", "repeated"), Fd("tensors", 10, "msg", "repeated", type_name=_P + "TensorProto"),
            Fd("doc_string", 13, "string"), Fd("type", 20, "enum", type_name=_P + "AttributeProto.AttributeType")],
            enums=[("AttributeType", _AT)]),
        Msg("NodeProto", [Fd("input", 1, "string", "repeated"), Fd("output", 2, "string", "repeated"),
                          Fd("name", 3, "string"), Fd("op_type", 4, "string"),
                          Fd("attribute", 5, "msg", "repeated", type_name=_P + "AttributeProto"),
                          Fd("doc_string", 6, "string"), Fd("domain", 7, "string")]),
        Msg("TensorShapeProto", [Fd("dim", 1, "msg", "repeated", type_name=_P + "TensorShapeProto.Dimension")],
            nested=[Msg("Dimension", [Fd("dim_value", 1, "int64", oneof="value"),
                                      Fd("dim_param", 2, "string", oneof="value"), Fd("denotation", 3, "string")])]),
        Msg("TypeProto", [Fd("tensor_type", 1, "msg", type_name=_P + "TypeProto.Tensor", oneof="value"),
                          Fd("denotation", 6, "string")],
            nested=[Msg("Tensor", [Fd("elem_type", 1, "int32"),
                                   Fd("shape", 2, "msg", type_name=_P + "TensorShapeProto")])]),
        Msg("ValueInfoProto", [Fd("name", 1, "string"), Fd("type", 2, "msg", type_name=_P + "TypeProto"),
                               Fd("doc_string", 3, "string")]),
        Msg("GraphProto", [Fd("node", 1, "msg", "repeated", type_name=_P + "NodeProto"), Fd("name", 2, "string"),
                           Fd("initializer", 5, "msg", "repeated", type_name=_P + "TensorProto"),
                           Fd("doc_string", 10, "string"),
                           Fd("input", 11, "msg", "repeated", type_name=_P + "ValueInfoProto"),
                           Fd("output", 12, "msg", "repeated", type_name=_P + "ValueInfoProto"),
                           Fd("value_info", 13, "msg", "repeated", type_name=_P + "ValueInfoProto")]),
        Msg("OperatorSetIdProto", [Fd("domain", 1, "string"), Fd("version", 2, "int64")]),
        Msg("ModelProto", [Fd("ir_version", 1, "int64"), Fd("producer_name", 2, "string"),
                           Fd("producer_version", 3, "string"), Fd("domain", 4, "string"),
                           Fd("model_version", 5, "int64"), Fd("doc_string", 6, "string"),
                           Fd("graph", 7, "msg", type_name=_P + "GraphProto"),
                           Fd("opset_import", 8, "msg", "repeated", type_name=_P + "OperatorSetIdProto")]),
    ]
    _, classes, enums = build("bigdl_onnx.proto", "onnx", msgs, enums=[("DataType", _DT)])
    return classes


_NP = {1: np.float32, 2: np.uint8, 3: np.int8, 5: np.int16, 6: np.int32, 7: np.int64, 9: np.bool_, 10: np.float16,
       11: np.float64, 4: np.uint16, 12: np.uint32, 13: np.uint64}


def to_array(t) -> np.ndarray:
    """TensorProto → numpy (``converter_utils.parse_tensor_data``)."""
    dt = _NP[t.data_type]
    shape = list(t.dims)
    if t.raw_data:
        a = np.frombuffer(t.raw_data, dtype=np.dtype(dt).newbyteorder("<")).astype(dt)
    elif t.data_type in (1,):
        a = np.array(t.float_data, dtype=dt)
    elif t.data_type == 11:
        a = np.array(t.double_data, dtype=dt)
    elif t.data_type in (7,):
        a = np.array(t.int64_data, dtype=dt)
    elif t.data_type in (12, 13):
        a = np.array(t.uint64_data, dtype=dt)
    elif t.data_type == 10:
        a = np.array(t.int32_data, dtype=np.uint16).view(np.float16)
    else:
        a = np.array(t.int32_data, dtype=dt)
    return a.reshape(shape)


class helper:
    """Builders for ONNX protos (the ``onnx.helper`` subset)."""

    @staticmethod
    def make_tensor(name, array) -> object:
        a = np.ascontiguousarray(np.asarray(array))
        rev = {np.dtype(v): k for k, v in _NP.items()}
        t = onnx_classes()["onnx.TensorProto"]()
        t.name = name
        t.data_type = rev[a.dtype]
        t.dims.extend(a.shape)
        t.raw_data = a.astype(a.dtype.newbyteorder("<")).tobytes()
        return t

    @staticmethod
    def make_node(op_type, inputs, outputs, name="", **attrs):
        C = onnx_classes()
        n = C["onnx.NodeProto"]()
        n.op_type, n.name = op_type, name or (outputs[0] if outputs else op_type)
        n.input.extend(inputs)
        n.output.extend(outputs)
        for k, v in sorted(attrs.items()):
            a = n.attribute.add()
            a.name = k
            if isinstance(v, bool) or isinstance(v, (int, np.integer)):
                a.i, a.type = int(v), 2
            elif isinstance(v, float):
                a.f, a.type = v, 1
            elif isinstance(v, str):
                a.s, a.type = v.encode(), 3
            elif isinstance(v, (list, tuple)) and all(isinstance(x, (int, np.integer)) for x in v):
                a.ints.extend(int(x) for x in v)
                a.type = 7
            elif isinstance(v, (list, tuple)):
                a.floats.extend(float(x) for x in v)
                a.type = 6
            else:
                a.t.CopyFrom(v)
                a.type = 4
        return n

    @staticmethod
    def make_value_info(name, shape, elem_type=1):
        v = onnx_classes()["onnx.ValueInfoProto"]()
        v.name = name
        v.type.tensor_type.elem_type = elem_type
        for d in shape:
            dim = v.type.tensor_type.shape.dim.add()
            if isinstance(d, str):
                dim.dim_param = d
            else:
                dim.dim_value = int(d)
        return v

    @staticmethod
    def make_graph(nodes, name, inputs, outputs, initializer=()):
        g = onnx_classes()["onnx.GraphProto"]()
        g.name = name
        g.node.extend(nodes)
        g.input.extend(inputs)
        g.output.extend(outputs)
        g.initializer.extend(initializer)
        return g

    @staticmethod
    def make_model(graph, opset=11):
        m = onnx_classes()["onnx.ModelProto"]()
        m.ir_version = 6
        m.producer_name = "bigdl"
        m.graph.CopyFrom(graph)
        o = m.opset_import.add()
        o.version = opset
        return m


def _attrs(node) -> Dict[str, object]:
    out = {}
    for a in node.attribute:
        t = a.type
        if t == 1:
            out[a.name] = a.f
        elif t == 2:
            out[a.name] = int(a.i)
        elif t == 3:
            out[a.name] = a.s.decode()
        elif t == 4:
            out[a.name] = to_array(a.t)
        elif t == 6:
            out[a.name] = list(a.floats)
        elif t == 7:
            out[a.name] = [int(x) for x in a.ints]
        elif t == 8:
            out[a.name] = [s.decode() for s in a.strings]
        else:  # untyped (old exporters): infer from the populated field
            for f in ("ints", "floats"):
                if len(getattr(a, f)):
                    out[a.name] = list(getattr(a, f))
                    break
            else:
                out[a.name] = a.i if a.i else (a.f if a.f else (a.s.decode() if a.s else None))
    return out


from .loader import OnnxLoader, load, load_model_proto  # noqa: E402,F401
