"""Build protobuf message classes from a compact Python schema description (no protoc needed).

The image has the protobuf runtime but no ``protoc``; the reference's schemas
(``RES/serialization/bigdl.proto``, ``spark/dl/src/main/resources/caffe/caffe.proto``) are
re-declared in Python with the SAME field numbers / types, turned into a ``FileDescriptorProto`` and
registered in a private descriptor pool.  Binary and text formats are then handled by the
protobuf runtime (``SerializeToString``, ``ParseFromString``, ``text_format.Merge``).

Schema DSL::

    F(name, number, type, label="optional", type_name=None, default=None, packed=None, oneof=None)

``type`` is a scalar name ('int32', 'float', 'string', 'bytes', 'bool', 'int64', 'uint32', 'double',
'uint64', 'sint32', 'fixed32'…) or 'msg'/'enum' with ``type_name``; ``map(K, V)`` fields are
given as ``type='map', type_name=(key_type, value_type_or_typename)``.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

FDP = descriptor_pb2.FieldDescriptorProto

_SCALARS = {
    "double": FDP.TYPE_DOUBLE, "float": FDP.TYPE_FLOAT, "int64": FDP.TYPE_INT64, "uint64": FDP.TYPE_UINT64,
    "int32": FDP.TYPE_INT32, "fixed64": FDP.TYPE_FIXED64, "fixed32": FDP.TYPE_FIXED32, "bool": FDP.TYPE_BOOL,
    "string": FDP.TYPE_STRING, "bytes": FDP.TYPE_BYTES, "uint32": FDP.TYPE_UINT32, "sfixed32": FDP.TYPE_SFIXED32,
    "sfixed64": FDP.TYPE_SFIXED64, "sint32": FDP.TYPE_SINT32, "sint64": FDP.TYPE_SINT64,
}
_LABELS = {"optional": FDP.LABEL_OPTIONAL, "repeated": FDP.LABEL_REPEATED, "required": FDP.LABEL_REQUIRED}


class F:
    __slots__ = ("name", "number", "type", "label", "type_name", "default", "packed", "oneof")

    def __init__(self, name, number, type, label="optional", type_name=None, default=None, packed=None,
                 oneof=None):
        self.name, self.number, self.type, self.label = name, number, type, label
        self.type_name, self.default, self.packed, self.oneof = type_name, default, packed, oneof


class Msg:
    def __init__(self, name: str, fields: List[F], nested: Optional[List["Msg"]] = None,
                 enums: Optional[List[Tuple[str, List[Tuple[str, int]]]]] = None):
        self.name, self.fields = name, fields
        self.nested = nested or []
        self.enums = enums or []


def _camel(s: str) -> str:
    return "".join(p[:1].upper() + p[1:] for p in s.split("_"))


def _fill_msg(dp: descriptor_pb2.DescriptorProto, m: Msg, package: str, scope: str, syntax: str):
    dp.name = m.name
    for en, vals in m.enums:
        e = dp.enum_type.add()
        e.name = en
        for vn, vv in vals:
            v = e.value.add()
            v.name, v.number = vn, vv
    for n in m.nested:
        _fill_msg(dp.nested_type.add(), n, package, f"{scope}.{m.name}", syntax)
    oneofs: Dict[str, int] = {}
    for f in m.fields:
        fd = dp.field.add()
        fd.name, fd.number = f.name, f.number
        fd.json_name = f.name
        if f.type == "map":
            kt, vt = f.type_name
            entry = dp.nested_type.add()
            entry.name = _camel(f.name) + "Entry"
            entry.options.map_entry = True
            k = entry.field.add()
            k.name, k.number, k.label, k.type = "key", 1, FDP.LABEL_OPTIONAL, _SCALARS[kt]
            v = entry.field.add()
            v.name, v.number, v.label = "value", 2, FDP.LABEL_OPTIONAL
            if vt in _SCALARS:
                v.type = _SCALARS[vt]
            else:
                v.type = FDP.TYPE_MESSAGE
                v.type_name = vt
            fd.label = FDP.LABEL_REPEATED
            fd.type = FDP.TYPE_MESSAGE
            fd.type_name = f"{scope}.{m.name}.{entry.name}"
            continue
        fd.label = _LABELS[f.label]
        if f.type in _SCALARS:
            fd.type = _SCALARS[f.type]
        elif f.type == "msg":
            fd.type = FDP.TYPE_MESSAGE
            fd.type_name = f.type_name
        elif f.type == "enum":
            fd.type = FDP.TYPE_ENUM
            fd.type_name = f.type_name
        else:
            raise ValueError(f"bad field type {f.type}")
        if f.default is not None and syntax == "proto2":
            if isinstance(f.default, bool):
                fd.default_value = "true" if f.default else "false"
            else:
                fd.default_value = str(f.default)
        if f.packed is not None:
            fd.options.packed = bool(f.packed)
        if f.oneof:
            if f.oneof not in oneofs:
                oneofs[f.oneof] = len(dp.oneof_decl)
                dp.oneof_decl.add().name = f.oneof
            fd.oneof_index = oneofs[f.oneof]
        if syntax == "proto3" and f.label == "optional" and f.oneof is None:
            pass


def build(file_name: str, package: str, messages: List[Msg], enums=(), deps=(), syntax="proto3",
          pool: Optional[descriptor_pool.DescriptorPool] = None):
    """Returns (pool, {full_name: message_class}, {enum_name: {value_name: number}})."""
    pool = pool or descriptor_pool.DescriptorPool()
    fdp = descriptor_pb2.FileDescriptorProto()
    fdp.name = file_name
    fdp.package = package
    fdp.syntax = syntax
    for d in deps:
        fdp.dependency.append(d)
    scope = "." + package
    for en, vals in enums:
        e = fdp.enum_type.add()
        e.name = en
        for vn, vv in vals:
            v = e.value.add()
            v.name, v.number = vn, vv
    for m in messages:
        _fill_msg(fdp.message_type.add(), m, package, scope, syntax)
    if "google/protobuf/any.proto" in deps:
        from google.protobuf import any_pb2
        try:
            pool.FindFileByName("google/protobuf/any.proto")
        except KeyError:
            pool.Add(descriptor_pb2.FileDescriptorProto.FromString(any_pb2.DESCRIPTOR.serialized_pb))
    pool.Add(fdp)
    classes = {}

    def collect(desc):
        classes[desc.full_name] = message_factory.GetMessageClass(desc)
        for n in desc.nested_types:
            if not n.GetOptions().map_entry:
                collect(n)
    fd = pool.FindFileByName(file_name)
    for name in fd.message_types_by_name:
        collect(fd.message_types_by_name[name])
    enum_vals = {}
    for name, ed in fd.enum_types_by_name.items():
        enum_vals[name] = {v.name: v.number for v in ed.values}
    return pool, classes, enum_vals
