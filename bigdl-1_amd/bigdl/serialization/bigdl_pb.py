"""The ``.bigdl`` model schema, re-declared with the reference's field numbers and types
(``spark/dl/src/main/resources/serialization/bigdl.proto``, package
``com.intel.analytics.bigdl.serialization``, proto3) so files are interchangeable."""
from __future__ import annotations

from .proto_builder import F, Msg, build

PKG = "com.intel.analytics.bigdl.serialization"
P = "." + PKG

_DATA_TYPES = [("INT32", 0), ("INT64", 1), ("FLOAT", 2), ("DOUBLE", 3), ("STRING", 4), ("BOOL", 5), ("CHAR", 6),
               ("SHORT", 7), ("BYTES", 8), ("REGULARIZER", 9), ("TENSOR", 10), ("VARIABLE_FORMAT", 11),
               ("INITMETHOD", 12), ("MODULE", 13), ("NAME_ATTR_LIST", 14), ("ARRAY_VALUE", 15),
               ("DATA_FORMAT", 16), ("CUSTOM", 17), ("SHAPE", 18)]

_ENUMS = [
    ("VarFormat", [("EMPTY_FORMAT", 0), ("DEFAULT", 1), ("ONE_D", 2), ("IN_OUT", 3), ("OUT_IN", 4),
                   ("IN_OUT_KW_KH", 5), ("OUT_IN_KW_KH", 6), ("GP_OUT_IN_KW_KH", 7), ("GP_IN_OUT_KW_KH", 8),
                   ("OUT_IN_KT_KH_KW", 9)]),
    ("InitMethodType", [("EMPTY_INITIALIZATION", 0), ("RANDOM_UNIFORM", 1), ("RANDOM_UNIFORM_PARAM", 2),
                        ("RANDOM_NORMAL", 3), ("ZEROS", 4), ("ONES", 5), ("CONST", 6), ("XAVIER", 7),
                        ("BILINEARFILLER", 8)]),
    ("RegularizerType", [("L1L2Regularizer", 0), ("L1Regularizer", 1), ("L2Regularizer", 2)]),
    ("InputDataFormat", [("NCHW", 0), ("NHWC", 1)]),
    ("TensorType", [("DENSE", 0), ("QUANT", 1)]),
    ("DataType", _DATA_TYPES),
]

_MODULE = Msg("BigDLModule", [
    F("name", 1, "string"),
    F("subModules", 2, "msg", "repeated", P + ".BigDLModule"),
    F("weight", 3, "msg", type_name=P + ".BigDLTensor"),
    F("bias", 4, "msg", type_name=P + ".BigDLTensor"),
    F("preModules", 5, "string", "repeated"),
    F("nextModules", 6, "string", "repeated"),
    F("moduleType", 7, "string"),
    F("attr", 8, "map", type_name=("string", P + ".AttrValue")),
    F("version", 9, "string"),
    F("train", 10, "bool"),
    F("namePostfix", 11, "string"),
    F("id", 12, "int32"),
    F("inputShape", 13, "msg", type_name=P + ".Shape"),
    F("outputShape", 14, "msg", type_name=P + ".Shape"),
    F("hasParameters", 15, "bool"),
    F("parameters", 16, "msg", "repeated", P + ".BigDLTensor"),
    F("isMklInt8Enabled", 17, "bool"),
    F("inputDimMasks", 18, "int32"),
    F("inputScales", 19, "msg", "repeated", P + ".AttrValue"),
    F("outputDimMasks", 20, "int32"),
    F("outputScales", 21, "msg", "repeated", P + ".AttrValue"),
    F("weightDimMasks", 22, "int32"),
    F("weightScales", 23, "msg", "repeated", P + ".AttrValue"),
])

_INIT = Msg("InitMethod", [F("methodType", 1, "enum", type_name=P + ".InitMethodType"),
                           F("data", 2, "double", "repeated")])

_TENSOR = Msg("BigDLTensor", [
    F("datatype", 1, "enum", type_name=P + ".DataType"),
    F("size", 2, "int32", "repeated"),
    F("stride", 3, "int32", "repeated"),
    F("offset", 4, "int32"),
    F("dimension", 5, "int32"),
    F("nElements", 6, "int32"),
    F("isScalar", 7, "bool"),
    F("storage", 8, "msg", type_name=P + ".TensorStorage"),
    F("id", 9, "int32"),
    F("tensorType", 10, "enum", type_name=P + ".TensorType"),
])

_STORAGE = Msg("TensorStorage", [
    F("datatype", 1, "enum", type_name=P + ".DataType"),
    F("float_data", 2, "float", "repeated"),
    F("double_data", 3, "double", "repeated"),
    F("bool_data", 4, "bool", "repeated"),
    F("string_data", 5, "string", "repeated"),
    F("int_data", 6, "int32", "repeated"),
    F("long_data", 7, "int64", "repeated"),
    F("bytes_data", 8, "bytes", "repeated"),
    F("id", 9, "int32"),
])

_REG = Msg("Regularizer", [F("regularizerType", 1, "enum", type_name=P + ".RegularizerType"),
                           F("regularData", 2, "double", "repeated")])

_ARRAY = Msg("ArrayValue", [
    F("size", 1, "int32"),
    F("datatype", 2, "enum", type_name=P + ".DataType"),
    F("i32", 3, "int32", "repeated"),
    F("i64", 4, "int64", "repeated"),
    F("flt", 5, "float", "repeated"),
    F("dbl", 6, "double", "repeated"),
    F("str", 7, "string", "repeated"),
    F("boolean", 8, "bool", "repeated"),
    F("Regularizer", 9, "msg", "repeated", P + ".Regularizer"),
    F("tensor", 10, "msg", "repeated", P + ".BigDLTensor"),
    F("variableFormat", 11, "enum", "repeated", P + ".VarFormat"),
    F("initMethod", 12, "msg", "repeated", P + ".InitMethod"),
    F("bigDLModule", 13, "msg", "repeated", P + ".BigDLModule"),
    F("nameAttrList", 14, "msg", "repeated", P + ".NameAttrList"),
    F("dataFormat", 15, "enum", "repeated", P + ".InputDataFormat"),
    F("custom", 16, "msg", "repeated", ".google.protobuf.Any"),
    F("shape", 17, "msg", "repeated", P + ".Shape"),
])

_ATTR = Msg("AttrValue", [
    F("dataType", 1, "enum", type_name=P + ".DataType"),
    F("subType", 2, "string"),
    F("int32Value", 3, "int32", oneof="value"),
    F("int64Value", 4, "int64", oneof="value"),
    F("floatValue", 5, "float", oneof="value"),
    F("doubleValue", 6, "double", oneof="value"),
    F("stringValue", 7, "string", oneof="value"),
    F("boolValue", 8, "bool", oneof="value"),
    F("regularizerValue", 9, "msg", type_name=P + ".Regularizer", oneof="value"),
    F("tensorValue", 10, "msg", type_name=P + ".BigDLTensor", oneof="value"),
    F("variableFormatValue", 11, "enum", type_name=P + ".VarFormat", oneof="value"),
    F("initMethodValue", 12, "msg", type_name=P + ".InitMethod", oneof="value"),
    F("bigDLModuleValue", 13, "msg", type_name=P + ".BigDLModule", oneof="value"),
    F("nameAttrListValue", 14, "msg", type_name=P + ".NameAttrList", oneof="value"),
    F("arrayValue", 15, "msg", type_name=P + ".AttrValue.ArrayValue", oneof="value"),
    F("dataFormatValue", 16, "enum", type_name=P + ".InputDataFormat", oneof="value"),
    F("customValue", 17, "msg", type_name=".google.protobuf.Any", oneof="value"),
    F("shape", 18, "msg", type_name=P + ".Shape", oneof="value"),
], nested=[_ARRAY])

_NAL = Msg("NameAttrList", [F("name", 1, "string"), F("attr", 2, "map", type_name=("string", P + ".AttrValue"))])

_SHAPE = Msg("Shape", [
    F("shapeType", 1, "enum", type_name=P + ".Shape.ShapeType"),
    F("ssize", 2, "int32"),
    F("shapeValue", 3, "int32", "repeated"),
    F("shape", 4, "msg", "repeated", P + ".Shape"),
], enums=[("ShapeType", [("SINGLE", 0), ("MULTI", 1)])])

POOL, CLASSES, ENUMS = build("bigdl_hip/bigdl.proto", PKG,
                             [_MODULE, _INIT, _TENSOR, _STORAGE, _REG, _ATTR, _NAL, _SHAPE], _ENUMS,
                             deps=["google/protobuf/any.proto"], syntax="proto3")

BigDLModule = CLASSES[PKG + ".BigDLModule"]
BigDLTensor = CLASSES[PKG + ".BigDLTensor"]
TensorStorage = CLASSES[PKG + ".TensorStorage"]
AttrValue = CLASSES[PKG + ".AttrValue"]
ArrayValue = CLASSES[PKG + ".AttrValue.ArrayValue"]
NameAttrList = CLASSES[PKG + ".NameAttrList"]
InitMethodPB = CLASSES[PKG + ".InitMethod"]
RegularizerPB = CLASSES[PKG + ".Regularizer"]
ShapePB = CLASSES[PKG + ".Shape"]
DataType = ENUMS["DataType"]
