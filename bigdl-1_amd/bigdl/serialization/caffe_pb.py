"""The subset of ``caffe.proto`` (package ``caffe``, proto2) the Caffe loader/persister needs,
re-declared with the upstream field numbers, types and defaults so ``.prototxt`` text and
``.caffemodel`` binaries parse with the stock protobuf runtime (``CaffeLoader.scala:85-195``
reads both into ``NetParameter``).  Messages the loader only needs to *skip* are declared with
their scalar fields so text-format files that set them still parse."""
from __future__ import annotations

from .proto_builder import F, Msg, build

PKG = "caffe"
P = ".caffe"


def _eng(n):
    return F("engine", n, "enum", type_name=P + ".Engine", default="DEFAULT")


_FILLER = Msg("FillerParameter", [
    F("type", 1, "string", default="constant"), F("value", 2, "float", default=0.0),
    F("min", 3, "float", default=0.0), F("max", 4, "float", default=1.0), F("mean", 5, "float", default=0.0),
    F("std", 6, "float", default=1.0), F("sparse", 7, "int32", default=-1),
    F("variance_norm", 8, "enum", type_name=P + ".FillerParameter.VarianceNorm", default="FAN_IN"),
], enums=[("VarianceNorm", [("FAN_IN", 0), ("FAN_OUT", 1), ("AVERAGE", 2)])])

_BLOB_SHAPE = Msg("BlobShape", [F("dim", 1, "int64", "repeated", packed=True)])
_BLOB = Msg("BlobProto", [
    F("shape", 7, "msg", type_name=P + ".BlobShape"), F("data", 5, "float", "repeated", packed=True),
    F("diff", 6, "float", "repeated", packed=True), F("double_data", 8, "double", "repeated", packed=True),
    F("double_diff", 9, "double", "repeated", packed=True), F("num", 1, "int32", default=0),
    F("channels", 2, "int32", default=0), F("height", 3, "int32", default=0), F("width", 4, "int32", default=0),
])
_NET_STATE = Msg("NetState", [F("phase", 1, "enum", type_name=P + ".Phase", default="TEST"),
                              F("level", 2, "int32", default=0), F("stage", 3, "string", "repeated")])
_RULE = Msg("NetStateRule", [F("phase", 1, "enum", type_name=P + ".Phase"), F("min_level", 2, "int32"),
                             F("max_level", 3, "int32"), F("stage", 4, "string", "repeated"),
                             F("not_stage", 5, "string", "repeated")])
_PARAM_SPEC = Msg("ParamSpec", [
    F("name", 1, "string"), F("share_mode", 2, "enum", type_name=P + ".ParamSpec.DimCheckMode"),
    F("lr_mult", 3, "float", default=1.0), F("decay_mult", 4, "float", default=1.0),
], enums=[("DimCheckMode", [("STRICT", 0), ("PERMISSIVE", 1)])])

_NET = Msg("NetParameter", [
    F("name", 1, "string"), F("input", 3, "string", "repeated"),
    F("input_shape", 8, "msg", "repeated", P + ".BlobShape"), F("input_dim", 4, "int32", "repeated"),
    F("force_backward", 5, "bool", default=False), F("state", 6, "msg", type_name=P + ".NetState"),
    F("debug_info", 7, "bool", default=False), F("layer", 100, "msg", "repeated", P + ".LayerParameter"),
    F("layers", 2, "msg", "repeated", P + ".V1LayerParameter"),
])

# ---------------------------------------------------------------------------------- layer params
_CONV = Msg("ConvolutionParameter", [
    F("num_output", 1, "uint32"), F("bias_term", 2, "bool", default=True), F("pad", 3, "uint32", "repeated"),
    F("kernel_size", 4, "uint32", "repeated"), F("stride", 6, "uint32", "repeated"),
    F("dilation", 18, "uint32", "repeated"), F("pad_h", 9, "uint32", default=0), F("pad_w", 10, "uint32", default=0),
    F("kernel_h", 11, "uint32"), F("kernel_w", 12, "uint32"), F("stride_h", 13, "uint32"), F("stride_w", 14, "uint32"),
    F("group", 5, "uint32", default=1), F("weight_filler", 7, "msg", type_name=P + ".FillerParameter"),
    F("bias_filler", 8, "msg", type_name=P + ".FillerParameter"), _eng(15), F("axis", 16, "int32", default=1),
    F("force_nd_im2col", 17, "bool", default=False),
])
_POOL = Msg("PoolingParameter", [
    F("pool", 1, "enum", type_name=P + ".PoolingParameter.PoolMethod", default="MAX"),
    F("pad", 4, "uint32", default=0), F("pad_h", 9, "uint32", default=0), F("pad_w", 10, "uint32", default=0),
    F("kernel_size", 2, "uint32"), F("kernel_h", 5, "uint32"), F("kernel_w", 6, "uint32"),
    F("stride", 3, "uint32", default=1), F("stride_h", 7, "uint32"), F("stride_w", 8, "uint32"), _eng(11),
    F("global_pooling", 12, "bool", default=False),
], enums=[("PoolMethod", [("MAX", 0), ("AVE", 1), ("STOCHASTIC", 2)])])
_IP = Msg("InnerProductParameter", [
    F("num_output", 1, "uint32"), F("bias_term", 2, "bool", default=True),
    F("weight_filler", 3, "msg", type_name=P + ".FillerParameter"),
    F("bias_filler", 4, "msg", type_name=P + ".FillerParameter"), F("axis", 5, "int32", default=1),
    F("transpose", 6, "bool", default=False),
])
_LRN = Msg("LRNParameter", [
    F("local_size", 1, "uint32", default=5), F("alpha", 2, "float", default=1.0), F("beta", 3, "float", default=0.75),
    F("norm_region", 4, "enum", type_name=P + ".LRNParameter.NormRegion", default="ACROSS_CHANNELS"),
    F("k", 5, "float", default=1.0), _eng(6),
], enums=[("NormRegion", [("ACROSS_CHANNELS", 0), ("WITHIN_CHANNEL", 1)])])
_ELTWISE = Msg("EltwiseParameter", [
    F("operation", 1, "enum", type_name=P + ".EltwiseParameter.EltwiseOp", default="SUM"),
    F("coeff", 2, "float", "repeated"), F("stable_prod_grad", 3, "bool", default=True),
], enums=[("EltwiseOp", [("PROD", 0), ("SUM", 1), ("MAX", 2)])])


def _simple(name, fields):
    return Msg(name, fields)


_SIMPLE = [
    _simple("DropoutParameter", [F("dropout_ratio", 1, "float", default=0.5)]),
    _simple("SoftmaxParameter", [_eng(1), F("axis", 2, "int32", default=1)]),
    _simple("ConcatParameter", [F("axis", 2, "int32", default=1), F("concat_dim", 1, "uint32", default=1)]),
    _simple("BatchNormParameter", [F("use_global_stats", 1, "bool"),
                                   F("moving_average_fraction", 2, "float", default=0.999),
                                   F("eps", 3, "float", default=1e-5)]),
    _simple("ScaleParameter", [F("axis", 1, "int32", default=1), F("num_axes", 2, "int32", default=1),
                               F("filler", 3, "msg", type_name=P + ".FillerParameter"),
                               F("bias_term", 4, "bool", default=False),
                               F("bias_filler", 5, "msg", type_name=P + ".FillerParameter")]),
    _simple("BiasParameter", [F("axis", 1, "int32", default=1), F("num_axes", 2, "int32", default=1),
                              F("filler", 3, "msg", type_name=P + ".FillerParameter")]),
    _simple("ReLUParameter", [F("negative_slope", 1, "float", default=0.0), _eng(2)]),
    _simple("PReLUParameter", [F("filler", 1, "msg", type_name=P + ".FillerParameter"),
                               F("channel_shared", 2, "bool", default=False)]),
    _simple("ELUParameter", [F("alpha", 1, "float", default=1.0)]),
    _simple("PowerParameter", [F("power", 1, "float", default=1.0), F("scale", 2, "float", default=1.0),
                               F("shift", 3, "float", default=0.0)]),
    _simple("ExpParameter", [F("base", 1, "float", default=-1.0), F("scale", 2, "float", default=1.0),
                             F("shift", 3, "float", default=0.0)]),
    _simple("LogParameter", [F("base", 1, "float", default=-1.0), F("scale", 2, "float", default=1.0),
                             F("shift", 3, "float", default=0.0)]),
    _simple("ReshapeParameter", [F("shape", 1, "msg", type_name=P + ".BlobShape"), F("axis", 2, "int32", default=0),
                                 F("num_axes", 3, "int32", default=-1)]),
    _simple("FlattenParameter", [F("axis", 1, "int32", default=1), F("end_axis", 2, "int32", default=-1)]),
    _simple("SliceParameter", [F("axis", 3, "int32", default=1), F("slice_point", 2, "uint32", "repeated"),
                               F("slice_dim", 1, "uint32", default=1)]),
    _simple("TileParameter", [F("axis", 1, "int32", default=1), F("tiles", 2, "int32")]),
    _simple("ThresholdParameter", [F("threshold", 1, "float", default=0.0)]),
    _simple("InputParameter", [F("shape", 1, "msg", "repeated", P + ".BlobShape")]),
    _simple("TanhParameter", [_eng(1)]),
    _simple("SigmoidParameter", [_eng(1)]),
    _simple("RecurrentParameter", [F("num_output", 1, "uint32", default=0),
                                   F("weight_filler", 2, "msg", type_name=P + ".FillerParameter"),
                                   F("bias_filler", 3, "msg", type_name=P + ".FillerParameter"),
                                   F("debug_info", 4, "bool", default=False),
                                   F("expose_hidden", 5, "bool", default=False)]),
    _simple("DummyDataParameter", [F("data_filler", 1, "msg", "repeated", P + ".FillerParameter"),
                                   F("shape", 6, "msg", "repeated", P + ".BlobShape"),
                                   F("num", 2, "uint32", "repeated"), F("channels", 3, "uint32", "repeated"),
                                   F("height", 4, "uint32", "repeated"), F("width", 5, "uint32", "repeated")]),
    _simple("TransformationParameter", [F("scale", 1, "float", default=1.0), F("mirror", 2, "bool", default=False),
                                        F("crop_size", 3, "uint32", default=0), F("mean_file", 4, "string"),
                                        F("mean_value", 5, "float", "repeated"), F("force_color", 6, "bool"),
                                        F("force_gray", 7, "bool")]),
    _simple("LossParameter", [F("ignore_label", 1, "int32"), F("normalization", 3, "int32"),
                              F("normalize", 2, "bool")]),
    _simple("AccuracyParameter", [F("top_k", 1, "uint32", default=1), F("axis", 2, "int32", default=1),
                                  F("ignore_label", 3, "int32")]),
    _simple("ArgMaxParameter", [F("out_max_val", 1, "bool"), F("top_k", 2, "uint32", default=1),
                                F("axis", 3, "int32")]),
    _simple("CropParameter", [F("axis", 1, "int32", default=2), F("offset", 2, "uint32", "repeated")]),
    _simple("DataParameter", [F("source", 1, "string"), F("batch_size", 4, "uint32"), F("rand_skip", 7, "uint32"),
                              F("backend", 8, "int32"), F("scale", 2, "float", default=1.0),
                              F("mean_file", 3, "string"), F("crop_size", 5, "uint32"), F("mirror", 6, "bool"),
                              F("force_encoded_color", 9, "bool"), F("prefetch", 10, "uint32", default=4)]),
    _simple("ImageDataParameter", [F("source", 1, "string"), F("batch_size", 4, "uint32", default=1),
                                   F("rand_skip", 7, "uint32"), F("shuffle", 8, "bool"), F("new_height", 9, "uint32"),
                                   F("new_width", 10, "uint32"), F("is_color", 11, "bool", default=True),
                                   F("scale", 2, "float", default=1.0), F("mean_file", 3, "string"),
                                   F("crop_size", 5, "uint32"), F("mirror", 6, "bool"),
                                   F("root_folder", 12, "string")]),
    _simple("MemoryDataParameter", [F("batch_size", 1, "uint32"), F("channels", 2, "uint32"),
                                    F("height", 3, "uint32"), F("width", 4, "uint32")]),
    _simple("InfogainLossParameter", [F("source", 1, "string")]),
    _simple("HingeLossParameter", [F("norm", 1, "int32", default=1)]),
    _simple("ContrastiveLossParameter", [F("margin", 1, "float", default=1.0), F("legacy_version", 2, "bool")]),
    _simple("MVNParameter", [F("normalize_variance", 1, "bool", default=True), F("across_channels", 2, "bool"),
                             F("eps", 3, "float", default=1e-9)]),
    _simple("ReductionParameter", [F("operation", 1, "int32", default=1), F("axis", 2, "int32", default=0),
                                   F("coeff", 3, "float", default=1.0)]),
    _simple("EmbedParameter", [F("num_output", 1, "uint32"), F("input_dim", 2, "uint32"),
                               F("bias_term", 3, "bool", default=True),
                               F("weight_filler", 4, "msg", type_name=P + ".FillerParameter"),
                               F("bias_filler", 5, "msg", type_name=P + ".FillerParameter")]),
    _simple("ROIPoolingParameter", [F("pooled_h", 1, "uint32"), F("pooled_w", 2, "uint32"),
                                    F("spatial_scale", 3, "float", default=1.0)]),
    _simple("ProposalParameter", [F("feat_stride", 1, "uint32", default=16), F("base_size", 2, "uint32", default=16),
                                  F("min_size", 3, "uint32", default=16), F("ratio", 4, "float", "repeated"),
                                  F("scale", 5, "float", "repeated"), F("pre_nms_topn", 6, "uint32", default=6000),
                                  F("post_nms_topn", 7, "uint32", default=300),
                                  F("nms_thresh", 8, "float", default=0.7)]),
    _simple("SmoothL1LossParameter", [F("sigma", 1, "float", default=1.0)]),
    _simple("PythonParameter", [F("module", 1, "string"), F("layer", 2, "string"), F("param_str", 3, "string"),
                                F("share_in_parallel", 4, "bool")]),
    _simple("ParameterParameter", [F("shape", 1, "msg", type_name=P + ".BlobShape")]),
    _simple("HDF5DataParameter", [F("source", 1, "string"), F("batch_size", 2, "uint32"), F("shuffle", 3, "bool")]),
    _simple("HDF5OutputParameter", [F("file_name", 1, "string")]),
    _simple("SPPParameter", [F("pyramid_height", 1, "uint32"), F("pool", 2, "int32"), _eng(6)]),
    _simple("WindowDataParameter", [F("source", 1, "string"), F("scale", 2, "float", default=1.0),
                                    F("mean_file", 3, "string"), F("batch_size", 4, "uint32"),
                                    F("crop_size", 5, "uint32"), F("mirror", 6, "bool"),
                                    F("fg_threshold", 7, "float", default=0.5),
                                    F("bg_threshold", 8, "float", default=0.5),
                                    F("fg_fraction", 9, "float", default=0.25), F("context_pad", 10, "uint32"),
                                    F("crop_mode", 11, "string", default="warp"), F("cache_images", 12, "bool"),
                                    F("root_folder", 13, "string")]),
]

# name → (V2 field number, V1 field number or None)
_LAYER_PARAMS = {
    "transform_param": ("TransformationParameter", 100, 36), "loss_param": ("LossParameter", 101, 42),
    "accuracy_param": ("AccuracyParameter", 102, 27), "argmax_param": ("ArgMaxParameter", 103, 23),
    "batch_norm_param": ("BatchNormParameter", 139, None), "bias_param": ("BiasParameter", 141, None),
    "concat_param": ("ConcatParameter", 104, 9), "contrastive_loss_param": ("ContrastiveLossParameter", 105, 40),
    "convolution_param": ("ConvolutionParameter", 106, 10), "crop_param": ("CropParameter", 144, None),
    "data_param": ("DataParameter", 107, 11), "dropout_param": ("DropoutParameter", 108, 12),
    "dummy_data_param": ("DummyDataParameter", 109, 26), "eltwise_param": ("EltwiseParameter", 110, 24),
    "elu_param": ("ELUParameter", 140, None), "embed_param": ("EmbedParameter", 137, None),
    "exp_param": ("ExpParameter", 111, 41), "flatten_param": ("FlattenParameter", 135, None),
    "hdf5_data_param": ("HDF5DataParameter", 112, 13), "hdf5_output_param": ("HDF5OutputParameter", 113, 14),
    "hinge_loss_param": ("HingeLossParameter", 114, 29), "image_data_param": ("ImageDataParameter", 115, 15),
    "infogain_loss_param": ("InfogainLossParameter", 116, 16),
    "inner_product_param": ("InnerProductParameter", 117, 17), "input_param": ("InputParameter", 143, None),
    "log_param": ("LogParameter", 134, None), "lrn_param": ("LRNParameter", 118, 18),
    "memory_data_param": ("MemoryDataParameter", 119, 22), "mvn_param": ("MVNParameter", 120, 34),
    "parameter_param": ("ParameterParameter", 145, None), "pooling_param": ("PoolingParameter", 121, 19),
    "power_param": ("PowerParameter", 122, 21), "prelu_param": ("PReLUParameter", 131, None),
    "python_param": ("PythonParameter", 130, None), "recurrent_param": ("RecurrentParameter", 146, None),
    "reduction_param": ("ReductionParameter", 136, None), "relu_param": ("ReLUParameter", 123, 30),
    "reshape_param": ("ReshapeParameter", 133, None), "scale_param": ("ScaleParameter", 142, None),
    "sigmoid_param": ("SigmoidParameter", 124, 38), "softmax_param": ("SoftmaxParameter", 125, 39),
    "spp_param": ("SPPParameter", 132, None), "slice_param": ("SliceParameter", 126, 31),
    "tanh_param": ("TanhParameter", 127, 37), "threshold_param": ("ThresholdParameter", 128, 25),
    "tile_param": ("TileParameter", 138, None), "window_data_param": ("WindowDataParameter", 129, 20),
    "roi_pooling_param": ("ROIPoolingParameter", 8266711, None),
    "smooth_l1_loss_param": ("SmoothL1LossParameter", 8266712, None),
    "proposal_param": ("ProposalParameter", 8266713, None),
}

_LAYER = Msg("LayerParameter", [
    F("name", 1, "string"), F("type", 2, "string"), F("bottom", 3, "string", "repeated"),
    F("top", 4, "string", "repeated"), F("phase", 10, "enum", type_name=P + ".Phase"),
    F("loss_weight", 5, "float", "repeated"), F("param", 6, "msg", "repeated", P + ".ParamSpec"),
    F("blobs", 7, "msg", "repeated", P + ".BlobProto"), F("propagate_down", 11, "bool", "repeated"),
    F("include", 8, "msg", "repeated", P + ".NetStateRule"), F("exclude", 9, "msg", "repeated", P + ".NetStateRule"),
] + [F(k, v[1], "msg", type_name=f"{P}.{v[0]}") for k, v in _LAYER_PARAMS.items()])

V1_TYPES = [("NONE", 0), ("ABSVAL", 35), ("ACCURACY", 1), ("ARGMAX", 30), ("BNLL", 2), ("CONCAT", 3),
            ("CONTRASTIVE_LOSS", 37), ("CONVOLUTION", 4), ("DATA", 5), ("DECONVOLUTION", 39), ("DROPOUT", 6),
            ("DUMMY_DATA", 32), ("EUCLIDEAN_LOSS", 7), ("ELTWISE", 25), ("EXP", 38), ("FLATTEN", 8),
            ("HDF5_DATA", 9), ("HDF5_OUTPUT", 10), ("HINGE_LOSS", 28), ("IM2COL", 11), ("IMAGE_DATA", 12),
            ("INFOGAIN_LOSS", 13), ("INNER_PRODUCT", 14), ("LRN", 15), ("MEMORY_DATA", 29),
            ("MULTINOMIAL_LOGISTIC_LOSS", 16), ("MVN", 34), ("POOLING", 17), ("POWER", 26), ("RELU", 18),
            ("SIGMOID", 19), ("SIGMOID_CROSS_ENTROPY_LOSS", 27), ("SILENCE", 36), ("SOFTMAX", 20),
            ("SOFTMAX_LOSS", 21), ("SPLIT", 22), ("SLICE", 33), ("TANH", 23), ("WINDOW_DATA", 24),
            ("THRESHOLD", 31)]

_V1 = Msg("V1LayerParameter", [
    F("bottom", 2, "string", "repeated"), F("top", 3, "string", "repeated"), F("name", 4, "string"),
    F("include", 32, "msg", "repeated", P + ".NetStateRule"), F("exclude", 33, "msg", "repeated", P + ".NetStateRule"),
    F("type", 5, "enum", type_name=P + ".V1LayerParameter.LayerType"),
    F("blobs", 6, "msg", "repeated", P + ".BlobProto"), F("param", 1001, "string", "repeated"),
    F("blobs_lr", 7, "float", "repeated"), F("weight_decay", 8, "float", "repeated"),
    F("loss_weight", 35, "float", "repeated"),
] + [F(k, v[2], "msg", type_name=f"{P}.{v[0]}") for k, v in _LAYER_PARAMS.items() if v[2] is not None],
    enums=[("LayerType", V1_TYPES)])

_ENUMS = [("Phase", [("TRAIN", 0), ("TEST", 1)]), ("Engine", [("DEFAULT", 0), ("CAFFE", 1), ("CUDNN", 2)])]

POOL, CLASSES, ENUMS = build("bigdl_hip/caffe.proto", PKG,
                             [_FILLER, _BLOB_SHAPE, _BLOB, _NET_STATE, _RULE, _PARAM_SPEC, _NET, _LAYER, _V1, _CONV,
                              _POOL, _IP, _LRN, _ELTWISE] + _SIMPLE, _ENUMS, syntax="proto2")

NetParameter = CLASSES["caffe.NetParameter"]
LayerParameter = CLASSES["caffe.LayerParameter"]
V1LayerParameter = CLASSES["caffe.V1LayerParameter"]
BlobProto = CLASSES["caffe.BlobProto"]
BlobShape = CLASSES["caffe.BlobShape"]
V1_TYPE_NAME = {v: k for k, v in V1_TYPES}
V1_TYPE_VALUE = dict(V1_TYPES)
