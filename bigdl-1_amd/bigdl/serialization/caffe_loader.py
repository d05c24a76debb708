"""Caffe model import (``DL/utils/caffe/CaffeLoader.scala``, ``Converter.scala``,
``LayerConverter.scala``, ``V1LayerConverter.scala``).

* ``load_caffe_weights(model, prototxt, caffemodel, match_all)`` copies blobs into an existing
  model by layer name (``CaffeLoader.load`` / ``copyParameters`` :205-275).
* ``CaffeLoader.loadCaffe(prototxt, caffemodel, customized, output_names)`` builds a ``Graph``
  from the net definition (V2 ``layer`` or V1 ``layers``), wiring bottoms → tops, resolving
  ``Split`` layers, turning loss layers into a ``ParallelCriterion`` and copying weights
  (``createCaffeModel`` :283-453).  Returns (model, criterion).
* ``load_caffe_model`` is the Python-API entry (model only).

Conversion rules follow the reference: Pooling is always ``ceil`` mode, conv input planes come
from the weight blob, InnerProduct gets a ``View(nIn)`` in front when nIn != nOut, BatchNorm
blobs (mean, var, scale-factor) become running statistics of an affine-free BN, Eltwise SUM
with coefficients becomes MulConstant+CAddTable.  Blobs are copied in Caffe's row-major order,
which is the logical order of our weights whatever their physical (KRSC) layout is.
"""
from __future__ import annotations

import logging
from typing import Callable, Dict, List, Optional

import numpy as np
import torch
from google.protobuf import text_format

from . import caffe_pb as C

log = logging.getLogger("bigdl.caffe")


class CaffeConversionException(Exception):
    pass


class Customizable:
    """User converter for a layer type (``CaffeLoader.scala`` ``Customizable``): implement
    ``convertor(layer) -> [ModuleNode...]``; ``contexts`` gets name2LayerV1/V2 and netparam."""

    def __init__(self):
        self.contexts = {}

    def convertor(self, layer):  # pragma: no cover - abstract
        raise NotImplementedError

    def registerContext(self, name, ctx):
        self.contexts[name] = ctx


# ------------------------------------------------------------------------------------------ io
def _read_net(prototxt_path: str, model_path: Optional[str]):
    net = C.NetParameter()
    with open(prototxt_path, "r", encoding="ascii", errors="replace") as f:
        text_format.Merge(f.read(), net, allow_unknown_field=True)
    if model_path is None:
        return net
    weights = C.NetParameter()
    with open(model_path, "rb") as f:
        weights.ParseFromString(f.read())
    by_name = {}
    for l in weights.layers:
        by_name[l.name] = l
    for l in weights.layer:
        by_name[l.name] = l
    for coll in (net.layers, net.layer):
        for l in coll:
            w = by_name.get(l.name)
            if w is not None:
                del l.blobs[:]
                l.blobs.extend(w.blobs)
            else:
                log.warning(f"layer {l.name} of type {_layer_type(l)} does not exist in weight file")
    return net


def _layer_type(layer) -> str:
    if isinstance(layer, C.V1LayerParameter):
        return C.V1_TYPE_NAME.get(layer.type, str(layer.type))
    return layer.type


def blob_to_tensor(blob) -> torch.Tensor:
    data = np.asarray(blob.data if len(blob.data) else blob.double_data, dtype=np.float32)
    return torch.from_numpy(data.copy())


def blob_shape(blob) -> List[int]:
    if blob.HasField("shape"):
        return [int(d) for d in blob.shape.dim]
    return [blob.num, blob.channels, blob.height, blob.width]


# ------------------------------------------------------------------------------------------ converters
def _node(m):
    from ..nn.graph import ModuleNode
    return ModuleNode(m)


def _named(m, layer):
    return m.set_name(layer.name)


def _conv(layer):
    from ..nn import SpatialConvolution, SpatialDilatedConvolution, SpatialFullConvolution
    p = layer.convolution_param
    group = p.group or 1
    if not layer.blobs:
        raise CaffeConversionException(f"{layer.name}: convolution weight blob missing")
    ws = blob_shape(layer.blobs[0])
    n_in = (ws[1] if layer.blobs[0].HasField("shape") else layer.blobs[0].channels) * group
    n_out = ws[0] if layer.blobs[0].HasField("shape") else layer.blobs[0].num
    with_bias = len(layer.blobs) > 1
    kw, kh = p.kernel_w, p.kernel_h
    if kw == 0 or kh == 0:
        kw = kh = p.kernel_size[0]
    dw, dh = p.stride_w, p.stride_h
    if dw == 0 or dh == 0:
        dw = dh = p.stride[0] if len(p.stride) else 1
    pw, ph = p.pad_w, p.pad_h
    if (pw == 0 or ph == 0) and len(p.pad):
        pw = ph = p.pad[0]
    dil = p.dilation[0] if len(p.dilation) else 1
    if _layer_type(layer).upper() == "DECONVOLUTION":
        m = SpatialFullConvolution(n_out, n_in, kw, kh, dw, dh, pw, ph, 0, 0, group, not with_bias)
    elif dil == 1:
        m = SpatialConvolution(n_in, n_out, kw, kh, dw, dh, pw, ph, group, with_bias=with_bias)
    else:
        m = SpatialDilatedConvolution(n_in, n_out, kw, kh, dw, dh, pw, ph, dil, dil)
    return [_node(_named(m, layer))]


def _inner_product(layer):
    from ..nn import Linear, View
    p = layer.inner_product_param
    if not layer.blobs:
        raise CaffeConversionException(f"{layer.name}: inner product weight blob missing")
    b0 = layer.blobs[0]
    n_in = int(b0.shape.dim[1]) if b0.HasField("shape") else b0.width
    n_out = p.num_output
    lin = _node(_named(Linear(n_in, n_out, with_bias=p.bias_term), layer))
    if n_in != n_out:
        view = _node(View(n_in))
        lin(view)
        return [view, lin]
    return [lin]


def _relu(layer):
    from ..nn import ReLU, LeakyReLU
    slope = layer.relu_param.negative_slope if layer.HasField("relu_param") else 0.0
    return [_node(_named(ReLU(True) if slope == 0 else LeakyReLU(slope), layer))]


def _lrn(layer):
    from ..nn import SpatialCrossMapLRN, SpatialWithinChannelLRN
    p = layer.lrn_param
    if p.norm_region == 0:
        m = SpatialCrossMapLRN(p.local_size, p.alpha, p.beta, p.k)
    else:
        m = SpatialWithinChannelLRN(p.local_size, p.alpha, p.beta)
    return [_node(_named(m, layer))]


def _pooling(layer):
    from ..nn import SpatialMaxPooling, SpatialAveragePooling
    p = layer.pooling_param
    kw, kh = p.kernel_w, p.kernel_h
    if kw == 0 or kh == 0:
        kw = kh = p.kernel_size
    dw, dh = p.stride_w, p.stride_h
    if dw == 0 or dh == 0:
        dw = dh = p.stride
    pw, ph = p.pad_w, p.pad_h
    if pw == 0 or ph == 0:
        pw = ph = p.pad
    if p.pool == 0:
        m = SpatialMaxPooling(kw, kh, dw, dh, pw, ph).ceil()
    elif p.pool == 1:
        m = SpatialAveragePooling(kw, kh, dw, dh, pw, ph, p.global_pooling).ceil()
    else:
        raise CaffeConversionException(f"{layer.name}: stochastic pooling is not supported")
    return [_node(_named(m, layer))]


def _simple(factory):
    def conv(layer):
        return [_node(_named(factory(layer), layer))]
    return conv


def _batch_norm(layer):
    from ..nn import SpatialBatchNormalization
    b = layer.blobs
    n = blob_shape(b[0])[0] if b[0].HasField("shape") else b[0].num
    eps = layer.batch_norm_param.eps if layer.HasField("batch_norm_param") else 1e-5
    bn = SpatialBatchNormalization(n, eps, affine=False)
    sf = float(b[2].data[0]) if len(b) > 2 and len(b[2].data) else 1.0
    scale = 0.0 if sf == 0 else 1.0 / sf
    with torch.no_grad():
        bn.runningMean.copy_(blob_to_tensor(b[0])[:n] * scale)
        bn.runningVar.copy_(blob_to_tensor(b[1])[:n] * scale)
    return [_node(_named(bn, layer))]


def _scale(layer):
    from ..nn import Scale, CMul
    if len(layer.blobs) > 1:
        bs = blob_shape(layer.blobs[1])
        size = [1, bs[0], 1, 1] if len(bs) == 1 else bs
        return [_node(_named(Scale(size), layer))]
    if not layer.blobs:
        raise CaffeConversionException(f"{layer.name}: scale weight blob missing")
    shape = blob_shape(layer.blobs[0])
    p = layer.scale_param
    axis, na = p.axis, p.num_axes
    na = len(shape) - 1 if na == -1 else na + axis
    size = shape[axis - 1:na - 1] if na - 1 > axis - 1 else shape
    return [_node(_named(CMul(size), layer))]


def _bias(layer):
    from ..nn import Add
    size = int(np.prod(blob_shape(layer.blobs[0])))
    return [_node(_named(Add(size), layer))]


def _eltwise(layer):
    from ..nn import CMulTable, CMaxTable, CAddTable, CSubTable, MulConstant, Graph
    p = layer.eltwise_param
    if p.operation == 0:
        return [_node(_named(CMulTable(), layer))]
    if p.operation == 2:
        return [_node(_named(CMaxTable(), layer))]
    c1 = p.coeff[0] if len(p.coeff) else 1.0
    c2 = p.coeff[1] if len(p.coeff) > 1 else 1.0
    if c1 == 1 and c2 == 1:
        return [_node(_named(CAddTable(), layer))]
    if c1 == 1 and c2 == -1:
        return [_node(_named(CSubTable(), layer))]
    m1, m2 = _node(MulConstant(c1)), _node(MulConstant(c2))
    add = _node(_named(CAddTable(), layer))(m1, m2)
    return [_node(Graph([m1, m2], [add]))]


def _input(layer):
    from ..nn import Input
    out = []
    for t in layer.top:
        n = Input()
        n.element.set_name(t)
        out.append(n)
    return out


def _mk_table():
    from ..nn import (SoftMax, Tanh, Sigmoid, Abs, JoinTable, InferReshape, Log, Power, PReLU, Recurrent,
                      BinaryThreshold, Exp, SplitTable, Tile, ELU, Dropout)
    return {
        "CONVOLUTION": _conv, "DECONVOLUTION": _conv, "INNERPRODUCT": _inner_product, "INNER_PRODUCT": _inner_product,
        "RELU": _relu, "LRN": _lrn, "POOLING": _pooling,
        "DROPOUT": _simple(lambda l: Dropout(l.dropout_param.dropout_ratio)),
        "SOFTMAX": _simple(lambda l: SoftMax()), "SOFTMAX_LOSS": None, "SOFTMAXWITHLOSS": None,
        "TANH": _simple(lambda l: Tanh()), "SIGMOID": _simple(lambda l: Sigmoid()),
        "SIGMOIDCROSSENTROPYLOSS": _simple(lambda l: Sigmoid()), "ABSVAL": _simple(lambda l: Abs()),
        "BATCHNORM": _batch_norm,
        "CONCAT": _simple(lambda l: JoinTable(l.concat_param.axis + 1, 0)),
        "ELU": _simple(lambda l: ELU(l.elu_param.alpha if l.HasField("elu_param") else 1.0)),
        "FLATTEN": _simple(lambda l: InferReshape([0, -1])), "LOG": _simple(lambda l: Log()),
        "POWER": _simple(lambda l: Power(l.power_param.power, l.power_param.scale, l.power_param.shift)),
        "PRELU": _simple(lambda l: PReLU(blob_shape(l.blobs[0])[0] if l.blobs[0].HasField("shape")
                                         else l.blobs[0].num)),
        "RECURRENT": _simple(lambda l: Recurrent()), "RNN": _simple(lambda l: Recurrent()),
        "RESHAPE": _simple(lambda l: InferReshape([int(d) for d in l.reshape_param.shape.dim])),
        "SCALE": _scale, "BIAS": _bias,
        "THRESHOLD": _simple(lambda l: BinaryThreshold(l.threshold_param.threshold
                                                       if l.threshold_param.HasField("threshold") else 1e-6)),
        "EXP": _simple(lambda l: Exp()), "SLICE": _simple(lambda l: SplitTable(l.slice_param.axis)),
        "TILE": _simple(lambda l: Tile(l.tile_param.axis + 1, l.tile_param.tiles)),
        "ELTWISE": _eltwise,
        "INPUT": _input, "DATA": _input, "DUMMYDATA": _input, "DUMMY_DATA": _input, "ANNOTATEDDATA": _input,
        "MEMORYDATA": _input, "MEMORY_DATA": _input, "ACCURACY": None, "SILENCE": None,
    }


_DATA_TYPES = {"INPUT", "DATA", "DUMMYDATA", "DUMMY_DATA", "ANNOTATEDDATA", "MEMORYDATA", "MEMORY_DATA"}


class CaffeLoader:
    def __init__(self, prototxt_path: str, model_path: Optional[str], match_all: bool = True,
                 customized_converters: Optional[Dict[str, Customizable]] = None, strict: bool = True):
        self.prototxt_path, self.model_path = prototxt_path, model_path
        self.match_all = match_all
        self.customized = {k.upper(): v for k, v in (customized_converters or {}).items()}
        self.strict = strict
        self.net = _read_net(prototxt_path, model_path)
        self.name2v1 = {l.name: l for l in self.net.layers}
        self.name2v2 = {l.name: l for l in self.net.layer}
        for c in self.customized.values():
            c.registerContext("name2LayerV1", self.name2v1)
            c.registerContext("name2LayerV2", self.name2v2)
            c.registerContext("netparam", self.net)
        from ..nn import ParallelCriterion
        self.criterions = ParallelCriterion()
        self._table = _mk_table()

    # -- weights -----------------------------------------------------------------------------
    def _layer(self, name):
        return self.name2v2.get(name) or self.name2v1.get(name)

    def _copy(self, name, params):
        layer = self._layer(name)
        if layer is None:
            if self.match_all:
                raise CaffeConversionException(f"module {name} cannot map a layer in caffe model")
            log.info(f"{name} uses initialized parameters")
            return
        idx = 0
        with torch.no_grad():
            if len(layer.blobs) > idx and "weight" in params:
                w = params["weight"]
                src = blob_to_tensor(layer.blobs[idx])
                if src.numel() != w.numel():
                    raise CaffeConversionException(
                        f"weight element number is not equal between caffe layer and bigdl module {name}, data "
                        f"shape in caffe is {blob_shape(layer.blobs[idx])}, while data shape in bigdl is "
                        f"{tuple(w.shape)}")
                w.copy_(src.reshape(w.shape).to(w.dtype))
                idx += 1
            if len(layer.blobs) > idx and "bias" in params and params["bias"] is not None:
                b = params["bias"]
                src = blob_to_tensor(layer.blobs[idx])
                if src.numel() != b.numel():
                    raise CaffeConversionException(f"bias element number is not equal for {name}")
                b.copy_(src.reshape(b.shape).to(b.dtype))

    def copyParameters(self, model):
        table = model.getParametersTable()
        for name, params in table.items():
            if params is None or not ("weight" in params or "bias" in params):
                continue
            self._copy(name, params)
        return model

    # -- graph -------------------------------------------------------------------------------
    def _convert(self, layer):
        t = _layer_type(layer).upper()
        if t in self._table:
            f = self._table[t]
            return f(layer) if f is not None else None
        if t in self.customized:
            return self.customized[t].convertor(layer)
        if not self.strict:
            from ..nn import Identity
            log.warning(f"caffe layer type {t} ({layer.name}) not supported: mapped to Identity")
            return [_node(Identity().set_name(layer.name))]
        raise CaffeConversionException(f"{t} is not supported in BigDL for now")

    def _try_criterion(self, t, name) -> bool:
        from ..nn import ClassNLLCriterion, MSECriterion, HingeEmbeddingCriterion, CrossEntropyCriterion, \
            CosineEmbeddingCriterion
        t = t.upper()
        if t in ("SOFTMAX_LOSS", "SOFTMAXWITHLOSS"):
            self.criterions.add(ClassNLLCriterion())
            return False
        if t in ("EUCLIDEANLOSS", "EUCLIDEAN_LOSS"):
            self.criterions.add(MSECriterion())
            return True
        if t in ("HINGELOSS", "HINGE_LOSS"):
            self.criterions.add(HingeEmbeddingCriterion())
            return True
        if t in ("SIGMOIDCROSSENTROPYLOSS", "SIGMOID_CROSS_ENTROPY_LOSS"):
            self.criterions.add(CrossEntropyCriterion())
            return False
        if t in ("INFOGAINLOSS", "INFOGAIN_LOSS"):
            layer = self._layer(name)
            w = blob_to_tensor(layer.blobs[2]) if layer is not None and len(layer.blobs) > 2 else None
            self.criterions.add(ClassNLLCriterion(w))
            return True
        if t in ("CONTRASTIVELOSS", "CONTRASTIVE_LOSS"):
            self.criterions.add(CosineEmbeddingCriterion())
            return True
        return False

    def createCaffeModel(self, output_names=()):
        from ..nn import Graph, Input
        layers: List = []
        layers_map = {}
        top2layer = {}
        split_map = {}
        src = list(self.net.layers) if len(self.net.layers) else list(self.net.layer)
        ordered = {}
        for l in src:
            ordered[l.name] = l  # later definitions override earlier ones, keeping first position
        all_layers = list(ordered.values())
        for name in self.net.input:
            n = Input()
            n.element.set_name(name)
            top2layer[name] = name
            layers_map[name] = n
            layers.append(n)
        for layer in all_layers:
            t = _layer_type(layer).upper()
            name = layer.name
            if t == "SPLIT":
                if len(layer.bottom) != 1:
                    raise CaffeConversionException("split dependency should only be one!")
                for top in layer.top:
                    if layer.bottom[0] in top2layer:
                        split_map[top] = layers_map[top2layer[layer.bottom[0]]]
                continue
            if self._try_criterion(t, name):
                continue
            if t in _DATA_TYPES:
                for n in self._convert(layer) or []:
                    top2layer[n.element.get_name()] = n.element.get_name()
                    layers_map[n.element.get_name()] = n
                    layers.append(n)
                continue
            nodes = self._convert(layer)
            if not nodes:
                continue
            head = nodes[0]
            for dep in layer.bottom:
                if dep in top2layer:
                    head(layers_map[top2layer[dep]])
            cur = head
            while cur.next_nodes:
                layers.append(cur)
                cur = cur.next_nodes[0]
            layers.append(cur)
            layers_map[name] = cur
            for top in layer.top:
                top2layer[top] = name
        for layer in all_layers:
            for b in layer.bottom:
                if b in split_map and layer.name in layers_map:
                    layers_map[layer.name](split_map[b])
        layers = [n for n in layers if (n.prev_nodes or n.next_nodes) or n.element.get_name() in output_names]
        inputs = [n for n in layers if not n.prev_nodes]
        outputs = [n for n in layers if not n.next_nodes or n.element.get_name() in output_names]
        model = Graph(inputs, outputs)
        model.set_name(self.net.name or "caffe_model")
        self.copyParameters(model)
        return model, self.criterions

    @staticmethod
    def load(model, def_path, model_path, match_all=True, customized_converters=None):
        return CaffeLoader(def_path, model_path, match_all, customized_converters).copyParameters(model)

    @staticmethod
    def loadCaffe(def_path, model_path, customized_converters=None, output_names=()):
        return CaffeLoader(def_path, model_path, True, customized_converters).createCaffeModel(output_names)


def load_caffe_weights(model, def_path, model_path, match_all=True, customized_converters=None):
    return CaffeLoader.load(model, def_path, model_path, match_all, customized_converters)


def load_caffe_model(def_path, model_path, customized_converters=None, output_names=(), strict=False):
    """Python-API ``Model.load_caffe_model``: the graph only; unknown layer types map to
    Identity with a warning unless ``strict``."""
    loader = CaffeLoader(def_path, model_path, True, customized_converters, strict=strict)
    return loader.createCaffeModel(output_names)[0]
