"""Caffe model export (``DL/utils/caffe/CaffePersister.scala:229``, ``toCaffe*`` in
``Converter.scala`` / ``LayerConverter.scala`` / ``V1LayerConverter.scala``).

``CaffePersister.persist(prototxt, caffemodel, module, useV2=True, overwrite=False)`` walks the
graph in topological order and emits one Caffe layer per module (tops named after the layer,
bottoms taken from the predecessors' tops); ``View`` nodes are elided (Caffe's InnerProduct
flattens implicitly).  The ``.caffemodel`` carries the blobs, the ``.prototxt`` the same net
without blobs.  A ``Sequential`` chain is accepted and exported as the equivalent linear graph.
"""
from __future__ import annotations

import os

import numpy as np
import torch
from google.protobuf import text_format

from . import caffe_pb as C
from .caffe_loader import CaffeConversionException


def _blob(t: torch.Tensor, shape=None):
    b = C.BlobProto()
    arr = t.detach().float().cpu().contiguous().reshape(-1).numpy()
    b.data.extend(arr.tolist())
    b.shape.dim.extend(list(shape if shape is not None else t.shape))
    return b


def _v1_type(name):
    return C.V1_TYPE_VALUE[name]


class CaffePersister:
    def __init__(self, prototxt_path, model_path, module, useV2=True, overwrite=False):
        self.prototxt_path, self.model_path = prototxt_path, model_path
        self.module, self.useV2, self.overwrite = module, useV2, overwrite

    # ------------------------------------------------------------------------------ per layer
    def _layer(self, name, v2_type, v1_type, bottoms):
        if self.useV2:
            l = C.LayerParameter()
            l.type = v2_type
        else:
            l = C.V1LayerParameter()
            if v1_type is None:
                raise CaffeConversionException(f"{v2_type} has no V1 layer type")
            l.type = _v1_type(v1_type)
        l.name = name
        l.bottom.extend(bottoms)
        l.top.append(name)
        return l

    def _convert(self, m, bottoms):
        from ..nn import (SpatialConvolution, SpatialFullConvolution, ReLU, SpatialCrossMapLRN, SpatialWithinChannelLRN,
                          SpatialMaxPooling, SpatialAveragePooling, Linear, Dropout, LogSoftMax, SoftMax, Tanh, Sigmoid,
                          Abs, SpatialBatchNormalization, JoinTable, ELU, InferReshape, Log, Power, PReLU, Reshape,
                          Scale, Add, Threshold, Exp, SplitTable, Replicate, CMaxTable, CAddTable, CSubTable,
                          CMulTable, Identity)
        name = m.get_name()
        L = self._layer
        if isinstance(m, SpatialConvolution):
            l = L(name, "Convolution", "CONVOLUTION", bottoms)
            p = l.convolution_param
            p.num_output, p.group = m.nOutputPlane, m.nGroup
            p.kernel_w, p.kernel_h, p.stride_w, p.stride_h = m.kernelW, m.kernelH, m.strideW, m.strideH
            p.pad_w, p.pad_h = max(m.padW, 0), max(m.padH, 0)
            if m.dilationW != 1:
                p.dilation.append(m.dilationW)
            p.bias_term = bool(m.withBias)
            g = m.nGroup
            l.blobs.append(_blob(m.weight, [m.nOutputPlane, m.nInputPlane // g, m.kernelH, m.kernelW]))
            if m.withBias:
                l.blobs.append(_blob(m.bias))
            return l
        if isinstance(m, SpatialFullConvolution):
            l = L(name, "Deconvolution", "DECONVOLUTION", bottoms)
            p = l.convolution_param
            p.num_output, p.group = m.nOutputPlane, m.nGroup
            p.kernel_w, p.kernel_h, p.stride_w, p.stride_h = m.kW, m.kH, m.dW, m.dH
            p.pad_w, p.pad_h = m.padW, m.padH
            p.bias_term = not m.noBias
            l.blobs.append(_blob(m.weight, [m.nInputPlane, m.nOutputPlane // m.nGroup, m.kH, m.kW]))
            if not m.noBias:
                l.blobs.append(_blob(m.bias))
            return l
        if isinstance(m, (SpatialCrossMapLRN, SpatialWithinChannelLRN)):
            l = L(name, "LRN", "LRN", bottoms)
            p = l.lrn_param
            p.local_size, p.alpha, p.beta = m.size, m.alpha, m.beta
            if isinstance(m, SpatialCrossMapLRN):
                p.k = m.k
            else:
                p.norm_region = 1
            return l
        if isinstance(m, ReLU):
            return L(name, "ReLU", "RELU", bottoms)
        if isinstance(m, (SpatialMaxPooling, SpatialAveragePooling)):
            l = L(name, "Pooling", "POOLING", bottoms)
            p = l.pooling_param
            p.pool = 0 if isinstance(m, SpatialMaxPooling) else 1
            p.kernel_w, p.kernel_h, p.stride_w, p.stride_h = m.kW, m.kH, m.dW, m.dH
            p.pad_w, p.pad_h = m.padW, m.padH
            if getattr(m, "globalPooling", False):
                p.global_pooling = True
            return l
        if isinstance(m, Linear):
            l = L(name, "InnerProduct", "INNER_PRODUCT", bottoms)
            p = l.inner_product_param
            p.num_output, p.bias_term = m.outputSize, bool(m.withBias)
            l.blobs.append(_blob(m.weight))
            if m.withBias:
                l.blobs.append(_blob(m.bias))
            return l
        if isinstance(m, Dropout):
            l = L(name, "Dropout", "DROPOUT", bottoms)
            l.dropout_param.dropout_ratio = m.p
            return l
        if isinstance(m, (LogSoftMax, SoftMax)):
            return L(name, "Softmax", "SOFTMAX", bottoms)
        if isinstance(m, Tanh):
            return L(name, "TanH", "TANH", bottoms)
        if isinstance(m, Sigmoid):
            return L(name, "Sigmoid", "SIGMOID", bottoms)
        if isinstance(m, Abs):
            return L(name, "AbsVal", "ABSVAL", bottoms)
        if isinstance(m, SpatialBatchNormalization):
            l = L(name, "BatchNorm", None, bottoms)
            l.batch_norm_param.eps = m.eps
            l.blobs.append(_blob(m.runningMean))
            l.blobs.append(_blob(m.runningVar))
            l.blobs.append(_blob(torch.ones(1)))
            if not m.affine:
                return l
            # Caffe BatchNorm has no affine part: gamma/beta go to a following Scale layer
            sc = L(name + "_scale", "Scale", None, [name])
            sc.scale_param.bias_term = True
            sc.blobs.append(_blob(m.weight))
            sc.blobs.append(_blob(m.bias))
            return [l, sc]
        if isinstance(m, JoinTable):
            l = L(name, "Concat", "CONCAT", bottoms)
            l.concat_param.axis = m.dimension - 1
            return l
        if isinstance(m, ELU):
            l = L(name, "ELU", None, bottoms)
            l.elu_param.alpha = m.alpha
            return l
        if isinstance(m, InferReshape):
            return L(name, "Flatten", "FLATTEN", bottoms)
        if isinstance(m, Log):
            return L(name, "Log", None, bottoms)
        if isinstance(m, Power):
            l = L(name, "Power", "POWER", bottoms)
            l.power_param.power, l.power_param.scale, l.power_param.shift = m.power, m.scale, m.shift
            return l
        if isinstance(m, PReLU):
            l = L(name, "PReLU", None, bottoms)
            l.blobs.append(_blob(m.weight))
            return l
        if isinstance(m, Reshape):
            l = L(name, "Reshape", None, bottoms)
            l.reshape_param.shape.dim.extend([0] + [int(s) for s in m.size])
            return l
        if isinstance(m, Scale):
            l = L(name, "Scale", None, bottoms)
            l.scale_param.bias_term = True
            l.blobs.append(_blob(m.cmul.weight if hasattr(m, "cmul") else m.weight))
            l.blobs.append(_blob(m.cadd.bias if hasattr(m, "cadd") else m.bias))
            return l
        if isinstance(m, Add):
            l = L(name, "Bias", None, bottoms)
            l.blobs.append(_blob(m.bias))
            return l
        if isinstance(m, Threshold) and not isinstance(m, ReLU):
            l = L(name, "Threshold", "THRESHOLD", bottoms)
            l.threshold_param.threshold = m.threshold
            return l
        if isinstance(m, Exp):
            return L(name, "Exp", "EXP", bottoms)
        if isinstance(m, SplitTable):
            l = L(name, "Slice", "SLICE", bottoms)
            l.slice_param.axis = m.dimension
            return l
        if isinstance(m, Replicate):
            l = L(name, "Tile", None, bottoms)
            l.tile_param.axis = m.dim - 1
            l.tile_param.tiles = m.nFeatures
            return l
        if isinstance(m, (CMaxTable, CAddTable, CSubTable, CMulTable)):
            l = L(name, "Eltwise", "ELTWISE", bottoms)
            if isinstance(m, CMaxTable):
                l.eltwise_param.operation = 2
            elif isinstance(m, CMulTable):
                l.eltwise_param.operation = 0
            else:
                l.eltwise_param.operation = 1
                if isinstance(m, CSubTable):
                    l.eltwise_param.coeff.extend([1.0, -1.0])
            return l
        if isinstance(m, Identity):
            return None
        raise CaffeConversionException(f"{m} is not supported")

    # ------------------------------------------------------------------------------ graph walk
    def _graph(self):
        from ..nn import Graph, Sequential, Input
        m = self.module
        if isinstance(m, Graph):
            return m
        if isinstance(m, Sequential):
            inp = Input()
            inp.element.set_name("data")
            x = inp
            for sub in m.modules:
                x = sub(x)
            g = Graph(inp, x)
            g.set_name(m.get_name())
            return g
        raise CaffeConversionException(f"container {m} is not supported, only graph supported")

    def convert(self):
        from ..nn import View
        from ..nn.graph import _InputLayer
        g = self._graph()
        net = C.NetParameter()
        net.name = self.module.get_name()
        tops = {}
        for n in g.forward_order:
            m = n.element
            bottoms = []
            for p in n.prev_nodes:
                bottoms.extend(tops.get(p._id, []))
            if isinstance(m, _InputLayer) or not n.prev_nodes and isinstance(m, _InputLayer):
                l = self._layer(m.get_name(), "Input", None, []) if self.useV2 else None
                if l is not None:
                    net.layer.append(l)
                else:
                    net.input.append(m.get_name())
                tops[n._id] = [m.get_name()]
                continue
            if isinstance(m, View):
                tops[n._id] = bottoms
                continue
            l = self._convert(m, bottoms)
            if l is None:
                tops[n._id] = bottoms
                continue
            ls = l if isinstance(l, list) else [l]
            (net.layer if self.useV2 else net.layers).extend(ls)
            tops[n._id] = list(ls[-1].top)
        return net

    def save(self):
        net = self.convert()
        for path in (self.prototxt_path, self.model_path):
            if os.path.exists(path) and not self.overwrite:
                raise FileExistsError(f"{path} already exists; pass overwrite=True")
        with open(self.model_path, "wb") as f:
            f.write(net.SerializeToString())
        bare = C.NetParameter()
        bare.CopyFrom(net)
        for coll in (bare.layer, bare.layers):
            for l in coll:
                del l.blobs[:]
        with open(self.prototxt_path, "w") as f:
            f.write(text_format.MessageToString(bare))

    @staticmethod
    def persist(prototxt_path, model_path, module, useV2=True, overwrite=False):
        CaffePersister(prototxt_path, model_path, module, useV2, overwrite).save()


def save_caffe(module, prototxt_path, model_path, use_v2=True, overwrite=False):
    CaffePersister.persist(prototxt_path, model_path, module, use_v2, overwrite)
