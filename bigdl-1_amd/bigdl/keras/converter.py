"""Keras 1.2.2 model import (``pyspark/bigdl/keras/converter.py``: ``DefinitionLoader``,
``WeightLoader``, ``WeightsConverter``, ``LayerConverter``).

Keras itself is not needed: the JSON model definition is parsed directly and each layer config is
instantiated as the same-named :mod:`bigdl.nn.keras` layer (they share Keras 1.2.2's argument
names and shape inference); functional ``Model`` configs are rebuilt node by node from their
``inbound_nodes``.  Weights come from a Keras HDF5 file (needs ``h5py``, which this image lacks —
the loader says so) or from a ``{layer_name: [arrays in Keras order]}`` mapping / ``.npz`` file;
``WeightsConverter`` reorders them into BigDL layouts exactly as the reference does (Dense
transpose, LSTM/GRU gate concatenation, th/tf convolution kernels, …).
"""
from __future__ import annotations

import inspect
import json
from typing import Dict, List, Optional

import numpy as np
import torch

from ..nn.keras import layers as KL
from ..nn.keras import topology as KT


def _layer_classes():
    out = {}
    for mod in (KL, KT):
        for n, v in vars(mod).items():
            if isinstance(v, type) and issubclass(v, KT.KerasLayer):
                out[n] = v
    return out


_RENAMES = {"output_dim": "output_dim"}


def _kwargs(cls, cfg: dict):
    sig = inspect.signature(cls.__init__)
    kw = {}
    for k, v in cfg.items():
        if k in ("batch_input_shape",):
            if v is not None and "input_shape" in sig.parameters:
                kw["input_shape"] = tuple(v[1:])
            continue
        if k == "input_dtype" or k == "trainable":
            continue
        if k in sig.parameters:
            if isinstance(v, dict) and "class_name" in v:  # regularizers / constraints configs
                v = None if v.get("class_name") in (None, "None") else v
                if k.endswith("regularizer") and v is not None:
                    from ..optim.regularizer import L1L2Regularizer
                    c = v.get("config", {})
                    v = L1L2Regularizer(float(c.get("l1", 0.0)), float(c.get("l2", 0.0)))
                elif v is not None:
                    continue
            if isinstance(v, list) and k in ("pool_size", "strides", "subsample", "size", "padding", "dims",
                                             "target_shape", "cropping", "atrous_rate"):
                v = tuple(tuple(x) if isinstance(x, list) else x for x in v)
            kw[k] = v
    return kw


def _make_layer(class_name: str, cfg: dict, classes):
    if class_name == "InputLayer":
        return None
    if class_name in ("TimeDistributed", "Bidirectional"):
        inner = cfg["layer"]
        sub = _make_layer(inner["class_name"], inner["config"], classes)
        kw = {"input_shape": tuple(cfg["batch_input_shape"][1:])} if cfg.get("batch_input_shape") else {}
        if class_name == "Bidirectional":
            kw["merge_mode"] = cfg.get("merge_mode", "concat")
        return classes[class_name](sub, name=cfg.get("name"), **kw)
    cls = classes.get(class_name)
    if cls is None:
        raise NotImplementedError(f"unsupported Keras layer {class_name}")
    return cls(**_kwargs(cls, cfg))


class DefinitionLoader:
    """Keras JSON → BigDL Keras-API model."""

    def __init__(self, kmodel_json: dict):
        self.json = kmodel_json
        self.classes = _layer_classes()

    @classmethod
    def from_json_path(cls, json_path):
        with open(json_path) as f:
            return cls(json.load(f)).to_bigdl()

    @classmethod
    def from_json_str(cls, json_str):
        return cls(json.loads(json_str)).to_bigdl()

    @classmethod
    def from_hdf5_path(cls, hdf5_path):
        h5 = _h5py()
        with h5.File(hdf5_path, "r") as f:
            cfg = f.attrs["model_config"]
        return cls(json.loads(cfg.decode() if isinstance(cfg, bytes) else cfg)).to_bigdl()

    def to_bigdl(self):
        cn, cfg = self.json["class_name"], self.json["config"]
        if cn == "Sequential":
            return self._sequential(cfg if isinstance(cfg, list) else cfg["layers"])
        if cn == "Model":
            return self._functional(cfg)
        raise NotImplementedError(f"unsupported Keras model class {cn}")

    def _sequential(self, layers):
        m = KT.Sequential()
        for l in layers:
            layer = _make_layer(l["class_name"], l["config"], self.classes)
            if layer is None:
                continue
            if l["config"].get("name"):
                layer.set_name(l["config"]["name"])
            m.add(layer)
        return m

    def _functional(self, cfg):
        nodes = {}
        for l in cfg["layers"]:
            c = l["config"]
            name = l.get("name") or c.get("name")
            if l["class_name"] == "InputLayer":
                nodes[name] = KT.Input(shape=tuple(c["batch_input_shape"][1:]), name=name)
                continue
            layer = _make_layer(l["class_name"], c, self.classes)
            layer.set_name(name)
            inbound = l["inbound_nodes"][0] if l["inbound_nodes"] else []
            prevs = [nodes[ref[0]] for ref in inbound]
            nodes[name] = layer(*prevs)
        ins = [nodes[r[0]] for r in cfg["input_layers"]]
        outs = [nodes[r[0]] for r in cfg["output_layers"]]
        return KT.Model(ins if len(ins) > 1 else ins[0], outs if len(outs) > 1 else outs[0])


class WeightsConverter:
    """Keras 1.2.2 weight lists → BigDL parameter order/layout (``converter.py:110-287``)."""

    @staticmethod
    def convert(klayer, weights: List[np.ndarray]) -> List[np.ndarray]:
        name = type(klayer).__name__.lower()
        fn = getattr(WeightsConverter, f"convert_{name}", None)
        return fn(klayer, weights) if fn else list(weights)

    @staticmethod
    def convert_dense(klayer, w):
        return [np.transpose(w[0])] + list(w[1:])

    convert_timedistributeddense = convert_dense

    @staticmethod
    def convert_batchnormalization(klayer, w):
        return [w[0], w[1]]

    @staticmethod
    def convert_convolution2d(klayer, w):
        k = w[0]
        if getattr(klayer, "dim_ordering", "th") == "tf":
            k = np.transpose(k, (3, 2, 0, 1))
        return [k] + list(w[1:])

    convert_atrousconvolution2d = convert_convolution2d

    @staticmethod
    def convert_convolution1d(klayer, w):
        k = w[0]  # Keras 1D: (filter_length, 1, input_dim, nb_filter)
        if k.ndim == 4:
            k = np.transpose(k, (3, 2, 0, 1))
        return [k] + list(w[1:])

    convert_atrousconvolution1d = convert_convolution1d

    @staticmethod
    def convert_deconvolution2d(klayer, w):
        return [np.transpose(w[0], (1, 0, 2, 3))] + list(w[1:])

    @staticmethod
    def convert_simplernn(klayer, w):
        return [np.transpose(w[0]), w[2], np.transpose(w[1])]

    @staticmethod
    def convert_lstm(klayer, w):
        w1 = np.concatenate((w[0].T, w[3].T, w[6].T, w[9].T))
        w2 = np.concatenate((w[2], w[5], w[8], w[11]))
        w3 = np.concatenate((w[1].T, w[4].T, w[7].T, w[10].T))
        return [w1, w2, w3]

    @staticmethod
    def convert_gru(klayer, w):
        w1 = np.concatenate((w[3].T, w[0].T, w[6].T))
        w2 = np.concatenate((w[5], w[2], w[8]))
        w3 = np.concatenate((w[4].T, w[1].T))
        w4 = w[7].T
        return [w1, w2, w3, w4]

    @staticmethod
    def convert_highway(klayer, w):
        if len(w) == 2:
            return [w[1].T, w[0].T]
        return [w[1].T, w[3], w[0].T, w[2]]


def _h5py():
    try:
        import h5py  # noqa: F401
        return h5py
    except ImportError as e:  # pragma: no cover - environment dependent
        raise ImportError("Keras HDF5 weights need h5py, which is not installed; pass the weights as a "
                          "{layer_name: [arrays]} dict or an .npz file to WeightLoader instead") from e


def _named_layers(model) -> Dict[str, object]:
    out = {}
    for m in model.flattened_modules() if hasattr(model, "flattened_modules") else []:
        if isinstance(m, KT.KerasLayer) and not isinstance(m, KT.KerasModel):
            out[m.get_name()] = m
    return out


class WeightLoader:
    @staticmethod
    def load_weights(bmodel, weights: Dict[str, List[np.ndarray]], by_name: bool = True):
        """Assign Keras-ordered arrays per layer name (converted to BigDL layouts)."""
        layers = _named_layers(bmodel)
        for name, arrays in weights.items():
            if name not in layers:
                if by_name:
                    continue
                raise KeyError(f"layer {name} not in the model")
            klayer = layers[name]
            conv = WeightsConverter.convert(klayer, [np.asarray(a) for a in arrays])
            params = klayer.parameters()
            if params is None:
                continue
            targets = params[0]
            if len(conv) < len(targets):
                raise ValueError(f"{name}: {len(conv)} arrays for {len(targets)} parameters")
            for t, a in zip(targets, conv):
                src = torch.from_numpy(np.ascontiguousarray(a)).float()
                if src.numel() != t.numel():
                    raise ValueError(f"{name}: weight of {src.numel()} elements for a {tuple(t.shape)} parameter")
                t.data.copy_(src.reshape(t.shape))
            if type(klayer).__name__ == "BatchNormalization" and len(arrays) >= 4:
                extra = klayer.getExtraParameter()
                if extra:
                    extra[0].copy_(torch.from_numpy(np.asarray(arrays[2])).float())
                    extra[1].copy_(torch.from_numpy(np.asarray(arrays[3])).float())
        return bmodel

    @staticmethod
    def load_weights_from_npz(bmodel, path, by_name=True):
        """``.npz`` with keys ``<layer>/<index>`` (the HDF5 layout flattened)."""
        data = np.load(path, allow_pickle=False)
        per: Dict[str, List] = {}
        for k in sorted(data.files, key=lambda s: (s.rsplit("/", 1)[0], int(s.rsplit("/", 1)[1]))):
            layer, _ = k.rsplit("/", 1)
            per.setdefault(layer, []).append(data[k])
        return WeightLoader.load_weights(bmodel, per, by_name)

    @staticmethod
    def load_weights_from_hdf5(bmodel, filepath, by_name=False):
        h5 = _h5py()
        per = {}
        with h5.File(filepath, "r") as f:
            g = f["model_weights"] if "model_weights" in f else f
            for name in g.attrs["layer_names"]:
                name = name.decode() if isinstance(name, bytes) else name
                lg = g[name]
                per[name] = [np.asarray(lg[w]) for w in lg.attrs["weight_names"]]
        return WeightLoader.load_weights(bmodel, per, by_name)

    @staticmethod
    def load_weights_from_json_hdf5(def_json, weights_hdf5, by_name=False):
        model = DefinitionLoader.from_json_path(def_json)
        return WeightLoader.load_weights_from_hdf5(model, weights_hdf5, by_name)


def load_keras(json_path=None, hdf5_path=None, by_name=False):
    """``Model.load_keras`` (``PY/nn/layer.py``): definition from JSON (or the HDF5's
    ``model_config``), weights from the HDF5 file when given."""
    if json_path is None and hdf5_path is None:
        raise ValueError("json_path or hdf5_path is required")
    model = DefinitionLoader.from_json_path(json_path) if json_path else DefinitionLoader.from_hdf5_path(hdf5_path)
    if hdf5_path:
        if hdf5_path.endswith(".npz"):
            WeightLoader.load_weights_from_npz(model, hdf5_path, by_name or True)
        else:
            WeightLoader.load_weights_from_hdf5(model, hdf5_path, by_name)
    return model
