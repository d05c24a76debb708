"""``object Module`` static helpers (``DL/nn/Module.scala:32-166``): model loaders and ``flatten``."""
from __future__ import annotations

import torch


class Module:
    @staticmethod
    def loadModule(path: str, weight_path: str = None):
        from ..serialization.module_serializer import load_module
        return load_module(path, weight_path)

    load_module = loadModule

    @staticmethod
    def load(path: str):
        """Legacy ``Module.load`` (Java serialisation in the reference) → the .bigdl loader."""
        return Module.loadModule(path)

    @staticmethod
    def loadTorch(path: str):
        from ..serialization.torch_file import load_torch
        return load_torch(path)

    load_torch = loadTorch

    @staticmethod
    def loadCaffeModel(def_path: str, model_path: str):
        from ..serialization.caffe_loader import load_caffe_model
        return load_caffe_model(def_path, model_path)

    load_caffe_model = loadCaffeModel

    @staticmethod
    def loadCaffe(model, def_path: str, model_path: str, match_all: bool = True):
        from ..serialization.caffe_loader import load_caffe_weights
        return load_caffe_weights(model, def_path, model_path, match_all)

    @staticmethod
    def loadTF(path, inputs, outputs, byte_order="little_endian", bin_file=None, generated_backward=False):
        """``Module.loadTF`` (Module.scala:72-86): a TensorFlow GraphDef (binary .pb or text
        .pbtxt) → BigDL Graph, see :meth:`bigdl.utils.tf.loader.TensorflowLoader.load`."""
        from ..utils.tf.loader import TensorflowLoader
        bo = "big" if str(byte_order).lower().startswith("big") else "little"
        return TensorflowLoader.load(path, list(inputs), list(outputs), bo, bin_file, generated_backward)

    @staticmethod
    def flatten(parameters):
        """Compact a list of tensors into one storage (``Module.flatten``); returns the flat tensor
        and re-points nothing (callers copy back) — used for weight snapshots."""
        if not parameters:
            return torch.empty(0)
        return torch.cat([p.reshape(-1).float() for p in parameters])

    @staticmethod
    def isCompact(parameters) -> bool:
        if not parameters:
            return True
        base = parameters[0].untyped_storage().data_ptr()
        off = parameters[0].storage_offset()
        for p in parameters:
            if p.untyped_storage().data_ptr() != base or p.storage_offset() != off or not p.is_contiguous():
                return False
            off += p.numel()
        return True
