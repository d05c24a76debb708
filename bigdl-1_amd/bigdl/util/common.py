"""pyspark ``bigdl.util.common`` compatibility (``pyspark/bigdl/util/common.py``).

There is no JVM: ``callBigDlFunc("float", "createLinear", 3, 4)`` resolves ``createX`` to the
class ``X`` of this package and calls it; ``JTensor`` is a host ndarray holder; the Spark context
helpers return local stand-ins (one process per GPU replaces Spark executors)."""
from __future__ import annotations

import os
from typing import Any, List, Optional

import numpy as np
import torch

from ..dataset.core import Sample as _Sample
from ..utils.engine import Engine
from ..utils.random import RNG as _RNG


class JavaValue:
    """Base of the pyspark wrapper classes; here the object IS the implementation."""

    def jvm_class_constructor(self):
        return "create" + type(self).__name__

    def __init__(self, jvalue=None, bigdl_type="float", *args):
        self.value = self
        self.bigdl_type = bigdl_type


class JActivity:
    def __init__(self, value):
        self.value = value


class EvaluatedResult:
    def __init__(self, result, total_num, method):
        self.result, self.total_num, self.method = result, total_num, method

    def __str__(self):
        return f"Evaluated result: {self.result}, total_num: {self.total_num}, method: {self.method}"


def get_dtype(bigdl_type):
    return "float64" if bigdl_type == "double" else "float32"


class JTensor:
    """Dense (``storage``, ``shape``) or sparse (+``indices``) ndarray holder."""

    def __init__(self, storage, shape, bigdl_type="float", indices=None):
        self.storage = np.asarray(storage, dtype=get_dtype(bigdl_type)).reshape(-1)
        self.shape = np.asarray(shape, dtype=np.int32)
        self.indices = None if indices is None else np.asarray(indices, dtype=np.int32)
        self.bigdl_type = bigdl_type

    @classmethod
    def from_ndarray(cls, a_ndarray, bigdl_type="float"):
        if a_ndarray is None:
            return None
        a = np.asarray(a_ndarray)
        return cls(a.reshape(-1), a.shape, bigdl_type)

    @classmethod
    def sparse(cls, a_ndarray, i_ndarray, shape, bigdl_type="float"):
        return cls(a_ndarray, shape, bigdl_type, i_ndarray)

    def to_ndarray(self):
        if self.indices is not None:
            dense = np.zeros(tuple(self.shape), dtype=self.storage.dtype)
            idx = self.indices.reshape(len(self.shape), -1)
            dense[tuple(idx)] = self.storage
            return dense
        return self.storage.reshape(tuple(self.shape))

    def to_tensor(self) -> torch.Tensor:
        if self.indices is not None:
            idx = torch.as_tensor(self.indices.reshape(len(self.shape), -1), dtype=torch.long)
            return torch.sparse_coo_tensor(idx, torch.as_tensor(self.storage), tuple(self.shape))
        return torch.from_numpy(self.to_ndarray().copy())

    def __repr__(self):
        return f"JTensor: storage: {self.storage}, shape: {self.shape}"

    __str__ = __repr__


class Sample(_Sample):
    """pyspark ``Sample``: ``Sample.from_ndarray(features, labels)`` (a scalar label becomes a
    1-element tensor); features/labels may be ndarrays, lists of ndarrays or JTensors."""

    def __init__(self, features, labels=None, bigdl_type="float"):
        def conv(x):
            if isinstance(x, JTensor):
                return x.to_tensor()
            return x
        if isinstance(features, (list, tuple)):
            features = [conv(f) for f in features]
        else:
            features = conv(features)
        if isinstance(labels, (list, tuple)):
            labels = [conv(l) for l in labels]
        else:
            labels = conv(labels)
        super().__init__(features, labels)
        self.bigdl_type = bigdl_type

    @classmethod
    def from_ndarray(cls, features, labels, bigdl_type="float"):
        if isinstance(labels, (int, float, np.integer, np.floating)):
            labels = np.array([labels], dtype=np.float32)
        return cls(features, labels, bigdl_type)

    @classmethod
    def from_jtensor(cls, features, labels, bigdl_type="float"):
        return cls(features, labels, bigdl_type)


class RNG:
    def __init__(self, bigdl_type="float"):
        self.bigdl_type = bigdl_type

    def set_seed(self, seed):
        _RNG.setSeed(seed)

    def uniform(self, a, b, size):
        return np.asarray([_RNG.uniform(a, b) for _ in range(int(np.prod(size)))], dtype=np.float32).reshape(size)


def init_engine(bigdl_type="float"):
    Engine.init()


def init_executor_gateway(sc=None, bigdl_type="float"):
    return None


def get_node_and_core_number(bigdl_type="float"):
    return Engine.node_number(), Engine.core_number()


def redire_spark_logs(bigdl_type="float", log_path=None):
    from ..utils.logger import redirect_logs
    redirect_logs(log_path or os.path.join(os.getcwd(), "bigdl.log"))


def show_bigdl_info_logs(bigdl_type="float"):
    import logging
    logging.getLogger("bigdl").setLevel(logging.INFO)


def get_bigdl_conf():
    from ..utils import config
    return config.describe()


def to_list(a):
    if isinstance(a, list):
        return a
    return [a]


def to_sample_rdd(x, y, numSlices=None):
    """No Spark: a list of Samples (the "RDD" of the pyspark API)."""
    return [Sample.from_ndarray(f, l) for f, l in zip(x, y)]


def create_spark_conf():
    from ..utils import config
    return dict(config.describe())


def get_spark_context(conf=None):
    return None


def get_spark_sql_context(sc=None):
    return None


def create_tmp_path():
    import tempfile
    return tempfile.mkdtemp(prefix="bigdl")


def _resolve(name: str):
    import importlib
    short = name[len("create"):] if name.startswith("create") else name
    for modname in ("bigdl.nn", "bigdl.nn.criterion", "bigdl.optim", "bigdl.optim.optimizer", "bigdl.optim.trigger",
                    "bigdl.optim.validation", "bigdl.nn.keras", "bigdl.transform.vision.image", "bigdl.dataset",
                    "bigdl.visualization"):
        try:
            m = importlib.import_module(modname)
        except ImportError:
            continue
        if hasattr(m, short):
            return getattr(m, short)
    raise AttributeError(f"no BigDL function {name}")


def callBigDlFunc(bigdl_type, name, *args):
    """``PythonBigDL.createX(args)`` → ``X(*args)`` (303 creators in the reference)."""
    return _resolve(name)(*args)


def callJavaFunc(func, *args):
    return func(*args)
