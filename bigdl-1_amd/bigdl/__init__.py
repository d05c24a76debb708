"""bigdl — an MI355X-native deep-learning engine with BigDL's API (Torch-style Tensor/nn, Optimizer,
.bigdl/Caffe/Torch model formats).  Compute: PyTorch-ROCm device tensors + hand-written HIP/CDNA4
kernels (``bigdl.ops``); distributed: one process per GPU over RCCL (``bigdl.parallel``)."""
from .version import __version__, BIGDL_VERSION
from .utils import Engine, init_engine, Table, T, RNG
from .tensor import Tensor

__all__ = ["__version__", "BIGDL_VERSION", "Engine", "init_engine", "Table", "T", "RNG", "Tensor"]
