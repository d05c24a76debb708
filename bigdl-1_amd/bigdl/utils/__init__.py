from .table import Table, T, to_table
from .shape import Shape, SingleShape, MultiShape
from .random import RNG, RandomGenerator
from .engine import Engine, init_engine
from . import config
from .logger import get_logger

__all__ = ["Table", "T", "to_table", "Shape", "SingleShape", "MultiShape", "RNG", "RandomGenerator",
           "Engine", "init_engine", "config", "get_logger"]


def acc_float(t):
    """Accumulation dtype of a tensor: bf16/fp16/fp32 → fp32, but float64 stays float64 (the
    reference's Double models; the fp64 gradient checker, nn/gradient_checker.py)."""
    import torch
    return t if t.dtype == torch.float64 else t.float()
