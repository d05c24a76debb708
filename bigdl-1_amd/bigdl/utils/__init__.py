from .table import Table, T, to_table
from .shape import Shape, SingleShape, MultiShape
from .random import RNG, RandomGenerator
from .engine import Engine, init_engine
from . import config
from .logger import get_logger

__all__ = ["Table", "T", "to_table", "Shape", "SingleShape", "MultiShape", "RNG", "RandomGenerator",
           "Engine", "init_engine", "config", "get_logger"]
