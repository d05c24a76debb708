"""bigdl.nn — Torch-style modules with explicit forward/backward (``DL/nn``)."""
from .abstractnn import (AbstractModule, TensorModule, AutogradModule, AbstractCriterion, AutogradCriterion,
                         Activity, LayerException, FlatParameters)
from .containers import Container, Sequential, Concat, ConcatTable, ParallelTable, MapTable, Bottle
from .graph import Graph, StaticGraph, Model, Input, ModuleNode, to_graph
from .dynamic_graph import (DynamicGraph, Scheduler, FrameManager, ControlNodes, SwitchControlNode,
                            MergeControlNode)
from .layers import *  # noqa: F401,F403
from .criterion import *  # noqa: F401,F403
from .initialization_method import *  # noqa: F401,F403
Module = AbstractModule
from .int8_convertible import MklInt8Convertible, calc_tensor_scale, install as _install_int8
_install_int8()
