"""TensorFlow data-flow ops: ``TensorArray*``, ``Stack*`` and ``AssignGrad``
(reference: ``DL/nn/tf/DataFlowOps.scala:30-679``, ``DL/nn/tf/StateOps.scala:106-113``).

These are the resources a TF ``while_loop`` graph threads through its iterations (``tf.TensorArray``
for per-step inputs / outputs, a stack for the gradient loop's saved activations).  A resource lives in
a process-wide registry keyed by its handle; the ops pass the handle along as a plain string (the
reference's ``Tensor[String]`` scalar) together with the ``flow`` scalar TF uses to order the
writes before the reads.

Semantics follow the reference exactly: a TensorArray slot is written once (a gradient array created by
``TensorArrayGrad`` aggregates repeated writes instead), a read clears the slot when
``clearAfterRead``, ``dynamicSize`` lets a write grow the array, and ``TensorArrayGrad`` locks the
source array's size.  Tensors keep their device: an array filled with GPU tensors returns GPU tensors.
"""
from __future__ import annotations

import threading
from typing import Dict, List, Optional, Sequence

import torch

from ...utils.table import Table
from ..ops import Operation

__all__ = ["TensorArray", "TensorArrayCreator", "TensorArrayGrad", "TensorArrayWrite", "TensorArrayRead",
           "TensorArrayGather", "TensorArrayScatter", "TensorArrayConcat", "TensorArraySplit", "TensorArraySize",
           "TensorArrayClose", "StackCreator", "StackPush", "StackPop", "AssignGrad"]

_LOCK = threading.Lock()

#: the scalar every data-flow op returns as its "flow" output (orders TF reads after writes)
FLOW_OUT = torch.tensor(0.0)


def _handle(v) -> str:
    if isinstance(v, Table):  # the creator's whole (handle, flow) output wired as one input
        v = v[1]
    if isinstance(v, str):
        return v
    if isinstance(v, bytes):
        return v.decode()
    raise TypeError(f"a resource handle must be a string scalar, got {type(v).__name__}")


def _int(v) -> int:
    if isinstance(v, torch.Tensor):
        if v.numel() != 1:
            raise ValueError("index must be a scalar")
        return int(v.reshape(-1)[0])
    return int(v)


def _ints(v) -> List[int]:
    t = torch.as_tensor(v)
    if t.dim() != 1:
        raise ValueError("indices must be a vector")
    return [int(i) for i in t.tolist()]


class TensorArray:
    """The array itself (``DataFlowOps.scala:30-160``)."""

    _arrays: Dict[str, "TensorArray"] = {}

    def __init__(self, init_size: int, shape: Optional[Sequence[int]] = None, dynamic_size: bool = False,
                 clear_after_read: bool = True, identical_element_shapes: bool = False,
                 multiple_writes_aggregate: bool = False):
        self.init_size = int(init_size)
        self.shape = list(shape) if shape is not None else None
        self.dynamic_size = dynamic_size
        self.clear_after_read = clear_after_read
        self.identical_element_shapes = identical_element_shapes
        self.multiple_writes_aggregate = multiple_writes_aggregate
        self._other_shape = None
        self.tensors: List[Optional[torch.Tensor]] = [None] * self.init_size

    def lock_size(self):
        self.dynamic_size = False

    def __getitem__(self, index: int) -> torch.Tensor:
        t = self.tensors[index]
        if t is None:
            raise ValueError(f"tensor on index {index} has not been inited or has been cleared")
        if self.clear_after_read:
            self.tensors[index] = None
        return t

    def grad(self) -> "TensorArray":
        self.lock_size()
        return TensorArray(self.size(), multiple_writes_aggregate=True)

    def size(self) -> int:
        return len(self.tensors)

    def shape_of(self, index: int) -> List[int]:
        t = self.tensors[index]
        if t is None:
            raise ValueError(f"tensor on index {index} has not been inited or has been cleared")
        return list(t.shape)

    def __setitem__(self, index: int, tensor: torch.Tensor):
        if not self.multiple_writes_aggregate and index < len(self.tensors) and self.tensors[index] is not None:
            raise ValueError("There's already a tensor on the given index")
        cur = list(tensor.shape)
        if self.identical_element_shapes:
            if self._other_shape is None:
                self._other_shape = cur
            elif cur != self._other_shape:
                raise ValueError("insert tensor size does not match other tensor size")
        if self.shape is not None and cur != self.shape:
            raise ValueError("insert tensor size does not match required size")
        if self.dynamic_size and index >= len(self.tensors):
            self.tensors.extend([None] * (index + 1 - len(self.tensors)))
        elif index >= self.init_size:
            raise ValueError("cannot grow size when dynamicSize is false")
        if self.tensors[index] is None:
            self.tensors[index] = tensor.detach().clone()
        else:
            self.tensors[index] = self.tensors[index] + tensor

    # ---- registry ---------------------------------------------------------------------------
    @classmethod
    def get(cls, key: str) -> "TensorArray":
        with _LOCK:
            if key not in cls._arrays:
                raise KeyError(f"Cannot find TensorArray for name {key}")
            return cls._arrays[key]

    @classmethod
    def put(cls, key: str, value: "TensorArray"):
        with _LOCK:
            cls._arrays[key] = value

    @classmethod
    def exist(cls, key: str) -> bool:
        with _LOCK:
            return key in cls._arrays

    @classmethod
    def release(cls, key: str):
        with _LOCK:
            cls._arrays.pop(key, None)


class _Resource(Operation):
    """An op that allocates a named resource; the handle is unique per op instance."""

    def __init__(self, name: str = ""):
        super().__init__()
        self._resource_name = name

    def _handle_name(self) -> str:
        base = self._resource_name or self.get_name()
        return f"{base}{id(self)}"


class TensorArrayCreator(_Resource):
    """size (int scalar) → Table(handle, flow) (``DataFlowOps.scala:163-205``)."""

    SCALA_PACKAGE = "com.intel.analytics.bigdl.nn.tf"

    def __init__(self, shape=None, dynamicSize: bool = False, clearAfterRead: bool = True,
                 identicalElementShapes: bool = False, tensorArrayName: str = ""):
        super().__init__(tensorArrayName)
        self.shape = list(shape) if shape is not None else None
        self.dynamicSize, self.clearAfterRead = dynamicSize, clearAfterRead
        self.identicalElementShapes = identicalElementShapes
        self.tensorArrayName = tensorArrayName

    def updateOutput(self, input):
        size = _int(input)
        h = self._handle_name()
        TensorArray.put(h, TensorArray(size, self.shape, self.dynamicSize, self.clearAfterRead,
                                       self.identicalElementShapes))
        self.output = Table(h, FLOW_OUT)
        return self.output

    def release(self):
        TensorArray.release(self._handle_name())


class TensorArrayGrad(Operation):
    """Table(handle, flow) → Table(grad handle, flow): the gradient array of a source, created once and
    locked to the source's size (``DataFlowOps.scala:207-229``)."""

    SCALA_PACKAGE = "com.intel.analytics.bigdl.nn.tf"

    def __init__(self, source: str):
        super().__init__()
        self.source = source

    def updateOutput(self, input):
        h = _handle(input[1])
        name = h + self.source
        with _LOCK:
            arr = TensorArray._arrays.get(h)
            if arr is None:
                raise KeyError(f"Cannot find TensorArray for name {h}")
            if name not in TensorArray._arrays:
                TensorArray._arrays[name] = arr.grad()
        self.output = Table(name, FLOW_OUT)
        return self.output


class TensorArrayWrite(Operation):
    """Table(handle, index, value, flow) → flow (``DataFlowOps.scala:231-257``)."""

    SCALA_PACKAGE = "com.intel.analytics.bigdl.nn.tf"

    def updateOutput(self, input):
        TensorArray.get(_handle(input[1]))[_int(input[2])] = input[3]
        self.output = FLOW_OUT
        return self.output


class TensorArrayRead(Operation):
    """Table(handle, index, flow) → the element (cleared from the array when clearAfterRead)."""

    SCALA_PACKAGE = "com.intel.analytics.bigdl.nn.tf"

    def updateOutput(self, input):
        self.output = TensorArray.get(_handle(input[1]))[_int(input[2])]
        return self.output


class TensorArrayGather(Operation):
    """Table(handle, indices, flow) → the selected elements stacked along a new first dimension
    (all must share one shape; ``DataFlowOps.scala:278-322``)."""

    SCALA_PACKAGE = "com.intel.analytics.bigdl.nn.tf"

    def updateOutput(self, input):
        arr = TensorArray.get(_handle(input[1]))
        idx = _ints(input[2])
        shapes = [arr.shape_of(i) for i in idx]
        if any(s != shapes[0] for s in shapes):
            raise ValueError("the selected tensors have different sizes")
        self.output = torch.stack([arr[i] for i in idx], 0) if idx else torch.empty(0)
        return self.output


class TensorArrayScatter(Operation):
    """Table(handle, indices, value, flow) → flow: element indices[i] = value[i]."""

    SCALA_PACKAGE = "com.intel.analytics.bigdl.nn.tf"

    def updateOutput(self, input):
        arr = TensorArray.get(_handle(input[1]))
        idx = _ints(input[2])
        value = input[3]
        if len(idx) != value.shape[0]:
            raise ValueError("indices length does not match value first dimension")
        for i, k in enumerate(idx):
            arr[k] = value[i]
        self.output = FLOW_OUT
        return self.output


class TensorArrayConcat(Operation):
    """Table(handle, flow) → Table(all elements concatenated along dim 0, their lengths as int32)."""

    SCALA_PACKAGE = "com.intel.analytics.bigdl.nn.tf"

    def updateOutput(self, input):
        arr = TensorArray.get(_handle(input[1]))
        lengths = torch.tensor([arr.shape_of(i)[0] for i in range(arr.size())], dtype=torch.int32)
        value = torch.cat([arr[i] for i in range(arr.size())], 0)
        self.output = Table(value, lengths)
        return self.output


class TensorArraySplit(Operation):
    """Table(handle, value, lengths, flow) → flow: element i = the i-th run of ``lengths[i]`` rows."""

    SCALA_PACKAGE = "com.intel.analytics.bigdl.nn.tf"

    def updateOutput(self, input):
        arr = TensorArray.get(_handle(input[1]))
        value = input[2]
        lengths = _ints(input[3])
        start = 0
        for i, n in enumerate(lengths):
            arr[i] = value.narrow(0, start, n)
            start += n
        self.output = FLOW_OUT
        return self.output


class TensorArraySize(Operation):
    """Table(handle, flow) → the array size (int32 scalar)."""

    SCALA_PACKAGE = "com.intel.analytics.bigdl.nn.tf"

    def updateOutput(self, input):
        h = input[1] if isinstance(input, Table) else input
        self.output = torch.tensor(TensorArray.get(_handle(h)).size(), dtype=torch.int32)
        return self.output


class TensorArrayClose(Operation):
    """handle (or Table(handle, flow)) → flow: releases the array."""

    SCALA_PACKAGE = "com.intel.analytics.bigdl.nn.tf"

    def updateOutput(self, input):
        h = input[1] if isinstance(input, Table) else input
        TensorArray.release(_handle(h))
        self.output = FLOW_OUT
        return self.output


# ------------------------------------------------------------------------------------------------ stack
class _Stack:
    """``DataFlowOps.scala:570-588``: push clones, pop returns the most recent."""

    _stacks: Dict[str, "_Stack"] = {}

    def __init__(self, max_size: int):
        self.max_size = max_size
        self.tensors: List[torch.Tensor] = []

    def push(self, t: torch.Tensor):
        if len(self.tensors) >= self.max_size:
            raise ValueError("Stack is full")
        self.tensors.append(t.detach().clone())

    def pop(self) -> torch.Tensor:
        if not self.tensors:
            raise ValueError("There's no tensors in the stack")
        return self.tensors.pop()

    @classmethod
    def get(cls, key: str) -> "_Stack":
        with _LOCK:
            if key not in cls._stacks:
                raise KeyError(f"Cannot find Stack for name {key}")
            return cls._stacks[key]


class StackCreator(_Resource):
    """[max size (int scalar, < 0 or absent = unbounded)] → handle (``DataFlowOps.scala:608-637``)."""

    SCALA_PACKAGE = "com.intel.analytics.bigdl.nn.tf"

    def __init__(self, name: str = ""):
        super().__init__(name)
        self.name_ = name

    def updateOutput(self, input=None):
        if input is not None and isinstance(input, torch.Tensor) and input.numel() not in (0, 1):
            raise ValueError("StackCreator: Input tensor should be a scalar or no input")
        n = _int(input) if isinstance(input, torch.Tensor) and input.numel() == 1 else -1
        h = self._handle_name()
        with _LOCK:
            _Stack._stacks[h] = _Stack(n if n >= 0 else 2 ** 62)
        self.output = h
        return self.output

    def release(self):
        with _LOCK:
            _Stack._stacks.pop(self._handle_name(), None)


class StackPush(Operation):
    """Table(handle, data) → data (a clone is pushed)."""

    SCALA_PACKAGE = "com.intel.analytics.bigdl.nn.tf"

    def updateOutput(self, input):
        data = input[2]
        _Stack.get(_handle(input[1])).push(data)
        self.output = data
        return self.output


class StackPop(Operation):
    """handle (or Table(handle, control...)) → the most recently pushed tensor."""

    SCALA_PACKAGE = "com.intel.analytics.bigdl.nn.tf"

    def updateOutput(self, input):
        h = input[1] if isinstance(input, Table) else input
        self.output = _Stack.get(_handle(h)).pop()
        return self.output


class AssignGrad(Operation):
    """Copies its input into a fixed gradient tensor (``StateOps.scala:106-113``); output null."""

    SCALA_PACKAGE = "com.intel.analytics.bigdl.nn.tf"

    def __init__(self, grad: torch.Tensor):
        super().__init__()
        self.grad = grad

    def updateOutput(self, input):
        self.grad.copy_(input)
        self.output = None
        return self.output
