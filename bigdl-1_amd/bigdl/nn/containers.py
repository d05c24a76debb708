"""Containers: ``DL/nn/Container.scala:40-237``, ``Sequential.scala``, ``Concat.scala:44``,
``ConcatTable.scala``, ``ParallelTable.scala``, ``MapTable.scala``, ``Bottle.scala``.
"""
from __future__ import annotations

from typing import List

import torch

from ..utils.table import Table
from .abstractnn import AbstractModule, map_activity


def _add_act(a, b):
    """Accumulate gradient activities (tensor or table)."""
    if a is None:
        return b
    if isinstance(a, torch.Tensor):
        if a.numel() == 0:
            return b
        return a + b
    t = Table()
    for k in set(a.keys()) | set(b.keys()):
        if k in a and k in b:
            t[k] = _add_act(a[k], b[k])
        else:
            t[k] = a[k] if k in a else b[k]
    return t


class Container(AbstractModule):
    def __init__(self, *modules):
        super().__init__()
        self.modules: List[AbstractModule] = []
        for m in modules:
            self.add(m)

    def add(self, module: AbstractModule):
        self.modules.append(module)
        return self

    def children(self):
        return list(self.modules)

    def layers(self):
        return list(self.modules)

    def __getitem__(self, i):
        return self.modules[i]

    def __len__(self):
        return len(self.modules)

    def _param_entries(self):
        out = list(super()._param_entries())
        for m in self.modules:
            out.extend(m._param_entries())
        return out

    def parameters(self):
        ws, gs = [], []
        for m, w, g in self._param_entries():
            ws.append(getattr(m, w))
            gs.append(getattr(m, g))
        if not ws:
            return None
        return ws, gs

    def getExtraParameter(self):
        out = []
        for m in self.modules:
            e = m.getExtraParameter()
            if e:
                out.extend(e)
        return out or None

    def setExtraParameter(self, extra):
        i = 0
        for m in self.modules:
            e = m.getExtraParameter()
            if e:
                m.setExtraParameter(extra[i:i + len(e)])
                i += len(e)
        return self

    def zeroGradParameters(self):
        if self._arena is not None and self._arena.grad is not None and self._owns_arena():
            from .. import ops
            ops.zero_fill(self._arena.grad)
            return
        for m in self.modules:
            m.zeroGradParameters()

    def _owns_arena(self):
        ents = self._param_entries()
        return len(ents) == len(self._arena.slices)

    def _set_arena_recursive(self, arena):
        self._arena = arena
        for m in self.modules:
            m._set_arena_recursive(arena)

    def getParametersTable(self):
        t = Table()
        for m in self.modules:
            sub = m.getParametersTable()
            for k, v in sub.items():
                t[k] = v
        return t

    def findModules(self, type_name: str):
        return [m for m in self.flattened_modules() if type(m).__name__ == type_name]

    def flattened_layers(self, include_container=False):
        out = []
        for m in self.modules:
            if isinstance(m, Container):
                if include_container:
                    out.append(m)
                out.extend(m.flattened_layers(include_container))
            else:
                out.append(m)
        return out

    def __repr__(self):
        inner = "\n  ".join(repr(m).replace("\n", "\n  ") for m in self.modules)
        return f"{type(self).__name__}[{self.get_name()}] {{\n  {inner}\n}}"


class Sequential(Container):
    """Chains ``forward`` and runs ``backward`` in reverse (``Sequential.scala:35-100``)."""

    def updateOutput(self, input):
        x = input
        for m in self.modules:
            x = m.forward(x)
        return x

    def updateGradInput(self, input, gradOutput):
        g = gradOutput
        for i in range(len(self.modules) - 1, 0, -1):
            g = self.modules[i].updateGradInput(self.modules[i - 1].output, g)
        return self.modules[0].updateGradInput(input, g)

    def accGradParameters(self, input, gradOutput):
        g = gradOutput
        for i in range(len(self.modules) - 1, 0, -1):
            m = self.modules[i]
            m.accGradParameters(self.modules[i - 1].output, g)
            g = m.gradInput
        self.modules[0].accGradParameters(input, g)

    def backward(self, input, gradOutput):
        import time
        t0 = time.perf_counter()
        ev = self._dev_start(gradOutput)
        g = gradOutput
        for i in range(len(self.modules) - 1, 0, -1):
            g = self.modules[i].backward(self.modules[i - 1].output, g)
        g = self.modules[0].backward(input, g)
        self.gradInput = g
        self._dev_stop(ev, 1)
        self.backward_time += time.perf_counter() - t0
        for h in self._grad_ready_hooks:
            h(self)
        return g


def _final_conv(m):
    """The conv whose output IS ``m``'s output (a conv, or a Sequential ending in conv [→ fused
    ReLU]), else None."""
    from .layers.conv import SpatialConvolution
    from .layers.activation import Threshold
    while isinstance(m, Sequential) and m.modules:
        last = m.modules[-1]
        if isinstance(last, Threshold) and last._passthrough == "mask" and len(m.modules) > 1:
            prev = m.modules[-2]
            return prev if isinstance(prev, SpatialConvolution) and prev._fused_relu else None
        m = last
    return m if isinstance(m, SpatialConvolution) and not m._fused_relu else None


class ConcatPlan:
    """Zero-copy channel concat for inference (K19): once the output shape of a concat is known for
    an input shape, the next forward preallocates the NHWC output and every branch's final conv
    writes its channel slice in its epilogue — the concat copy disappears.  Eval mode on the device
    only (training keeps separate branch tensors for the backward slices)."""

    def __init__(self, convs):
        self.convs = convs
        self.shapes = {}

    def arm(self, key, x):
        shp = self.shapes.get(key)
        if shp is None or not (isinstance(x, torch.Tensor) and x.is_cuda) or any(c is None for c in self.convs):
            return None
        big = torch.empty(shp, dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
        c0 = 0
        for c in self.convs:
            k = c.nOutputPlane
            c._out_target = big[:, c0:c0 + k]
            c0 += k
        return big

    def disarm(self):
        for c in self.convs:
            if c is not None:
                c._out_target = None

    def record(self, key, out):
        if (isinstance(out, torch.Tensor) and out.is_cuda and out.dim() == 4 and out.dtype == torch.bfloat16
                and out.shape[1] == sum(c.nOutputPlane for c in self.convs if c is not None)):
            self.shapes[key] = tuple(out.shape)


def _plan_key(x):
    return tuple(x.shape) if isinstance(x, torch.Tensor) else None


class Concat(Container):
    """Run every branch on the same input and concatenate along ``dimension`` (1-based)."""

    def __init__(self, dimension: int, *modules):
        super().__init__(*modules)
        self.dimension = dimension
        self._plan = None

    def updateOutput(self, input):
        plan = None
        if not self.train and self.dimension == 2 and isinstance(input, torch.Tensor) and input.dim() == 4:
            if self._plan is None:
                self._plan = ConcatPlan([_final_conv(m) for m in self.modules])
            plan = self._plan
        big = plan.arm(_plan_key(input), input) if plan is not None else None
        try:
            outs = [m.forward(input) for m in self.modules]
        finally:
            if plan is not None:
                plan.disarm()
        self._sizes = [o.shape[self.dimension - 1] for o in outs]
        if big is not None:
            from .layers.table_ops import _tiles_channels
            if _tiles_channels(big, outs):
                return big
        out = torch.cat(outs, dim=self.dimension - 1)
        if plan is not None:
            if out.is_cuda:
                out = out.contiguous(memory_format=torch.channels_last)
            plan.record(_plan_key(input), out)
        return out

    def _split_grad(self, gradOutput):
        return torch.split(gradOutput, self._sizes, dim=self.dimension - 1)

    def updateGradInput(self, input, gradOutput):
        gi = None
        for m, g in zip(self.modules, self._split_grad(gradOutput)):
            gi = _add_act(gi, m.updateGradInput(input, g.contiguous()))
        return gi

    def accGradParameters(self, input, gradOutput):
        for m, g in zip(self.modules, self._split_grad(gradOutput)):
            m.accGradParameters(input, g.contiguous())

    def backward(self, input, gradOutput):
        gi = None
        for m, g in zip(self.modules, self._split_grad(gradOutput)):
            gi = _add_act(gi, m.backward(input, g.contiguous()))
        self.gradInput = gi
        return gi


def _deterministic():
    from ..utils import config
    return bool(config.get_property("bigdl.deterministic"))


class ConcatTable(Container):
    """Apply each member to the same input; output is a Table (``ConcatTable.scala``).

    With ``_residual`` set by :mod:`bigdl.nn.fusion` (ResNet block tail) the shortcut runs first and
    the main branch's last BN emits ReLU(BN(·) + shortcut) directly; the following CAddTable/ReLU
    are pass-throughs."""

    _residual = None

    def updateOutput(self, input):
        if self._residual is not None:
            return self._fused_forward(input)
        return Table(*[m.forward(input) for m in self.modules])

    def _fused_forward(self, input):
        br, bn, shortcut, relu = self._residual
        last = shortcut.modules[-1] if isinstance(shortcut, Sequential) and shortcut.modules else None
        if last is not None and getattr(last, "_defer_ok", False) and not _deterministic():
            # shortcut conv → BN: the BN only finalizes its statistics and hands over its input and
            # coefficients (ops.reference.BNOut); the tail BN applies it inside its own pass, so the
            # shortcut activation is never written or re-read (one fewer full pass per stage)
            h2 = input
            for m in shortcut.modules[:-1]:
                h2 = m.forward(h2)
            last._defer_next = True
            try:
                r = last.forward(h2)
            finally:
                last.__dict__.pop("_defer_next", None)
            shortcut.output = r
        else:
            r = shortcut.forward(input)
        h = input
        for m in br.modules[:-1]:
            h = m.forward(h)
        self._bn_in = h
        y = bn.forward_residual(h, r, relu)
        br.output = y
        return Table(y, r)

    def _fused_backward(self, input, gradOutput):
        br, bn, shortcut, relu = self._residual
        g = gradOutput[1] if isinstance(gradOutput, Table) else gradOutput
        gb, gres = bn.backward_residual(self._bn_in, g)
        # shortcut first, so the branch's first conv can sum its gradient in the dgrad epilogue
        gs = shortcut.backward(input, gres)
        from .layers.conv import SpatialConvolution
        from ..ops.reference import StridedGrad
        first = br.modules[0]
        fold = (isinstance(first, SpatialConvolution) and isinstance(gs, (torch.Tensor, StridedGrad))
                and len(br.modules) > 1)
        if isinstance(gs, StridedGrad) and not fold:
            gs = gs.dense()
        if fold:
            first._grad_residual = gs
        for i in range(len(br.modules) - 2, -1, -1):
            prev = br.modules[i - 1].output if i > 0 else input
            gb = br.modules[i].backward(prev, gb)
        br.gradInput = gb
        if fold:
            first._grad_residual = None
            return gb
        return _add_act(gb, gs)

    def updateGradInput(self, input, gradOutput):
        if self._residual is not None:
            self._fused_done = True
            return self._fused_backward(input, gradOutput)
        gi = None
        for i, m in enumerate(self.modules):
            gi = _add_act(gi, m.updateGradInput(input, gradOutput[i + 1]))
        return gi

    def accGradParameters(self, input, gradOutput):
        if self._residual is not None and getattr(self, "_fused_done", False):
            self._fused_done = False
            return
        for i, m in enumerate(self.modules):
            m.accGradParameters(input, gradOutput[i + 1])

    def backward(self, input, gradOutput):
        if self._residual is not None:
            gi = self._fused_backward(input, gradOutput)
        else:
            gi = None
            for i, m in enumerate(self.modules):
                gi = _add_act(gi, m.backward(input, gradOutput[i + 1]))
        self.gradInput = gi
        for h in self._grad_ready_hooks:
            h(self)
        return gi


class ParallelTable(Container):
    """i-th member applied to the i-th input element."""

    def updateOutput(self, input):
        return Table(*[m.forward(input[i + 1]) for i, m in enumerate(self.modules)])

    def updateGradInput(self, input, gradOutput):
        return Table(*[m.updateGradInput(input[i + 1], gradOutput[i + 1]) for i, m in enumerate(self.modules)])

    def accGradParameters(self, input, gradOutput):
        for i, m in enumerate(self.modules):
            m.accGradParameters(input[i + 1], gradOutput[i + 1])

    def backward(self, input, gradOutput):
        self.gradInput = Table(*[m.backward(input[i + 1], gradOutput[i + 1]) for i, m in enumerate(self.modules)])
        return self.gradInput


class MapTable(Container):
    """Apply one (shared-weight) module to every element of the input table."""

    def __init__(self, module: AbstractModule = None):
        super().__init__()
        self.module = module
        self._clones = []
        if module is not None:
            self.add(module)

    def _ensure(self, n):
        import copy
        while len(self._clones) < n:
            if not self._clones:
                self._clones.append(self.module)
            else:
                c = copy.copy(self.module)
                c.__dict__ = dict(self.module.__dict__)  # share parameter tensors
                self._clones.append(c)

    def updateOutput(self, input):
        n = input.length()
        self._ensure(n)
        return Table(*[self._clones[i].forward(input[i + 1]) for i in range(n)])

    def updateGradInput(self, input, gradOutput):
        return Table(*[self._clones[i].updateGradInput(input[i + 1], gradOutput[i + 1]) for i in range(input.length())])

    def accGradParameters(self, input, gradOutput):
        for i in range(input.length()):
            self._clones[i].accGradParameters(input[i + 1], gradOutput[i + 1])


class Bottle(Container):
    """Fold leading dims so an nInputDim-D module can process higher-D input (``Bottle.scala``)."""

    def __init__(self, module: AbstractModule, n_input_dim: int = 2, n_output_dim: int = -1):
        super().__init__(module)
        self.nInputDim = n_input_dim
        self.nOutputDim = n_output_dim if n_output_dim != -1 else n_input_dim

    def updateOutput(self, input):
        lead = input.shape[: input.dim() - self.nInputDim + 1]
        self._lead = lead
        x = input.reshape((-1,) + tuple(input.shape[input.dim() - self.nInputDim + 1:]))
        y = self.modules[0].forward(x)
        return y.reshape(tuple(lead) + tuple(y.shape[1:]))

    def updateGradInput(self, input, gradOutput):
        x = input.reshape((-1,) + tuple(input.shape[input.dim() - self.nInputDim + 1:]))
        g = gradOutput.reshape((-1,) + tuple(gradOutput.shape[len(self._lead):]))
        gi = self.modules[0].updateGradInput(x, g)
        return gi.reshape(input.shape)

    def accGradParameters(self, input, gradOutput):
        x = input.reshape((-1,) + tuple(input.shape[input.dim() - self.nInputDim + 1:]))
        g = gradOutput.reshape((-1,) + tuple(gradOutput.shape[len(self._lead):]))
        self.modules[0].accGradParameters(x, g)
