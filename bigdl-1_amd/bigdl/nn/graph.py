"""DAG models: ``ModuleNode``, ``Input``, ``Graph``/``StaticGraph``/``Model``.

Reference: ``DL/nn/Graph.scala:72-743``, ``StaticGraph.scala:14-211`` (topological forward order
precomputed at construction, backward in reverse with gradient accumulation for fan-out),
``DL/utils/DirectedGraph.scala`` (``topologySort`` 54, ``Node`` 190).
Build with ``Input()`` and the call syntax ``layer(node, ...)``; ``Graph(inputs, outputs)``.
``stopGradient`` / ``freeze`` by node name are supported.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import List

import torch

from ..utils.table import Table
from .abstractnn import AbstractModule
from .containers import Container, _add_act
from .layers.shape import Identity


class ModuleNode:
    _counter = 0

    def __init__(self, module: AbstractModule):
        self.element = module
        self.prev_nodes: List["ModuleNode"] = []
        self.prev_index: List[int] = []  # output index of the predecessor (0 = whole activity)
        self.next_nodes: List["ModuleNode"] = []
        ModuleNode._counter += 1
        self._id = ModuleNode._counter

    @staticmethod
    def create(module, prevs):
        n = ModuleNode(module)
        for p in prevs:
            if isinstance(p, tuple):  # (node, 1-based output index)
                node, idx = p
            else:
                node, idx = p, 0
            n.prev_nodes.append(node)
            n.prev_index.append(idx)
            node.next_nodes.append(n)
        return n

    def __call__(self, *prevs):
        for p in prevs:
            node, idx = (p if isinstance(p, tuple) else (p, 0))
            self.prev_nodes.append(node)
            self.prev_index.append(idx)
            node.next_nodes.append(self)
        return self

    def remove_pre_edges(self):
        for p in self.prev_nodes:
            p.next_nodes = [n for n in p.next_nodes if n is not self]
        self.prev_nodes = []
        self.prev_index = []
        return self

    def remove_next_edges(self):
        for n in self.next_nodes:
            keep = [(p, i) for p, i in zip(n.prev_nodes, n.prev_index) if p is not self]
            n.prev_nodes = [p for p, _ in keep]
            n.prev_index = [i for _, i in keep]
        self.next_nodes = []
        return self

    def set_name(self, name):
        self.element.set_name(name)
        return self

    def name(self):
        return self.element.get_name()

    def __repr__(self):
        return f"Node({self.element!r})"


class _InputLayer(Identity):
    SCALA_NAME = "Input"


def Input(name: str = None):
    """Create an input placeholder node (``DL/nn/Input.scala``)."""
    m = _InputLayer()
    if name:
        m.set_name(name)
    return ModuleNode(m)


def _topo(outputs: List[ModuleNode]) -> List[ModuleNode]:
    order, seen, temp = [], set(), set()

    def visit(n):
        if n._id in seen:
            return
        if n._id in temp:
            raise ValueError("graph has a cycle")
        temp.add(n._id)
        for p in n.prev_nodes:
            visit(p)
        temp.discard(n._id)
        seen.add(n._id)
        order.append(n)
    for o in outputs:
        visit(o)
    return order


class Graph(Container):
    """Static graph executor (``StaticGraph``)."""

    SCALA_NAME = "StaticGraph"

    def __init__(self, inputs, outputs, variables=None):
        super().__init__()
        self.inputs = inputs if isinstance(inputs, (list, tuple)) else [inputs]
        self.outputs_nodes = outputs if isinstance(outputs, (list, tuple)) else [outputs]
        self.inputs = list(self.inputs)
        self.outputs_nodes = list(self.outputs_nodes)
        self.forward_order = _topo(self.outputs_nodes)
        for n in self.inputs:
            if n not in self.forward_order:
                self.forward_order.insert(0, n)
        self.modules = [n.element for n in self.forward_order]
        self._stop_grad = set()

    # --- execution -------------------------------------------------------------------------
    def _node_input(self, n, acts):
        vals = []
        for p, idx in zip(n.prev_nodes, n.prev_index):
            a = acts[p._id]
            vals.append(a[idx] if idx and isinstance(a, Table) else a)
        if not vals:
            return None
        return vals[0] if len(vals) == 1 else Table(*vals)

    def _concat_plans(self):
        """JoinTable nodes whose every input is produced by a single-consumer conv (optionally
        through its fused ReLU) → :class:`ConcatPlan` (zero-copy concat at inference)."""
        from .containers import ConcatPlan
        from .layers.activation import Threshold
        from .layers.conv import SpatialConvolution
        from .layers.table_ops import JoinTable
        plans = []
        for n in self.forward_order:
            if not isinstance(n.element, JoinTable) or len(n.prev_nodes) < 2:
                continue
            convs = []
            for p in n.prev_nodes:
                c = None
                e = p.element
                if (isinstance(e, Threshold) and e._passthrough == "mask" and len(p.prev_nodes) == 1
                        and len(p.next_nodes) == 1):
                    q = p.prev_nodes[0]
                    if isinstance(q.element, SpatialConvolution) and q.element._fused_relu and len(q.next_nodes) == 1:
                        c = q.element
                elif isinstance(e, SpatialConvolution) and not e._fused_relu and len(p.next_nodes) == 1:
                    c = e
                convs.append(c)
            if all(c is not None for c in convs) and len({id(c) for c in convs}) == len(convs):
                plans.append((n.element, ConcatPlan(convs)))
        return plans

    def updateOutput(self, input):
        acts = {}
        if len(self.inputs) == 1:
            feeds = {self.inputs[0]._id: input}
        else:
            feeds = {n._id: input[i + 1] for i, n in enumerate(self.inputs)}
        self._node_inputs = {}
        plans = ()
        first = input if isinstance(input, torch.Tensor) else None
        if not self.train and first is not None and first.is_cuda:
            if getattr(self, "_plans", None) is None:
                self._plans = self._concat_plans()
            plans = self._plans
        key = tuple(first.shape) if first is not None else None
        for join, plan in plans:
            join._planned = plan.arm(key, first)
        try:
            for n in self.forward_order:
                if n._id in feeds:
                    x = feeds[n._id]
                else:
                    x = self._node_input(n, acts)
                self._node_inputs[n._id] = x
                acts[n._id] = n.element.forward(x)
        finally:
            for join, plan in plans:
                plan.disarm()
                join._planned = None
                plan.record(key, join.output)
        self._acts = acts
        outs = [acts[o._id] for o in self.outputs_nodes]
        return outs[0] if len(outs) == 1 else Table(*outs)

    def _backward_impl(self, input, gradOutput, call):
        grads = {}
        if len(self.outputs_nodes) == 1:
            grads[self.outputs_nodes[0]._id] = gradOutput
        else:
            for i, o in enumerate(self.outputs_nodes):
                grads[o._id] = _add_act(grads.get(o._id), gradOutput[i + 1])
        for n in reversed(self.forward_order):
            g = grads.get(n._id)
            if g is None:
                continue
            x = self._node_inputs[n._id]
            gi = call(n.element, x, g)
            if n.element.get_name() in self._stop_grad:
                continue
            if not n.prev_nodes:
                grads[("in", n._id)] = gi
                continue
            if len(n.prev_nodes) == 1:
                p, idx = n.prev_nodes[0], n.prev_index[0]
                grads[p._id] = self._acc(grads.get(p._id), gi, idx, p)
            else:
                for k, (p, idx) in enumerate(zip(n.prev_nodes, n.prev_index)):
                    grads[p._id] = self._acc(grads.get(p._id), gi[k + 1], idx, p)
        if len(self.inputs) == 1:
            return grads.get(("in", self.inputs[0]._id))
        return Table(*[grads.get(("in", n._id)) for n in self.inputs])

    def _acc(self, cur, g, idx, p):
        if idx:
            t = cur if isinstance(cur, Table) else Table()
            t[idx] = _add_act(t.get(idx), g)
            return t
        return _add_act(cur, g)

    def updateGradInput(self, input, gradOutput):
        return self._backward_impl(input, gradOutput, lambda m, x, g: m.updateGradInput(x, g))

    def accGradParameters(self, input, gradOutput):
        # relies on gradInput values computed by updateGradInput being cached on modules
        grads = {}
        if len(self.outputs_nodes) == 1:
            grads[self.outputs_nodes[0]._id] = gradOutput
        for n in reversed(self.forward_order):
            g = grads.get(n._id)
            if g is None:
                continue
            n.element.accGradParameters(self._node_inputs[n._id], g)
            gi = n.element.gradInput
            for k, (p, idx) in enumerate(zip(n.prev_nodes, n.prev_index)):
                gk = gi if len(n.prev_nodes) == 1 else gi[k + 1]
                grads[p._id] = self._acc(grads.get(p._id), gk, idx, p)

    def backward(self, input, gradOutput):
        import time
        t0 = time.perf_counter()
        ev = self._dev_start(gradOutput)
        self.gradInput = self._backward_impl(input, gradOutput, lambda m, x, g: m.backward(x, g))
        self._dev_stop(ev, 1)
        self.backward_time += time.perf_counter() - t0
        return self.gradInput

    # --- graph utilities ---------------------------------------------------------------------
    def node(self, name: str) -> ModuleNode:
        for n in self.forward_order:
            if n.element.get_name() == name:
                return n
        raise KeyError(name)

    def stopGradient(self, names):
        self._stop_grad.update(names)
        return self

    stop_gradient = stopGradient

    def getForwardExecutions(self):
        return list(self.forward_order)

    def saveGraphTopology(self, log_path):
        from ..visualization.summary import save_graph_topology
        save_graph_topology(self, log_path)
        return self

    save_graph_topology = saveGraphTopology


StaticGraph = Graph


def Model(inputs, outputs):
    """pyspark ``Model(inputs, outputs)`` (``PY/nn/layer.py:704``)."""
    return Graph(inputs, outputs)


def to_graph(module):
    """Sequential → Graph (``AbstractModule.toGraph``)."""
    from .containers import Sequential
    if isinstance(module, Graph):
        return module
    inp = Input()
    if isinstance(module, Sequential):
        x = inp
        for m in module.modules:
            x = m(x)
        return Graph(inp, x)
    return Graph(inp, module(inp))
