"""Dynamic (data-dependent) graph execution: ``DynamicGraph``, ``Scheduler``, ``FrameManager`` and
the ``ControlNodes`` builders (switch / merge / while loop).

Reference behaviour: ``DL/nn/DynamicGraph.scala:28-144`` (scheduler-driven forward, optional
generated backward), ``DL/nn/Scheduler.scala:36-294`` (ready queue, const-node memoisation across
runs, Switch branch selection, Merge input selection, loop frames), ``DL/nn/FrameManager.scala:31-130``
(frames, iteration barrier, NextIteration pending list) and ``DL/nn/tf/ControlOps.scala``
(``ControlNodes.switch/merge/whileLoop``; ``SwitchControlNode.trueEdge/falseEdge``).

Design: the scheduler is host-side control logic only — every node it fires runs its module's
``forward`` on whatever device the module lives on, so a loop body of HIP kernels stays stream
ordered; only the loop predicate (a 1-element tensor) is read back to the host each iteration,
exactly one sync per trip, which is the inherent cost of data-dependent control flow.

Loop semantics follow the reference: ``whileLoop`` EXITS when the condition subgraph yields true
(the Switch's true edge feeds ``Exit``, the false edge feeds the body).
"""
from __future__ import annotations

from collections import deque
from typing import Dict, List, Optional, Sequence

from ..utils.table import Table
from .graph import Graph, ModuleNode, _InputLayer
from .layers.shape import Identity


def _tf():
    from . import tf
    return tf


# ------------------------------------------------------------------------------------------ nodes
class SwitchControlNode(ModuleNode):
    """Node wrapping ``SwitchOps``: output 1 is the false branch, output 2 the true branch."""

    def trueEdge(self):
        return (self, 2)

    def falseEdge(self):
        return (self, 1)

    true_edge = trueEdge
    false_edge = falseEdge

    def availableNodes(self) -> List[ModuleNode]:
        out = self.element.output
        nexts = list(zip(self.next_nodes, self._next_edges()))
        if any(e == 0 for _, e in nexts):
            raise ValueError("a Switch output must be taken through trueEdge()/falseEdge()")
        trues = _uniq(n for n, e in nexts if e == 2)
        falses = _uniq(n for n, e in nexts if e == 1)
        if any(n in falses for n in trues):
            raise ValueError("a node cannot take both edges of one Switch")
        return falses if (isinstance(out, Table) and out.get(1) is not None) else trues

    def _next_edges(self):
        edges = []
        for n in self.next_nodes:
            for p, i in zip(n.prev_nodes, n.prev_index):
                if p is self:
                    edges.append(i)
                    break
        return edges


class MergeControlNode(ModuleNode):
    def append(self, dependency):
        self(dependency)
        return self


def _uniq(it):
    seen, out = set(), []
    for n in it:
        if id(n) not in seen:
            seen.add(id(n))
            out.append(n)
    return out


# ------------------------------------------------------------------------------------------ frames
class Frame:
    __slots__ = ("name", "parent", "barrier", "waiting_nodes", "nodes")

    def __init__(self, name: str, parent: Optional["Frame"]):
        self.name, self.parent = name, parent
        self.barrier = 0                  # NextIteration nodes still to arrive this iteration
        self.waiting_nodes: List[ModuleNode] = []
        self.nodes: List[ModuleNode] = []  # nodes re-run on every iteration of the frame


class FrameManager:
    """Frame bookkeeping of one scheduler (``FrameManager.scala``)."""

    def __init__(self):
        self.frames: Dict[str, Frame] = {}
        self.node_frame: Dict[int, Frame] = {}

    def create_frame(self, name: str, parent: Optional[Frame]) -> Frame:
        if name not in self.frames:
            self.frames[name] = Frame(name, parent)
        return self.frames[name]

    def _bind(self, node, frame):
        cur = self.node_frame.get(node._id)
        if cur is not None and cur is not frame:
            raise RuntimeError(f"node {node.name()} cannot be in two frames at the same time")
        self.node_frame[node._id] = frame

    def enter(self, node: ModuleNode, frame: Frame):
        self._bind(node, frame)
        if node not in frame.nodes and self._repeats(node, frame):
            frame.nodes.append(node)

    def pend(self, node: ModuleNode, frame: Frame):
        if not isinstance(node.element, _tf().NextIteration):
            raise RuntimeError("only NextIteration nodes can be pended")
        self._bind(node, frame)
        frame.barrier -= 1
        frame.waiting_nodes.append(node)

    @staticmethod
    def _repeats(node, frame) -> bool:
        tf = _tf()
        # a loop starts at "NextIteration → Merge"; everything downstream of a repeating node repeats
        if isinstance(node.element, tf.MergeOps) and len(node.prev_nodes) == 2 and any(
                isinstance(p.element, tf.NextIteration) for p in node.prev_nodes):
            return True
        return any(p in frame.nodes for p in node.prev_nodes)

    def __call__(self, node) -> Optional[Frame]:
        return self.node_frame.get(node._id)


# ------------------------------------------------------------------------------------------ scheduler
_CONST, _READY = "const", "ready"


class Scheduler:
    """Ready-queue executor for graphs with data-dependent control flow (``Scheduler.scala``).

    Node status survives ``reset()`` for const nodes (those whose every input is const, e.g. a
    ``Const`` or shape arithmetic on it): they run once per scheduler lifetime, not once per run.
    """

    def __init__(self, input_nodes: Sequence[ModuleNode], output_nodes: Sequence[ModuleNode],
                 executable: Optional[set] = None):
        self.input_nodes = list(input_nodes)
        self.output_nodes = list(output_nodes)
        self.executable = executable
        self.queue: deque = deque()
        self.status: Dict[int, str] = {}
        self.frames = FrameManager()

    def reset(self):
        self.queue.clear()
        self.queue.extend(self.input_nodes)
        self.status = {k: v for k, v in self.status.items() if v == _CONST}

    def not_executed(self, node) -> bool:
        return node._id not in self.status

    def is_const(self, node) -> bool:
        return self.status.get(node._id) == _CONST

    def is_finished(self) -> bool:
        if not self.queue:
            for n in self.output_nodes:
                if self.not_executed(n):
                    raise RuntimeError(f"graph execution stalled: output {n.name()} was never reached")
            return True
        return False

    def fetch(self) -> ModuleNode:
        tf = _tf()
        while True:
            node = self.queue.popleft()
            if isinstance(node.element, tf.ControlDependency) or self.is_const(node):
                self.schedule(node)
                if not self.queue:
                    return None
                continue
            return node

    def schedule(self, node: ModuleNode):
        tf = _tf()
        el = node.element
        cur = self.frames(node)
        if isinstance(el, tf.Enter) and not isinstance(el, (tf.Exit, tf.NextIteration)):
            nxt_frame = self.frames.create_frame(el.frame, cur)
        elif isinstance(el, tf.LoopCondition):
            if cur is None:
                raise RuntimeError("LoopCondition must be inside a loop frame")
            if cur.barrier != 0:
                raise RuntimeError("frame barrier must be 0 when the loop condition runs")
            cur.barrier = len(node.next_nodes)
            nxt_frame = cur
        elif isinstance(el, tf.NextIteration):
            if cur is None:
                raise RuntimeError("NextIteration must be inside a loop frame")
            nxt_frame = cur
        elif isinstance(el, tf.Exit):
            if cur is None:
                raise RuntimeError("Exit must be inside a loop frame")
            cur.barrier = 0
            nxt_frame = cur.parent
        else:
            nxt_frame = cur
        if not self.is_const(node):
            if not node.prev_nodes:
                const = isinstance(el, tf.Const)
            else:
                const = all(self.is_const(p) for p in node.prev_nodes) and not getattr(el, "is_random", False)
            self.status[node._id] = _CONST if const else _READY
        nexts = node.availableNodes() if isinstance(node, SwitchControlNode) else node.next_nodes
        self._select_nexts(nexts, node, nxt_frame)

    def _select_nexts(self, candidates, cur, frame):
        tf = _tf()
        for nxt in _uniq(candidates):
            if self.executable is not None and nxt._id not in self.executable:
                continue
            if isinstance(nxt.element, tf.MergeOps):
                if not self.not_executed(nxt):
                    raise RuntimeError(f"Merge node {nxt.name()} ran twice outside a loop or in one iteration")
                nxt.element.setSwitch(nxt.prev_nodes.index(cur) + 1)
                self._enqueue(nxt, frame)
            elif self._ready(nxt):
                self._enqueue(nxt, frame)

    def _ready(self, node) -> bool:
        if any(self.not_executed(p) for p in node.prev_nodes):
            return False
        for p in node.prev_nodes:
            if isinstance(p, SwitchControlNode) and node not in p.availableNodes():
                return False
        return True

    def _enqueue(self, node, frame):
        if isinstance(node.element, _tf().NextIteration):
            if frame is None:
                raise RuntimeError("NextIteration must be inside a loop frame")
            self.frames.pend(node, frame)
            self.status.pop(node._id, None)
            if frame.barrier == 0:
                self._next_iteration(frame)
        else:
            if frame is not None:
                self.frames.enter(node, frame)
            self.queue.append(node)

    def _next_iteration(self, frame: Frame):
        self.queue.extend(frame.waiting_nodes)
        frame.waiting_nodes.clear()
        tf = _tf()
        for n in frame.nodes:
            if not isinstance(n.element, tf.NextIteration):
                self.status.pop(n._id, None)


# ------------------------------------------------------------------------------------------ graph
def _reachable_backward(outputs: Sequence[ModuleNode]) -> List[ModuleNode]:
    order, seen, stack = [], set(), list(outputs)
    while stack:
        n = stack.pop()
        if n._id in seen:
            continue
        seen.add(n._id)
        order.append(n)
        stack.extend(n.prev_nodes)
    return order


class DynamicGraph(Graph):
    """Graph executed by a :class:`Scheduler`; supports Switch/Merge branches and while loops.

    ``generate_backward`` (default True) enables backward for graphs without control-flow ops:
    gradients flow in reverse execution order, exactly as the static graph.
    """

    SCALA_NAME = "DynamicGraph"

    def __init__(self, inputs, outputs, variables=None, generate_backward: bool = True):
        from .containers import Container
        Container.__init__(self)
        self.inputs = list(inputs) if isinstance(inputs, (list, tuple)) else [inputs]
        self.outputs_nodes = list(outputs) if isinstance(outputs, (list, tuple)) else [outputs]
        self.generate_backward = generate_backward
        tf = _tf()
        nodes = _reachable_backward(self.outputs_nodes)
        ids = {n._id for n in nodes}
        for n in self.inputs:
            if n._id not in ids:
                nodes.append(n)
                ids.add(n._id)
        self._all_nodes = nodes
        self.modules = [n.element for n in reversed(nodes) if not isinstance(n.element, tf.ControlDependency)]
        self._stop_grad = set()
        self._has_control = any(isinstance(n.element, (tf.SwitchOps, tf.MergeOps, tf.Enter, tf.LoopCondition))
                                for n in nodes)
        if generate_backward and self._has_control:
            raise ValueError("backward cannot be generated for a graph with control-flow ops "
                             "(pass generate_backward=False)")
        starts = [n for n in reversed(nodes) if not n.prev_nodes]
        self._scheduler = Scheduler(starts, self.outputs_nodes, ids)
        self._acts: Dict[int, object] = {}
        self.forward_order: List[ModuleNode] = []
        self.variables = variables

    def _node_input(self, n, acts):
        vals = []
        for p, idx in zip(n.prev_nodes, n.prev_index):
            a = acts.get(p._id)
            vals.append(a.get(idx) if (idx and isinstance(a, Table)) else a)
        if not vals:
            return None
        return vals[0] if len(vals) == 1 else Table(*vals)

    def updateOutput(self, input):
        s = self._scheduler
        s.reset()
        feeds = {}
        if len(self.inputs) == 1:
            feeds[self.inputs[0]._id] = input
        elif self.inputs:
            feeds = {n._id: input[i + 1] for i, n in enumerate(self.inputs)}
        acts = self._acts
        self._node_inputs = {}
        order = []
        while not s.is_finished():
            n = s.fetch()
            if n is None:
                continue
            x = feeds[n._id] if n._id in feeds else self._node_input(n, acts)
            self._node_inputs[n._id] = x
            acts[n._id] = n.element.forward(x)
            order.append(n)
            s.schedule(n)
        # const nodes skipped this run still feed backward through their cached activities
        self.forward_order = order
        outs = [acts[o._id] for o in self.outputs_nodes]
        self.output = outs[0] if len(outs) == 1 else Table(*outs)
        return self.output

    def _backward_impl(self, input, gradOutput, call):
        if not self.generate_backward:
            return None
        return super()._backward_impl(input, gradOutput, call)

    def accGradParameters(self, input, gradOutput):
        if self.generate_backward:
            super().accGradParameters(input, gradOutput)


def dynamic(inputs, outputs, variables=None, generate_backward: bool = True) -> DynamicGraph:
    """``Graph.dynamic(inputs, outputs, variables, generateBackward)``."""
    return DynamicGraph(inputs, outputs, variables, generate_backward)


Graph.dynamic = staticmethod(dynamic)


# ------------------------------------------------------------------------------------------ builders
class ControlNodes:
    """Builders for control-flow subgraphs (``ControlNodes`` in ``nn/tf/ControlOps.scala``)."""

    @staticmethod
    def switch(data: ModuleNode, condition: ModuleNode) -> SwitchControlNode:
        n = SwitchControlNode(_tf().SwitchOps())
        n(data, condition)
        return n

    @staticmethod
    def merge(*nodes) -> MergeControlNode:
        n = MergeControlNode(_tf().MergeOps())
        n(*nodes)
        return n

    @staticmethod
    def whileLoop(condition, body, loop_vars, name: Optional[str] = None) -> List[ModuleNode]:
        """``condition = (cond_inputs, cond_output)``; ``body = [(body_input, body_output), ...]``;
        ``loop_vars`` are the initial-value nodes.  Returns one Exit node per loop variable.
        The loop exits when ``cond_output`` is true."""
        tf = _tf()
        cond_inputs, cond_out = condition
        lc = ModuleNode(tf.LoopCondition())(cond_out)
        if name:
            lc.set_name(f"{name}/loopCondition")
        exits = []
        for i, ((inp, cin), (b_in, b_out)) in enumerate(zip(zip(loop_vars, cond_inputs), body), start=1):
            enter = ModuleNode(tf.Enter(name or "while_frame"))(inp)
            merge = ControlNodes.merge(enter)
            cin(merge)
            sw = ControlNodes.switch(merge, lc)
            ex = ModuleNode(tf.Exit())(sw.trueEdge())
            ident = ModuleNode(Identity())(sw.falseEdge())
            b_in(ident)
            nxt = ModuleNode(tf.NextIteration())(b_out)
            merge.append(nxt)
            if name:
                for nd, nm in ((enter, "enter"), (merge, "merge"), (sw, "switch"), (ex, "exit"),
                               (ident, "switchFalse"), (nxt, "nextIteration")):
                    nd.set_name(f"{name}/{nm}{i}")
            exits.append(ex)
        return exits

    while_loop = whileLoop
