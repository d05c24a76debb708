"""DynamicGraph / Scheduler / ControlNodes (``DL/nn/DynamicGraph.scala``, ``Scheduler.scala``,
``nn/tf/ControlOps.scala``); cases mirror ``TS/nn/DynamicGraphSpec.scala`` while-loop specs."""
import torch
import pytest

from bigdl.nn import (Input, Linear, AddConstant, Echo, ReLU, Graph, DynamicGraph, ControlNodes, CAddTable,
                      MSECriterion)
import importlib
O = importlib.import_module("bigdl.nn.ops")
from bigdl.nn import tf as TF
from bigdl.nn.graph import ModuleNode


def _while_plus_one(const_input=False, counter=None):
    inp = ModuleNode(TF.Const(torch.tensor([1.0]))) if const_input else Input()
    cond_in = Input()
    c9 = ModuleNode(TF.Const(torch.tensor([9.0])))

    def feval(m, x):
        if counter is not None:
            counter.append(1)
    echo = Echo(feval)(c9)
    less = O.Less()(echo, cond_in)
    upd_in = Input()
    add = AddConstant(1)(upd_in)
    exits = ControlNodes.whileLoop(([cond_in], less), [(upd_in, add)], [inp], "while")
    return inp, exits


def test_while_loop_counts_to_ten():
    inp, exits = _while_plus_one()
    g = DynamicGraph([inp], [exits[0]], None, False)
    assert float(g.forward(torch.tensor([1.0]))[0]) == 10.0


def test_while_loop_twice_const_once():
    cnt = []
    inp, exits = _while_plus_one(counter=cnt)
    g = Graph.dynamic([inp], [exits[0]], None, False)
    g.forward(torch.tensor([1.0]))
    r = g.forward(torch.tensor([3.0]))
    assert float(r[0]) == 10.0
    assert len(cnt) == 1  # the const subgraph ran once over both executions


def test_while_loop_const_start_no_inputs():
    inp, exits = _while_plus_one(const_input=True)
    g = DynamicGraph([], [exits[0]], None, False)
    assert float(g.forward(None)[0]) == 10.0
    assert float(g.forward(None)[0]) == 10.0


def test_switch_merge_branches():
    data = Input()
    pred = Input()
    sw = ControlNodes.switch(data, pred)
    t = AddConstant(10)(sw.trueEdge())
    f = AddConstant(-10)(sw.falseEdge())
    m = ControlNodes.merge(t, f)
    g = DynamicGraph([data, pred], [m], None, False)
    from bigdl.utils.table import Table
    assert float(g.forward(Table(torch.tensor([1.0]), torch.tensor(True)))[0]) == 11.0
    assert float(g.forward(Table(torch.tensor([1.0]), torch.tensor(False)))[0]) == -9.0


def test_dynamic_graph_backward_matches_static():
    torch.manual_seed(0)
    x = Input()
    l1 = Linear(4, 3)(x)
    r = ReLU()(l1)
    l2 = Linear(4, 3)(x)
    out = CAddTable()(r, l2)
    dg = DynamicGraph([x], [out])
    sg = Graph([x], [out])
    xin = torch.randn(5, 4)
    y1 = dg.forward(xin).clone()
    y2 = sg.forward(xin).clone()
    assert torch.allclose(y1, y2)
    gy = torch.randn(5, 3)
    dg.zeroGradParameters()
    g1 = dg.backward(xin, gy).clone()
    w1 = [t.clone() for t in dg.parameters()[1]]
    dg.zeroGradParameters()
    g2 = sg.backward(xin, gy).clone()
    w2 = sg.parameters()[1]
    assert torch.allclose(g1, g2)
    for a, b in zip(w1, w2):
        assert torch.allclose(a, b)


def test_control_ops_refuse_generated_backward():
    inp, exits = _while_plus_one()
    with pytest.raises(ValueError):
        DynamicGraph([inp], [exits[0]])
