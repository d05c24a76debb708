"""TensorFlow data-flow resources: TensorArray*, Stack* and AssignGrad (``DL/nn/tf/DataFlowOps.scala``,
``StateOps.scala``).  The graph cases reproduce the reference's specs
(``nn/ops/TensorArray{Scatter,Write,Split}Spec.scala``, ``nn/tf/StackOpsSpec.scala``: the same dynamic
graphs, run and round-tripped through ``.bigdl``) with value checks, and a TF 1.x GraphDef using
TensorArrayV3 ops loads through ``TensorflowLoader`` and runs in the TF graph executor (the values
``tensor_array.py`` in the reference's TF test resources computes: scatter→gather and
split→concat are identities, size reads the array length)."""
import pytest
import torch

from bigdl.nn import Graph, Identity
from bigdl.nn.graph import ModuleNode
import bigdl.nn.tf as TF
from bigdl.utils.table import Table


def _const(v):
    return ModuleNode(TF.Const(v))


def test_scatter_gather_close():
    data = torch.rand(3, 4)
    ta = TF.TensorArrayCreator()()
    idx = _const(torch.tensor([0, 1, 2], dtype=torch.int32))
    d = _const(data)
    scatter = TF.TensorArrayScatter()((ta, 1), (idx, 1), (d, 1))
    ctr = TF.ControlDependency()(scatter)
    gather = TF.TensorArrayGather()((ta, 1), (idx, 1), (ctr, 1))
    ctr2 = TF.ControlDependency()(gather)
    close = TF.TensorArrayClose()((ta, 1), (ctr2, 1))
    g = Graph.dynamic([ta], [gather, close])
    out = g.forward(torch.tensor(10, dtype=torch.int32))
    torch.testing.assert_close(out[1], data)
    assert float(out[2]) == 0.0  # the flow scalar
    h = ta.element.output[1]
    assert not TF.TensorArray.exist(h)  # closed


def test_write_read_and_grad_array():
    ta = TF.TensorArrayCreator()()
    d = _const(torch.tensor(1.0))
    i0 = _const(torch.tensor(0, dtype=torch.int32))
    write = TF.TensorArrayWrite()((ta, 1), (i0, 1), (d, 1))
    ctr = TF.ControlDependency()(write)
    read = TF.TensorArrayRead()((ta, 1), (i0, 1), (ctr, 1))
    grad = TF.TensorArrayGrad("grad")(ta)
    out = Identity()((grad, 2))
    g = Graph.dynamic([ta], [read, out])
    r = g.forward(torch.tensor(1, dtype=torch.int32))
    assert float(r[1]) == 1.0 and float(r[2]) == 0.0
    src = ta.element.output[1]
    ga = TF.TensorArray.get(src + "grad")
    assert ga.size() == 1 and ga.multiple_writes_aggregate
    # gradient arrays aggregate repeated writes; source arrays refuse them (and clear after a read)
    ga[0] = torch.tensor(2.0)
    ga[0] = torch.tensor(3.0)
    assert float(ga[0]) == 5.0
    arr = TF.TensorArray(2)
    arr[1] = torch.tensor(1.0)
    with pytest.raises(ValueError):
        arr[1] = torch.tensor(2.0)
    with pytest.raises(ValueError):
        arr[2] = torch.tensor(2.0)  # fixed size
    assert float(arr[1]) == 1.0
    with pytest.raises(ValueError):
        arr[1]  # cleared after read
    dyn = TF.TensorArray(1, dynamic_size=True)
    dyn[3] = torch.ones(2)
    assert dyn.size() == 4


def test_split_concat_size():
    data = torch.rand(3, 4)
    ta = TF.TensorArrayCreator()()
    d = _const(data)
    lengths = _const(torch.tensor([1, 2], dtype=torch.int32))
    split = TF.TensorArraySplit()((ta, 1), (d, 1), (lengths, 1))
    ctr = TF.ControlDependency()(split)
    concat = TF.TensorArrayConcat()(ta, ctr)
    size = TF.TensorArraySize()(ta, ctr)
    ctr2 = TF.ControlDependency()(concat, size)
    close = TF.TensorArrayClose()((ta, 1), (ctr2, 1))
    g = Graph.dynamic([ta], [concat, close, size])
    out = g.forward(torch.tensor(2, dtype=torch.int32))
    torch.testing.assert_close(out[1][1], data)
    assert out[1][2].tolist() == [1, 2]
    assert int(out[3]) == 2


def test_stack_push_pop():
    d = _const(torch.tensor(1.0))
    stack = TF.StackCreator()()
    push = TF.StackPush()(stack, d)
    ctr = TF.ControlDependency()(push)
    pop = TF.StackPop()(stack, ctr)
    g = Graph.dynamic([stack], [pop])
    assert float(g.forward(torch.tensor(1))) == 1.0
    s = TF.data_flow._Stack(1)
    s.push(torch.ones(1))
    with pytest.raises(ValueError):
        s.push(torch.ones(1))  # bounded by the creator's max size
    assert float(s.pop()) == 1.0
    with pytest.raises(ValueError):
        s.pop()


def test_assign_grad_copies_into_its_gradient():
    g = torch.zeros(3)
    m = TF.AssignGrad(g)
    assert m.forward(torch.tensor([1.0, 2.0, 3.0])) is None
    assert g.tolist() == [1.0, 2.0, 3.0]


def test_data_flow_graph_round_trips_through_bigdl(tmp_path):
    from bigdl.serialization import module_serializer as ms
    data = torch.rand(3, 4)
    ta = TF.TensorArrayCreator()()
    idx = _const(torch.tensor([0, 1, 2], dtype=torch.int32))
    scatter = TF.TensorArrayScatter()((ta, 1), (idx, 1), (_const(data), 1))
    gather = TF.TensorArrayGather()((ta, 1), (idx, 1), (TF.ControlDependency()(scatter), 1))
    g = Graph.dynamic([ta], [gather])
    p = str(tmp_path / "ta.bigdl")
    ms.save_module(g, p, over_write=True)
    g2 = ms.load_module(p)
    torch.testing.assert_close(g2.forward(torch.tensor(3, dtype=torch.int32)), data)


def _tensor_array_graphdef(path):
    from bigdl.utils.tf.proto import graph_classes, torch_to_tensor
    classes, _ = graph_classes()
    gd = classes["tensorflow.GraphDef"]()

    def node(name, op, inputs=(), **attrs):
        n = gd.node.add()
        n.name, n.op = name, op
        n.input.extend(inputs)
        for k, v in attrs.items():
            if isinstance(v, torch.Tensor):
                n.attr[k].tensor.CopyFrom(torch_to_tensor(v))
            elif isinstance(v, bool):
                n.attr[k].b = v
            elif isinstance(v, str):
                n.attr[k].s = v.encode()
        return n
    node("x", "Placeholder")
    node("n", "Const", value=torch.tensor(3, dtype=torch.int32))
    node("idx", "Const", value=torch.tensor([0, 1, 2], dtype=torch.int32))
    node("ta", "TensorArrayV3", ["n"], clear_after_read=True, dynamic_size=False)
    node("scatter", "TensorArrayScatterV3", ["ta", "idx", "x", "ta:1"])
    node("gather", "TensorArrayGatherV3", ["ta", "idx", "scatter"])
    node("out", "Identity", ["gather"])
    node("n2", "Const", value=torch.tensor(2, dtype=torch.int32))
    node("ta2", "TensorArrayV3", ["n2"])
    node("lens", "Const", value=torch.tensor([1, 2], dtype=torch.int32))
    node("split", "TensorArraySplitV3", ["ta2", "x", "lens", "ta2:1"])
    node("concat", "TensorArrayConcatV3", ["ta2", "split"])
    node("size", "TensorArraySizeV3", ["ta2", "split"])
    node("concat_value", "Identity", ["concat:0"])
    with open(path, "wb") as f:
        f.write(gd.SerializeToString())


def test_tensor_array_graphdef_loads_and_runs(tmp_path):
    from bigdl.utils.tf import TensorflowLoader
    p = str(tmp_path / "tensor_array.pb")
    _tensor_array_graphdef(p)
    x = torch.rand(3, 4)
    g = TensorflowLoader.load(p, ["x"], ["out"])
    torch.testing.assert_close(g.forward(x), x)
    g2 = TensorflowLoader.load(p, ["x"], ["concat_value", "size"])
    out = g2.forward(x)
    # (a graph output is a whole node: the Identity of concat:0 resolves to concat's Table output)
    torch.testing.assert_close(out[1][1], x)
    assert out[1][2].tolist() == [1, 2]
    assert int(out[2]) == 2


def test_tensor_array_graphdef_in_executor(tmp_path):
    from bigdl.utils.tf import TensorflowLoader
    from bigdl.utils.tf.executor import GraphExecutor
    p = str(tmp_path / "tensor_array.pb")
    _tensor_array_graphdef(p)
    ex = GraphExecutor(TensorflowLoader.parse(p))
    x = torch.rand(3, 4)
    out, concat, size = ex.run(["out", "concat", "size"], feeds={"x": x})
    torch.testing.assert_close(out, x)
    torch.testing.assert_close(concat, x)
    assert int(size) == 2
