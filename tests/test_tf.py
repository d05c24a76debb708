"""TensorFlow interop and TF op layers.  Fixtures under tests/fixtures/tf are the reference's own
test resources (``spark/dl/src/test/resources/tf``: a frozen 2-layer MLP ``test.pb``, typed
constants ``consts.pbtxt``, TFRecord files); expectations follow ``TensorflowLoaderSpec``,
``TFUtilsSpec`` and the ops specs."""
import os

import numpy as np
import pytest
import torch

from bigdl.nn import Sequential, Linear, Tanh, ReLU, SpatialConvolution, SpatialMaxPooling, Reshape, SoftMax
from bigdl.nn import ops as _nn_ops_attr  # noqa: F401  (bigdl.nn namespace)
from bigdl.utils.table import Table
from bigdl.utils.tf import TensorflowLoader, TensorflowSaver, TFRecordIterator, TFRecordWriter
from bigdl.utils.tf.proto import example_classes, tensor_to_torch
import bigdl.nn.ops as O
import bigdl.nn.tf as T

FX = os.path.join(os.path.dirname(__file__), "fixtures", "tf")


def _mlp_ref():
    m = Sequential()
    fc1 = Linear(1, 10)
    fc1.weight.data.fill_(0.2)
    fc1.bias.data.fill_(0.1)
    fc2 = Linear(10, 1)
    fc2.weight.data.fill_(0.2)
    fc2.bias.data.fill_(0.1)
    return m.add(fc1).add(Tanh()).add(fc2)


def test_parse_pb():
    assert len(TensorflowLoader.parse(os.path.join(FX, "test.pb"))) == 14


def test_load_graph_matches_reference_mlp():
    g = TensorflowLoader.load(os.path.join(FX, "test.pb"), ["Placeholder"], ["output"])
    assert len(g.modules) == 4  # input, fused Linear, Tanh, fused Linear
    x = torch.rand(4, 1)
    torch.testing.assert_close(g.forward(x), _mlp_ref().forward(x))


def test_load_from_inner_tensor_and_subgraph():
    g = TensorflowLoader.load(os.path.join(FX, "test.pb"), ["MatMul:0"], ["output"])
    assert len(g.modules) == 4
    g2 = TensorflowLoader.load(os.path.join(FX, "test.pb"), ["Tanh"], ["output"])
    assert len(g2.modules) == 3
    x = torch.rand(4, 10)
    ref = Sequential().add(Tanh()).add(Linear(10, 1))
    ref.modules[1].weight.data.fill_(0.2)
    ref.modules[1].bias.data.fill_(0.1)
    torch.testing.assert_close(g2.forward(x), ref.forward(x))


@pytest.mark.parametrize("inputs", [["Placeholder", "Placeholder"], ["Placeholder", "Placeholder:0"], ["MatMul:2"]])
def test_load_rejects_bad_inputs(inputs):
    with pytest.raises(ValueError):
        TensorflowLoader.load(os.path.join(FX, "test.pb"), inputs, ["output"])


def test_loaded_graph_is_trainable():
    g = TensorflowLoader.load(os.path.join(FX, "test.pb"), ["Placeholder"], ["output"])
    x = torch.rand(4, 1)
    y = g.forward(x)
    g.zeroGradParameters()
    g.backward(x, torch.ones_like(y))
    ws, gs = g.parameters()
    assert len(ws) == 4 and all(float(gg.abs().sum()) > 0 for gg in gs)


def test_parse_typed_consts():
    vals = {n.name: tensor_to_torch(n.attr["value"].tensor) for n in TensorflowLoader.parse(os.path.join(FX, "consts.pbtxt"))}
    assert vals["bool_const"].tolist() == [True, False, True, False]
    assert vals["float_const"].tolist() == [1.0, 2.0, 3.0, 4.0]
    assert vals["double_const"].dtype == torch.float64
    for k in ("int_const", "long_const", "int8_const", "uint8_const", "int16_const", "uint16_const"):
        assert vals[k].tolist() == [1, 2, 3, 4], k
    assert vals["string_const"] == [b"a", b"b", b"c", b"d"]


def test_saver_roundtrip_conv_net(tmp_path):
    torch.manual_seed(0)
    m = (Sequential().add(SpatialConvolution(3, 4, 3, 3, 1, 1, 1, 1)).add(ReLU())
         .add(SpatialMaxPooling(2, 2, 2, 2)).add(Reshape([4 * 4 * 4])).add(Linear(64, 5)).add(SoftMax()))
    m.reset()
    m.evaluate()
    x = torch.randn(2, 3, 8, 8)
    ref = m.forward(x)
    p = str(tmp_path / "net.pb")
    TensorflowSaver.save_graph(m, [("input", [-1, 3, 8, 8])], p)
    g = TensorflowLoader.load(p, ["input"], ["output"])
    torch.testing.assert_close(g.forward(x), ref, atol=1e-5, rtol=1e-4)


def test_saver_roundtrip_mlp(tmp_path):
    m = _mlp_ref()
    p = str(tmp_path / "mlp.pb")
    TensorflowSaver.save_graph(m, [("x", [-1, 1])], p)
    g = TensorflowLoader.load(p, ["x"], ["output"])
    x = torch.rand(3, 1)
    torch.testing.assert_close(g.forward(x), m.forward(x))


def test_tfrecord_read_write_and_parse_example(tmp_path):
    recs = list(TFRecordIterator(os.path.join(FX, "mnist_train.tfrecord")))
    assert len(recs) == 10
    assert list(TFRecordIterator(os.path.join(FX, "text.tfrecord"))) == [b"abcd"]
    out = T.ParseExample(["image/class/label", "image/height"], [torch.int64, torch.int64], [[1], [1]]).forward(recs)
    assert out[1].shape == (10, 1) and out[2].flatten().tolist() == [28] * 10
    p = str(tmp_path / "x.tfrecord")
    with TFRecordWriter(p) as w:
        for r in recs[:3]:
            w.write(r)
    assert list(TFRecordIterator(p)) == recs[:3]


def test_decode_image_from_tfrecord():
    E = example_classes()["tensorflow.Example"]
    for r in TFRecordIterator(os.path.join(FX, "decode_image_test_case.tfrecord")):
        f = E.FromString(r).features.feature
        data = f["image/encoded"].bytes_list.value[0]
        h, w = f["image/height"].int64_list.value[0], f["image/width"].int64_list.value[0]
        if f["image/format"].bytes_list.value[0] == b"raw":
            img = T.DecodeRaw(torch.uint8).forward(data).view(h, w, 1)
        else:
            img = T.DecodeImage(3).forward(data)
        assert tuple(img.shape[:2]) == (h, w) and img.dtype == torch.uint8


# ------------------------------------------------------------------------------------------------ ops
def test_elementwise_and_compare_ops():
    a, b = torch.tensor([1.0, -2.0, 3.5]), torch.tensor([2.0, -2.0, 1.0])
    assert O.Equal().forward(Table(a, b)).tolist() == [False, True, False]
    assert O.Greater().forward(Table(a, b)).tolist() == [False, False, True]
    assert O.FloorDiv().forward(Table(torch.tensor([7.0, -7.0]), torch.tensor([2.0, 2.0]))).tolist() == [3.0, -4.0]
    assert O.TruncateDiv().forward(Table(torch.tensor([7.0, -7.0]), torch.tensor([2.0, 2.0]))).tolist() == [3.0, -3.0]
    assert O.FloorMod().forward(Table(torch.tensor([-7.0]), torch.tensor([3.0]))).tolist() == [2.0]
    assert O.Mod().forward(Table(torch.tensor([-7.0]), torch.tensor([3.0]))).tolist() == [-1.0]
    assert O.Rint().forward(torch.tensor([0.5, 1.5, 2.5])).tolist() == [0.0, 2.0, 2.0]
    assert float(O.L2Loss().forward(torch.tensor([1.0, 2.0]))) == 2.5
    with pytest.raises(NotImplementedError):
        O.Exp().backward(a, a)


def test_index_ops():
    x = torch.arange(12.0).view(3, 4)
    assert O.Gather().forward(Table(x, torch.tensor([2, 0]))).tolist() == [x[2].tolist(), x[0].tolist()]
    oh = O.OneHot().forward(Table(torch.tensor([0, 2, -1]), torch.tensor(3), torch.tensor(1.0), torch.tensor(0.0)))
    assert oh.tolist() == [[1, 0, 0], [0, 0, 1], [0, 0, 0]]
    v, i = O.TopK(2).forward(torch.tensor([[1.0, 5.0, 3.0]])).values()
    assert v.tolist() == [[5.0, 3.0]] and i.tolist() == [[2, 3]]  # 1-based indices (startIndex = 1)
    assert O.InTopK(1).forward(Table(torch.tensor([[0.1, 0.9], [0.8, 0.2]]), torch.tensor([2, 2]))).tolist() == [True, False]
    s = O.SegmentSum().forward(Table(torch.tensor([[1.0], [2.0], [3.0]]), torch.tensor([0, 0, 1])))
    assert s.flatten().tolist() == [3.0, 3.0]
    assert O.Sum(False).forward(Table(x, torch.tensor([1]))).tolist() == x.sum(1).tolist()
    assert O.Tile().forward(Table(torch.tensor([1, 2]), torch.tensor([2]))).tolist() == [1, 2, 1, 2]
    assert O.Slice([1, 0], [-1, 2]).forward(x).tolist() == x[1:, :2].tolist()
    assert O.Pad().forward(Table(torch.ones(1, 2), torch.tensor([[1, 0], [0, 1]]))).shape == (2, 3)


def test_strided_slice_masks():
    x = torch.arange(24).view(2, 3, 4)
    ss = T.StridedSlice(shrink_axis_mask=1)
    out = ss.forward(Table(x, torch.tensor([1, 0, 0]), torch.tensor([2, 3, 4]), torch.tensor([1, 1, 2])))
    assert out.tolist() == x[1, :, ::2].tolist()
    rev = T.StridedSlice(begin_mask=1, end_mask=1).forward(Table(torch.arange(5), torch.tensor([0]), torch.tensor([0]),
                                                               torch.tensor([-1])))
    assert rev.tolist() == [4, 3, 2, 1, 0]


def test_tf_conv_and_pool_match_torch():
    torch.manual_seed(0)
    x = torch.randn(2, 7, 7, 3)
    f = torch.randn(3, 3, 3, 5)
    y = T.Conv2D([1, 2, 2, 1], "SAME").forward(Table(x, f))
    assert y.shape == (2, 4, 4, 5)
    ref = torch.nn.functional.conv2d(torch.nn.functional.pad(x.permute(0, 3, 1, 2), (1, 1, 1, 1)),
                                     f.permute(3, 2, 0, 1), stride=2).permute(0, 2, 3, 1)
    torch.testing.assert_close(y, ref, atol=1e-5, rtol=1e-5)
    p = T.AvgPool([1, 2, 2, 1], [1, 2, 2, 1], "SAME").forward(torch.ones(1, 3, 3, 1))
    assert torch.allclose(p, torch.ones(1, 2, 2, 1))  # padded cells excluded from the mean


def test_feature_columns():
    b = O.BucketizedCol([0.0, 10.0, 100.0]).forward(torch.tensor([-1.0, 5.0, 50.0, 500.0]))
    assert b.tolist() == [0, 1, 2, 3]
    sp = O.CategoricalColVocaList(["a", "b", "c"]).forward(["a,c", "b"])
    assert sp[2].tolist() == [0, 2, 1]
    ind = O.IndicatorCol(3).forward(sp)
    assert ind.tolist() == [[1, 0, 1], [0, 1, 0]]
    h = O.CategoricalColHashBucket(10).forward(["x,y", "z"])
    assert ((h[2] >= 0) & (h[2] < 10)).all()
    kv = O.Kv2Tensor(fea_len=4).forward(["0:1.5,3:2", "1:1"])
    assert kv.tolist() == [[1.5, 0, 0, 2.0], [0, 1.0, 0, 0]]


def _while_graphdef(path, limit=10.0):
    """``i = x; while i < limit: i = i + 1`` as TF 1.x emits it (Enter/Merge/LoopCond/Switch/
    Identity/NextIteration/Exit), written as a binary GraphDef."""
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
            elif isinstance(v, str):
                n.attr[k].s = v.encode()
            elif isinstance(v, bool):
                n.attr[k].b = v
        return n
    node("x", "Placeholder")
    node("limit", "Const", value=torch.tensor(limit))
    node("one", "Const", value=torch.tensor(1.0))
    node("while/Enter", "Enter", ["x"], frame_name="while/ctx")
    node("while/Merge", "Merge", ["while/Enter", "while/NextIteration"])
    node("while/Less/y", "Enter", ["limit"], frame_name="while/ctx", is_constant=True)
    node("while/Less", "Less", ["while/Merge", "while/Less/y"])
    node("while/LoopCond", "LoopCond", ["while/Less"])
    node("while/Switch", "Switch", ["while/Merge", "while/LoopCond"])
    node("while/Identity", "Identity", ["while/Switch:1"])
    node("while/add/y", "Enter", ["one"], frame_name="while/ctx", is_constant=True)
    node("while/add", "Add", ["while/Identity", "while/add/y"])
    node("while/NextIteration", "NextIteration", ["while/add"])
    node("while/Exit", "Exit", ["while/Switch"])
    node("out", "Mul", ["while/Exit", "one"])
    with open(path, "wb") as f:
        f.write(gd.SerializeToString())


def test_load_while_loop_as_dynamic_graph(tmp_path):
    from bigdl.nn import DynamicGraph
    p = str(tmp_path / "while.pb")
    _while_graphdef(p)
    g = TensorflowLoader.load(p, ["x"], ["out"])
    assert isinstance(g, DynamicGraph)
    assert float(g.forward(torch.tensor(1.0))) == 10.0
    assert float(g.forward(torch.tensor(-3.5))) == 10.5
    assert float(g.forward(torch.tensor(12.0))) == 12.0  # zero trips


def test_hash_bucket_matches_reference_golden():
    """``CategoricalColHashBucketSpec``: "1","2","3" → buckets 5, 53, 77 of 100 (Scala MurmurHash3)."""
    from bigdl.utils.hash_func import stringHashBucket32
    assert [stringHashBucket32(s, 100) for s in ("1", "2", "3")] == [5, 53, 77]
    sp = O.CategoricalColHashBucket(100).forward(["1,2", "2", "1,3,2"])
    assert sp[2].tolist() == [5, 53, 53, 5, 77, 53]
    # CrossColSpec goldens (two and three columns)
    c2 = O.CrossCol(100).forward(Table(["A,D", "B", "A,C"], ["1", "2", "3,4"]))
    assert c2[2].tolist() == [80, 98, 50, 99, 27, 89, 33]
    c3 = O.CrossCol(100).forward(Table(["A,D", "B", "A,C"], ["1", "2", "3,4"], ["1", "2", "3"]))
    assert c3[2].tolist() == [94, 34, 68, 82, 83, 97, 12]
