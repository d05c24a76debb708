"""Caffe import/export (reference: TS/utils/CaffeLoaderSpec.scala, CaffePersisterSpec.scala,
pyspark/test/bigdl/caffe/test_load_caffe.py).  Fixtures: the reference's own test.prototxt /
test.caffemodel (parsed with our re-declared caffe.proto; plain protobuf, nothing executed)."""
import os

import pytest
import torch

from bigdl.nn import (Graph, Input, JoinTable, Linear, ReLU, Sequential, SoftMax, SpatialConvolution,
                      SpatialCrossMapLRN, SpatialMaxPooling, SpatialAveragePooling, View, SpatialBatchNormalization,
                      CAddTable)
from bigdl.serialization.caffe_loader import CaffeLoader, CaffeConversionException, Customizable, load_caffe_model
from bigdl.serialization.caffe_persister import CaffePersister

RES = "/root/reference/spark/dl/src/test/resources/caffe"
PROTO, MODEL = os.path.join(RES, "test.prototxt"), os.path.join(RES, "test.caffemodel")
have_fixtures = pytest.mark.skipif(not os.path.exists(MODEL), reason="reference caffe fixtures not present")

CONV1_HEAD = [0.4156779647, 0.3547672033, 0.1817495823, -0.1393318474, 0.4004031420, 0.0634599924]
CONV1_BIAS = [0.0458712392, -0.0029324144, -0.0251041390, 0.0052924110]
CONV2_HEAD = [0.0154178329, 0.0157190431, 0.0033829932, -0.0048461366]
IP_HEAD = [0.0189033747, 0.0401176214, 0.0525088012, 0.3013394773]


def _small():
    return (Sequential().add(SpatialConvolution(3, 4, 2, 2).set_name("conv"))
            .add(SpatialConvolution(4, 3, 2, 2).set_name("conv2"))
            .add(Linear(27, 2, with_bias=False).set_name("ip")))


@have_fixtures
def test_load_weights_match_all():
    m = CaffeLoader.load(_small(), PROTO, MODEL)
    p = m.getParametersTable()
    torch.testing.assert_close(p["conv"]["weight"].reshape(-1)[:6], torch.tensor(CONV1_HEAD), atol=1e-6, rtol=0)
    torch.testing.assert_close(p["conv"]["bias"], torch.tensor(CONV1_BIAS), atol=1e-6, rtol=0)
    torch.testing.assert_close(p["conv2"]["weight"].reshape(-1)[:4], torch.tensor(CONV2_HEAD), atol=1e-6, rtol=0)
    torch.testing.assert_close(p["conv2"]["bias"], torch.zeros(3))
    torch.testing.assert_close(p["ip"]["weight"].reshape(-1)[:4], torch.tensor(IP_HEAD), atol=1e-6, rtol=0)


@have_fixtures
def test_load_weights_partial():
    m = _small()
    m.modules[1].set_name("conv3")
    before = m.modules[1].weight.clone()
    with pytest.raises(CaffeConversionException):
        CaffeLoader.load(_small().add(Linear(2, 2).set_name("nope")), PROTO, MODEL, match_all=True)
    CaffeLoader.load(m, PROTO, MODEL, match_all=False)
    torch.testing.assert_close(m.modules[1].weight, before)
    torch.testing.assert_close(m.modules[0].bias, torch.tensor(CONV1_BIAS), atol=1e-6, rtol=0)


@have_fixtures
def test_load_caffe_dynamic_and_customized():
    from bigdl.nn import Identity
    from bigdl.nn.graph import ModuleNode

    class Dummy(Customizable):
        def convertor(self, layer):
            return [ModuleNode(Identity().set_name("Dummy"))]

    g, crit = CaffeLoader.loadCaffe(PROTO, MODEL, {"DUMMY": Dummy()})
    p = g.getParametersTable()
    torch.testing.assert_close(p["conv"]["bias"], torch.tensor(CONV1_BIAS), atol=1e-6, rtol=0)
    x = torch.randn(2, 3, 5, 5)
    ref = _small()
    ref.modules.insert(2, View(27).setNumInputDims(3))
    CaffeLoader.load(ref, PROTO, MODEL)
    expected = torch.softmax(ref.forward(x), -1)
    torch.testing.assert_close(g.forward(x), expected, rtol=1e-5, atol=1e-6)
    assert len(crit.criterions) == 1  # SoftmaxWithLoss → ClassNLLCriterion
    with pytest.raises(CaffeConversionException):
        CaffeLoader.loadCaffe(PROTO, MODEL)
    g2 = load_caffe_model(PROTO, MODEL)  # Python API: unknown types → Identity
    torch.testing.assert_close(g2.forward(x), expected, rtol=1e-5, atol=1e-6)


def _inception_like():
    inp = Input()
    c1 = SpatialConvolution(3, 8, 3, 3, 1, 1, 1, 1).set_name("conv1")(inp)
    r1 = ReLU(True).set_name("relu1")(c1)
    n1 = SpatialCrossMapLRN(5, 1e-4, 0.75).set_name("norm1")(r1)
    p1 = SpatialMaxPooling(3, 3, 2, 2).ceil().set_name("pool1")(n1)
    b1 = SpatialConvolution(8, 4, 1, 1).set_name("b1")(p1)
    b2 = SpatialConvolution(8, 6, 3, 3, 1, 1, 1, 1).set_name("b2")(p1)
    cat = JoinTable(2, 0).set_name("cat")(b1, b2)
    bn = SpatialBatchNormalization(10, 1e-3).set_name("bn")(cat)
    s = CAddTable().set_name("sum")(bn, cat)
    ap = SpatialAveragePooling(4, 4, 4, 4).ceil().set_name("pool2")(s)
    v = View(10 * 4).set_name("view")(ap)
    fc = Linear(40, 5).set_name("fc")(v)
    out = SoftMax().set_name("prob")(fc)
    g = Graph(inp, out)
    g.set_name("tiny")
    return g


@pytest.mark.parametrize("v2", [True, False])
def test_persist_roundtrip(tmp_path, v2):
    torch.manual_seed(0)
    g = _inception_like()
    bn = [m for m in g.modules if isinstance(m, SpatialBatchNormalization)][0]
    bn.runningMean.uniform_(-0.1, 0.1)
    bn.runningVar.uniform_(0.5, 1.5)
    g.evaluate()
    x = torch.randn(2, 3, 15, 15)
    y = g.forward(x)
    proto, model = str(tmp_path / "m.prototxt"), str(tmp_path / "m.caffemodel")
    if not v2:
        g2 = Sequential().add(SpatialConvolution(3, 4, 3, 3).set_name("c")).add(ReLU(True).set_name("r")) \
            .add(View(4 * 13 * 13).set_name("v")).add(Linear(4 * 13 * 13, 3).set_name("ip"))
        g2.evaluate()
        y2 = g2.forward(x)
        CaffePersister.persist(proto, model, g2, useV2=False, overwrite=True)
        back, _ = CaffeLoader.loadCaffe(proto, model)
        back.evaluate()
        torch.testing.assert_close(back.forward(x).reshape(y2.shape), y2, rtol=1e-5, atol=1e-5)
        return
    CaffePersister.persist(proto, model, g, useV2=True, overwrite=True)
    back, _ = CaffeLoader.loadCaffe(proto, model)
    back.evaluate()
    torch.testing.assert_close(back.forward(x), y, rtol=1e-4, atol=1e-5)
    with pytest.raises(FileExistsError):
        CaffePersister.persist(proto, model, g, useV2=True, overwrite=False)
