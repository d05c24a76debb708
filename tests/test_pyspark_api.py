"""The pyspark ``bigdl.*`` surface (pyspark/bigdl/{nn/layer,nn/criterion,optim/optimizer,util/common}.py),
exercised the way ``pyspark/test/bigdl/test_simple_integration.py`` does, without Spark."""
import numpy as np
import torch

from bigdl.nn.layer import Sequential, Linear, ReLU, LogSoftMax, Model, Input, Layer, CAddTable
from bigdl.nn.criterion import ClassNLLCriterion, MSECriterion, Criterion
from bigdl.optim.optimizer import Optimizer, SGD, MaxEpoch, EveryEpoch, Top1Accuracy, TrainSummary, Adam, \
    MaxIteration, Loss
from bigdl.util.common import Sample, JTensor, init_engine, callBigDlFunc, to_sample_rdd, RNG


def test_train_predict_like_pyspark(tmp_path):
    init_engine()
    rng = np.random.RandomState(0)
    X = rng.randn(128, 4).astype(np.float32)
    y = (X[:, 0] + X[:, 1] > 0).astype(np.float32) + 1
    samples = to_sample_rdd(X, y)
    model = Sequential().add(Linear(4, 16)).add(ReLU()).add(Linear(16, 2)).add(LogSoftMax())
    opt = Optimizer(model=model, training_rdd=samples, criterion=ClassNLLCriterion(),
                    optim_method=SGD(learningrate=0.5), end_trigger=MaxEpoch(20), batch_size=32)
    opt.set_validation(batch_size=32, val_rdd=samples, trigger=EveryEpoch(), val_method=[Top1Accuracy(), Loss()])
    opt.set_train_summary(TrainSummary(str(tmp_path), "pyspark"))
    trained = opt.optimize()
    pred = trained.predict_class(samples)
    acc = float((pred == y).mean())
    assert acc > 0.9, acc
    res = trained.evaluate(samples, [Top1Accuracy()], 32)
    assert res[0][0].result()[0] > 0.9


def test_graph_model_and_weights():
    i1 = Input()
    i2 = Input()
    a = Linear(3, 2)(i1)
    b = Linear(3, 2)(i2)
    out = CAddTable()([a, b]) if False else CAddTable()(a, b)
    m = Model([i1, i2], [out])
    x1, x2 = np.random.randn(5, 3).astype(np.float32), np.random.randn(5, 3).astype(np.float32)
    y = m.forward([x1, x2])
    assert y.shape == (5, 2)
    w = m.get_weights()
    assert len(w) == 4
    m.set_weights([np.zeros_like(t) for t in w])
    assert np.allclose(m.forward([x1, x2]), 0)


def test_jtensor_sample_and_creators():
    a = np.arange(6, dtype=np.float32).reshape(2, 3)
    jt = JTensor.from_ndarray(a)
    assert np.array_equal(jt.to_ndarray(), a)
    sp = JTensor.sparse(np.array([1.0, 2.0]), np.array([[0, 1], [2, 0]]), np.array([2, 3]))
    assert sp.to_ndarray()[0, 2] == 1.0 and sp.to_ndarray()[1, 0] == 2.0
    s = Sample.from_ndarray(a, 3)
    assert s.label().tolist() == [3.0]
    lin = callBigDlFunc("float", "createLinear", 3, 2)
    assert isinstance(lin, Layer)
    crit = callBigDlFunc("float", "createMSECriterion")
    assert isinstance(crit, Criterion)
    r = RNG()
    r.set_seed(3)
    u1 = r.uniform(0, 1, [3])
    r.set_seed(3)
    assert np.allclose(u1, r.uniform(0, 1, [3]))
