"""CPU tests of the core: module contract, flat parameters, criteria, SGD semantics, LeNet training."""
import math

import numpy as np
import pytest
import torch

from bigdl.nn import (Sequential, Linear, ReLU, Tanh, SpatialConvolution, SpatialMaxPooling, Reshape, LogSoftMax,
                      ClassNLLCriterion, CrossEntropyCriterion, MSECriterion, ConcatTable, CAddTable, Identity)
from bigdl.utils.table import T, Table


def test_table_semantics():
    t = T(1, 2, 3)
    assert t.length() == 3 and t[1] == 1
    t.insert(2, 9)
    assert t.to_list() == [1, 9, 2, 3]
    assert t.remove(1) == 1 and t.to_list() == [9, 2, 3]


def test_linear_matches_formula_and_accumulates():
    m = Linear(3, 2)
    x = torch.randn(4, 3)
    y = m.forward(x)
    torch.testing.assert_close(y, x @ m.weight.t() + m.bias)
    gy = torch.randn(4, 2)
    m.zeroGradParameters()
    gi = m.backward(x, gy)
    torch.testing.assert_close(gi, gy @ m.weight)
    torch.testing.assert_close(m.gradWeight, gy.t() @ x)
    m.backward(x, gy)  # accumulates
    torch.testing.assert_close(m.gradWeight, 2 * gy.t() @ x)


def test_get_parameters_flattens_and_views():
    m = Sequential().add(Linear(3, 4)).add(ReLU()).add(Linear(4, 2))
    w, g = m.getParameters()
    assert w.numel() == 3 * 4 + 4 + 4 * 2 + 2
    w.fill_(0.5)
    assert float(m.modules[0].weight[0, 0]) == 0.5
    w2, g2 = m.getParameters()
    assert w2.data_ptr() == w.data_ptr()


def test_conv_weight_layout_logical_shape():
    c = SpatialConvolution(4, 8, 3, 3, n_group=2)
    assert tuple(c.weight.shape) == (2, 4, 2, 3, 3)
    x = torch.randn(2, 4, 5, 5)
    y = c.forward(x)
    w4 = c.weight.reshape(8, 2, 3, 3)
    ref = torch.nn.functional.conv2d(x, w4, c.bias, groups=2)
    torch.testing.assert_close(y, ref)


def test_conv_backward_vs_autograd():
    c = SpatialConvolution(3, 5, 3, 3, 2, 2, 1, 1)
    x = torch.randn(2, 3, 9, 9, requires_grad=True)
    y = c.forward(x.detach())
    gy = torch.randn_like(y)
    c.zeroGradParameters()
    gi = c.backward(x.detach(), gy)
    w = c.weight.reshape(5, 3, 3, 3).detach().clone().requires_grad_(True)
    b = c.bias.detach().clone().requires_grad_(True)
    yr = torch.nn.functional.conv2d(x, w, b, 2, 1)
    yr.backward(gy)
    torch.testing.assert_close(gi, x.grad, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(c.gradWeight.reshape(5, 3, 3, 3), w.grad, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(c.gradBias, b.grad, rtol=1e-4, atol=1e-5)


def test_same_padding():
    c = SpatialConvolution(1, 1, 3, 3, 2, 2, -1, -1)
    y = c.forward(torch.randn(1, 1, 8, 8))
    assert tuple(y.shape) == (1, 1, 4, 4)


def test_class_nll_one_based_and_padding():
    logp = torch.log_softmax(torch.randn(4, 5), -1)
    t = torch.tensor([1.0, 5.0, 3.0, 2.0])
    c = ClassNLLCriterion()
    l = c.forward(logp, t)
    ref = -(logp[0, 0] + logp[1, 4] + logp[2, 2] + logp[3, 1]) / 4
    assert abs(float(l) - float(ref)) < 1e-6
    c2 = ClassNLLCriterion(padding_value=2)
    l2 = c2.forward(logp, t)
    ref2 = -(logp[0, 0] + logp[1, 4] + logp[2, 2]) / 3
    assert abs(float(l2) - float(ref2)) < 1e-6


def test_cross_entropy_equals_logsoftmax_nll():
    torch.manual_seed(0)  # unseeded draws made the absolute tolerance flaky on large losses
    x = torch.randn(6, 10)
    t = torch.randint(1, 11, (6,)).float()
    ce = CrossEntropyCriterion()
    l = ce.forward(x, t)
    g = ce.backward(x, t)
    xr = x.clone().requires_grad_(True)
    lr = torch.nn.functional.cross_entropy(xr, t.long() - 1)
    lr.backward()
    assert abs(float(l) - float(lr)) <= 1e-5 * max(1.0, abs(float(lr)))
    torch.testing.assert_close(g, xr.grad, rtol=1e-4, atol=1e-6)


def test_resnet_block_backward_matches_autograd():
    m = Sequential().add(ConcatTable().add(Sequential().add(Linear(4, 4)).add(Tanh())).add(Identity())).add(
        CAddTable(True)).add(ReLU(True))
    x = torch.randn(3, 4)
    y = m.forward(x.clone())
    gy = torch.randn_like(y)
    gi = m.backward(x, gy)
    lin = m.modules[0].modules[0].modules[0]
    xr = x.clone().requires_grad_(True)
    yr = torch.relu(torch.tanh(xr @ lin.weight.t() + lin.bias) + xr)
    yr.backward(gy)
    torch.testing.assert_close(gi, xr.grad, rtol=1e-5, atol=1e-6)


def test_sgd_reference_semantics():
    """SGD.scala:61-124: dampening defaults to momentum; first step stores the gradient."""
    from bigdl.optim import SGD
    x = torch.tensor([1.0, 2.0, 3.0, 4.0])
    g = torch.tensor([0.1, 0.2, 0.3, 0.4])
    sgd = SGD(learningrate=0.5, momentum=0.9)
    sgd.optimize(lambda w: (0.0, g.clone()), x)
    torch.testing.assert_close(x, torch.tensor([1.0, 2.0, 3.0, 4.0]) - 0.5 * g)
    sgd.optimize(lambda w: (0.0, g.clone()), x)
    v = 0.9 * g + (1 - 0.9) * g
    torch.testing.assert_close(x, torch.tensor([1.0, 2.0, 3.0, 4.0]) - 0.5 * g - 0.5 * v)


def test_lr_schedules():
    from bigdl.optim import SGD, Step, Poly, Warmup, MultiStep
    s = SGD(learningrate=1.0, leaningrate_schedule=Step(2, 0.5))
    rates = []
    for _ in range(5):
        s.updateHyperParameter()
        rates.append(-s.getLearningRate())
    assert rates == [1.0, 1.0, 0.5, 0.5, 0.25]
    p = SGD(learningrate=1.0, leaningrate_schedule=Poly(2, 4))
    p.updateHyperParameter()
    p.updateHyperParameter()
    assert abs(-p.getLearningRate() - (1 - 1 / 4) ** 2) < 1e-9
    m = SGD(learningrate=1.0, leaningrate_schedule=MultiStep([1, 3], 0.1))
    r = []
    for _ in range(4):
        m.updateHyperParameter()
        r.append(round(-m.getLearningRate(), 6))
    assert r == [1.0, 0.1, 0.1, 0.01]


def _mnist_like(n=256, seed=0):
    g = torch.Generator().manual_seed(seed)
    labels = torch.randint(0, 10, (n,), generator=g)
    protos = torch.randn(10, 28, 28, generator=torch.Generator().manual_seed(99))
    x = protos[labels] + 0.3 * torch.randn(n, 28, 28, generator=g)
    return x, (labels + 1).float()


def test_lenet_local_optimizer_converges():
    """Config 1: LeNet-5 + LocalOptimizer on CPU learns a separable MNIST-shaped task."""
    from bigdl.models.lenet import LeNet5
    from bigdl.dataset import Sample
    from bigdl.optim import SGD, Optimizer, MaxEpoch, Top1Accuracy, EveryEpoch
    from bigdl.utils.engine import Engine
    Engine.init(device="cpu")
    x, y = _mnist_like(512)
    samples = [Sample(x[i], y[i]) for i in range(len(x))]
    model = LeNet5(10)
    opt = Optimizer.create(model, samples, ClassNLLCriterion(), MaxEpoch(3), 32,
                           SGD(learningrate=0.05, momentum=0.9, dampening=0.0), distributed=False)
    opt.setValidation(EveryEpoch(), samples[:128], [Top1Accuracy()], 64)
    trained = opt.optimize()
    trained.evaluate()
    out = trained.forward(x[:128])
    acc = float(((out.argmax(1) + 1).float() == y[:128]).float().mean())
    assert acc > 0.9, acc
    assert opt.state["score"] > 0.9


def test_pyspark_style_numpy_io():
    m = Sequential().add(Linear(3, 2))
    out = m.forward(np.ones((4, 3), dtype=np.float32))
    assert isinstance(out, np.ndarray) and out.shape == (4, 2)
    assert len(m.get_weights()) == 2


def test_dense_to_sparse_and_sparse_join_table():
    import torch
    from bigdl.nn import DenseToSparse, SparseJoinTable, SparseLinear
    from bigdl.utils.table import Table
    a = torch.tensor([[0.0, 2.0, 0.0], [1.0, 0.0, 0.0]])
    b = torch.tensor([[0.0, 0.0], [0.0, 3.0]])
    d2s = DenseToSparse()
    sa = d2s.forward(a)
    assert sa.is_sparse and torch.equal(sa.to_dense(), a)
    assert torch.equal(d2s.backward(a, torch.ones(2, 3)), torch.ones(2, 3))
    j = SparseJoinTable(2)
    out = j.forward(Table(sa, DenseToSparse().forward(b)))
    assert torch.equal(out.to_dense(), torch.cat([a, b], 1))
    gi = j.backward(Table(sa, b), torch.arange(10.0).view(2, 5))
    assert torch.equal(gi[2], torch.tensor([[3.0, 4.0], [8.0, 9.0]]))
    lin = SparseLinear(5, 4)
    dense = lin.forward(torch.cat([a, b], 1)).clone()
    assert torch.allclose(lin.forward(out), dense, atol=1e-6)
