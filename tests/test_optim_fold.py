"""Folding pure-L2 layer regularizers into the fused SGD update must not change the trajectory
(Regularizer.scala semantics: g += λ·scale·w inside accGradParameters)."""
import numpy as np
import torch

from bigdl import nn
from bigdl.dataset import Sample
from bigdl.optim import SGD
from bigdl.optim.optimizer import LocalOptimizer
from bigdl.optim.regularizer import L2Regularizer, L1L2Regularizer
from bigdl.optim.trigger import MaxIteration
from bigdl.utils import config
from bigdl.utils.random import RNG


def _run(fold: bool, wd=1e-3, user_wds=False):
    config.set_property("bigdl.optim.foldRegularizers", fold)
    try:
        RNG.setSeed(5)
        torch.manual_seed(5)
        m = nn.Sequential()
        m.add(nn.Linear(6, 8, wRegularizer=L2Regularizer(0.05), bRegularizer=L2Regularizer(0.01)))
        m.add(nn.Tanh())
        m.add(nn.Linear(8, 3, wRegularizer=L1L2Regularizer(0.01, 0.02)))  # L1 part: never folded
        m.add(nn.LogSoftMax())
        rng = np.random.RandomState(1)
        data = [Sample(rng.randn(6).astype(np.float32), np.array([1 + i % 3], np.float32)) for i in range(32)]
        n_params = sum(p.numel() for p in m.parameters()[0])
        wds = torch.linspace(0.5, 1.5, n_params) if user_wds else None
        sgd = SGD(learningrate=0.1, momentum=0.9, dampening=0.0, nesterov=True, weightdecay=wd, weightdecays=wds)
        opt = LocalOptimizer(m, data, nn.ClassNLLCriterion(), sgd, MaxIteration(6), 8)
        opt.optimize()
        return torch.cat([p.detach().reshape(-1).clone() for p in m.parameters()[0]])
    finally:
        config.clear_property("bigdl.optim.foldRegularizers")


def test_fold_matches_unfolded():
    torch.testing.assert_close(_run(True), _run(False), rtol=1e-5, atol=1e-6)


def test_fold_with_user_weight_decays():
    torch.testing.assert_close(_run(True, user_wds=True), _run(False, user_wds=True), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(_run(True, wd=0.0, user_wds=True), _run(False, wd=0.0, user_wds=True),
                               rtol=1e-5, atol=1e-6)


def test_adagrad_graph_mode_matches_eager():
    """Adagrad's replay-safe form (device-side iteration counter, tensor learning rate) computes
    the same updates as the eager form."""
    import torch
    from bigdl.optim import Adagrad
    torch.manual_seed(0)
    x1 = torch.randn(64)
    x2 = x1.clone()
    a, b = Adagrad(0.1, 0.01), Adagrad(0.1, 0.01)
    assert b.prepare_graph()
    for _ in range(5):
        g = torch.randn(64)
        a.optimize(lambda _x, g=g: (0.0, g.clone()), x1)
        b.optimize(lambda _x, g=g: (0.0, g.clone()), x2)
    torch.testing.assert_close(x1, x2, rtol=1e-6, atol=1e-7)
    assert float(b.state["_dev_n"]) == 5.0


def test_lbfgs_with_wolfe_line_search_rosenbrock():
    """LBFGS + LswolfeLineSearch (``LBFGSSpec`` style: Rosenbrock minimum at (1, 1))."""
    import torch
    from bigdl.optim import LBFGS, LswolfeLineSearch

    def rosen(x):
        a, b = x[0], x[1]
        f = (1 - a) ** 2 + 100 * (b - a * a) ** 2
        g = torch.stack([-2 * (1 - a) - 400 * a * (b - a * a), 200 * (b - a * a)])
        return f, g
    x = torch.tensor([-1.2, 1.0], dtype=torch.float64)
    opt = LBFGS(max_iter=100, tolfun=1e-12, tolx=1e-12, linesearch=LswolfeLineSearch())
    x, fs = opt.optimize(rosen, x)
    assert torch.allclose(x, torch.tensor([1.0, 1.0], dtype=torch.float64), atol=1e-4), x
    assert fs[-1] < 1e-8
