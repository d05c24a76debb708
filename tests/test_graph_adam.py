"""Adam inside a captured HIP-graph training step: the iteration count lives on the device
(``bigdl_adam_dev``), so replays follow the eager trajectory (bias corrections and the decayed
learning rate advance every replay instead of being baked in at capture)."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu

dev = "cuda"


def test_adam_device_counter_matches_host_scalars():
    from bigdl.ops import native_ops, reference
    torch.manual_seed(0)
    n = 1003
    w = torch.randn(n, device=dev)
    m, v = torch.zeros(n, device=dev), torch.zeros(n, device=dev)
    w2, m2, v2 = w.clone(), m.clone(), v.clone()
    nt = torch.zeros(1, device=dev)
    for it in range(5):
        g = torch.randn(n, device=dev)
        lr = 0.01 / (1 + it * 0.1)
        reference.adam_step(w, g, m, v, lr, 0.9, 0.999, 1e-8, it + 1)
        assert native_ops.adam_step_dev(w2, g, m2, v2, nt, 0.01, 0.1, 0.9, 0.999, 1e-8) is not NotImplemented
        nt.add_(1)
    torch.testing.assert_close(w2, w, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(v2, v, rtol=1e-5, atol=1e-7)


def test_hip_graph_train_step_adam_matches_eager():
    from bigdl.nn import Sequential, Linear, ReLU, LogSoftMax, ClassNLLCriterion
    from bigdl.optim import Adam
    from bigdl.optim.optimizer import LocalOptimizer
    from bigdl.optim.graph_step import GraphedTrainStep
    from bigdl.dataset import MiniBatch
    torch.manual_seed(0)
    m = Sequential().add(Linear(32, 64)).add(ReLU()).add(Linear(64, 10)).add(LogSoftMax()).cuda()
    m2 = copy.deepcopy(m)
    bs = [MiniBatch(torch.randn(16, 32, device=dev), (torch.randint(0, 10, (16,), device=dev) + 1).float())
          for _ in range(3)]
    mk = lambda mm: LocalOptimizer(mm, [bs[0]], ClassNLLCriterion(),  # noqa: E731
                                   Adam(learningrate=0.01, learningrate_decay=0.05), batch_size=16)
    eager, graphed = mk(m), mk(m2)
    eager.prepare()
    graphed.prepare()
    g = GraphedTrainStep(graphed, bs[0], warmup=3)  # the warmup updates are undone after capture
    le = [float(eager.train_step(bs[i % 3])) for i in range(8)]
    lg = [float(g.step(bs[i % 3])) for i in range(8)]
    torch.testing.assert_close(torch.tensor(lg), torch.tensor(le), rtol=1e-3, atol=1e-3)
    meth = list(graphed.optim_methods.values())[0]
    assert float(meth.state["_dev_n"]) == 8
    assert meth.state["evalCounter"] == 8  # host and device counters agree (no capture-pass drift)
    for a, b in zip(m.parameters()[0], m2.parameters()[0]):
        # host-side vs in-kernel bias correction: last-ulp differences amplified by Adam's 1/sqrt(v)
        torch.testing.assert_close(a, b, rtol=1e-3, atol=1e-4)


def _mlp_opt(meth, bs):
    from bigdl.nn import Sequential, Linear, ReLU, LogSoftMax, ClassNLLCriterion
    from bigdl.optim.optimizer import LocalOptimizer
    from bigdl.utils.random import RNG
    torch.manual_seed(0)
    RNG.setSeed(0)  # layer init draws from bigdl's RNG: both models start identical
    m = Sequential().add(Linear(32, 64)).add(ReLU()).add(Linear(64, 10)).add(LogSoftMax()).cuda()
    opt = LocalOptimizer(m, [bs[0]], ClassNLLCriterion(), meth, batch_size=16)
    opt.prepare()
    return m, opt


def _batches(n=3):
    from bigdl.dataset import MiniBatch
    g = torch.Generator().manual_seed(1)
    return [MiniBatch(torch.randn(16, 32, generator=g).to(dev),
                      (torch.randint(0, 10, (16,), generator=g) + 1).float().to(dev)) for _ in range(n)]


def test_hip_graph_sgd_momentum_dampening_first_step_matches_eager():
    """SGD with momentum and the default dampening (= momentum): the first update is v = g, later
    ones v = μv + (1-d)g.  The capture warmup created the momentum buffer; the restore raises the
    device first-iteration flag, so the FIRST replay applies v = g and clears it."""
    from bigdl.optim import SGD
    from bigdl.optim.graph_step import GraphedTrainStep
    bs = _batches()
    m1, eager = _mlp_opt(SGD(learningrate=0.1, momentum=0.9), bs)
    m2, graphed = _mlp_opt(SGD(learningrate=0.1, momentum=0.9), bs)
    g = GraphedTrainStep(graphed, bs[0])
    le = [float(eager.train_step(bs[i % 3])) for i in range(6)]
    lg = [float(g.step(bs[i % 3])) for i in range(6)]
    torch.testing.assert_close(torch.tensor(lg), torch.tensor(le), rtol=1e-4, atol=1e-4)
    for a, b in zip(m1.parameters()[0], m2.parameters()[0]):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)


def test_hip_graph_restore_checkpoint_follows_eager(tmp_path):
    """Capture a graphed Adam step, train, checkpoint, train on, then restore the checkpoint: the
    restored moments / counter are copied into the captured state tensors in place, so the graphed
    run continues exactly like an eager run restored from the same checkpoint."""
    from bigdl.optim import Adam
    from bigdl.optim.graph_step import graphed_train_step
    from bigdl.utils import config
    bs = _batches()
    config.set_property("bigdl.graph.capture", True)
    try:
        m1, eager = _mlp_opt(Adam(learningrate=0.01, learningrate_decay=0.05), bs)
        m2, graphed = _mlp_opt(Adam(learningrate=0.01, learningrate_decay=0.05), bs)
        for o in (eager, graphed):
            o.setCheckpoint(str(tmp_path / ("g" if o is graphed else "e")), None, is_overwrite=True)
        for i in range(4):
            eager.train_step(bs[i % 3])
            graphed_train_step(graphed, bs[i % 3])
        assert getattr(graphed, "_graphed", None) is not None
        eager.checkpoint()
        graphed.checkpoint()
        for i in range(3):  # diverge from the checkpoint, then come back
            eager.train_step(bs[i % 3])
            graphed_train_step(graphed, bs[i % 3])
        eager._restore_latest()
        graphed._restore_latest()
        le = [float(eager.train_step(bs[i % 3])) for i in range(5)]
        lg = [float(graphed_train_step(graphed, bs[i % 3])) for i in range(5)]
    finally:
        config.set_property("bigdl.graph.capture", False)
    torch.testing.assert_close(torch.tensor(lg), torch.tensor(le), rtol=1e-3, atol=1e-3)
    mg = list(graphed.optim_methods.values())[0]
    assert float(mg.state["_dev_n"]) == mg.state["evalCounter"] == 9
