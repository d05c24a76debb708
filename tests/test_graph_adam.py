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
    g = GraphedTrainStep(graphed, bs[0], warmup=3)
    for _ in range(3):
        eager.train_step(bs[0])
    le = [float(eager.train_step(bs[i % 3])) for i in range(8)]
    lg = [float(g.step(bs[i % 3])) for i in range(8)]
    torch.testing.assert_close(torch.tensor(lg), torch.tensor(le), rtol=1e-3, atol=1e-3)
    meth = list(graphed.optim_methods.values())[0]
    assert float(meth.state["_dev_n"]) == 3 + 8
