"""Config 4 readiness (BASELINE config 4: PTB 2-layer LSTM LM under the DistriOptimizer): the
LookupTable → Recurrent(LSTM) ×2 → TimeDistributed(Linear) model with TimeDistributedCriterion and
Adagrad, run SHARDED (each rank updates only its shard with Adagrad, the reference's per-partition
``optimMethod.optimize`` over ``[paramLocalStart, +paramLocalLen)``, DL/optim/DistriOptimizer.scala:378-386;
PTBWordLM.scala:88-92 trains with Adagrad) over gloo at world 2 must match a serial LocalOptimizer on the
concatenated global batch.  Every elementwise OptimMethod is checked the same way on a small MLP."""
import os
import sys

import pytest
import torch
import torch.multiprocessing as mp

from test_distri_cpu import _free_port

V, H, T, B = 40, 16, 5, 8


def _ptb():
    from bigdl.models.rnn import PTBModel
    from bigdl.utils.random import RNG
    RNG.setSeed(11)
    torch.manual_seed(11)
    return PTBModel.lstm(V, H, V, 2)


def _ptb_data():
    g = torch.Generator().manual_seed(5)
    x = (torch.randint(0, V, (B, T), generator=g) + 1).float()
    y = (torch.randint(0, V, (B, T), generator=g) + 1).float()
    return x, y


def _mlp():
    from bigdl.nn import Sequential, Linear, Tanh, LogSoftMax
    from bigdl.utils.random import RNG
    RNG.setSeed(7)
    torch.manual_seed(7)
    return Sequential().add(Linear(8, 16)).add(Tanh()).add(Linear(16, 4)).add(LogSoftMax())


def _mlp_data():
    g = torch.Generator().manual_seed(3)
    return torch.randn(B, 8, generator=g), (torch.randint(0, 4, (B,), generator=g) + 1).float()


def _method(name):
    from bigdl import optim as O
    return {"adagrad": lambda: O.Adagrad(learningrate=0.05, learningrate_decay=0.001),
            "adagrad_wd": lambda: O.Adagrad(learningrate=0.05, learningrate_decay=0.001, weightdecay=1e-3),
            "rmsprop": lambda: O.RMSprop(learningrate=0.01, learningrate_decay=0.001),
            "adadelta": lambda: O.Adadelta(decayrate=0.9, epsilon=1e-6),
            "adamax": lambda: O.Adamax(learningrate=0.01),
            "ftrl": lambda: O.Ftrl(learningrate=0.05, l1_regularization_strength=1e-4,
                                   l2_regularization_strength=1e-3, l2_shrinkage_regularization_strength=1e-4),
            "adam": lambda: O.Adam(learningrate=0.01)}[name]()


def _setup(kind):
    from bigdl.nn import CrossEntropyCriterion, TimeDistributedCriterion, ClassNLLCriterion
    if kind == "ptb":
        return _ptb(), _ptb_data(), TimeDistributedCriterion(CrossEntropyCriterion(), size_average=True)
    return _mlp(), _mlp_data(), ClassNLLCriterion()


def _weights(model):
    return torch.cat([p.reshape(-1) for p in model.parameters()[0]]).detach().clone()


def _worker(rank, world, port, kind, meth, comm_dtype, steps, out_q):
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bigdl-1_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from bigdl.utils import config
    config.set_property("bigdl.comm.sharded", True)
    config.set_property("bigdl.comm.dtype", comm_dtype)
    config.set_property("bigdl.comm.bucketMB", 0.002)  # several buckets: shard boundaries split layers
    from bigdl.utils.engine import Engine
    Engine.init(device="cpu", dist=True, backend="gloo")
    from bigdl.parallel import DistriOptimizer
    from bigdl.dataset import MiniBatch
    model, (x, y), crit = _setup(kind)
    per = x.shape[0] // world
    xs, ys = x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per]
    opt = DistriOptimizer(model, [MiniBatch(xs, ys)], crit, _method(meth))
    opt.prepare()
    for _ in range(steps):
        opt.train_step(MiniBatch(xs, ys))
    opt._finish()
    if rank == 0:
        out_q.put((bool(opt.sharded), _weights(model).numpy()))
    Engine.shutdown()


def _serial(kind, meth, steps):
    from bigdl.optim.optimizer import LocalOptimizer
    from bigdl.dataset import MiniBatch
    from bigdl.utils.engine import Engine
    Engine.init(device="cpu")
    model, (x, y), crit = _setup(kind)
    w0 = _weights(model)
    opt = LocalOptimizer(model, [MiniBatch(x, y)], crit, _method(meth))
    opt.prepare()
    for _ in range(steps):
        opt.train_step(MiniBatch(x, y))
    return w0, _weights(model)


def _run(kind, meth, comm_dtype, steps=3):
    w0, ref = _serial(kind, meth, steps)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, kind, meth, comm_dtype, steps, q)) for r in range(2)]
    for p in procs:
        p.start()
    sharded, got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert sharded, "the DistriOptimizer fell back to replicated mode"
    assert not torch.equal(ref, w0)  # the steps moved the weights
    return torch.from_numpy(got), ref, w0


@pytest.mark.parametrize("comm_dtype", ["fp32", "bf16"])
def test_ptb_lstm_adagrad_sharded_matches_serial(comm_dtype):
    got, ref, w0 = _run("ptb", "adagrad", comm_dtype)
    if comm_dtype == "fp32":
        torch.testing.assert_close(got, ref, rtol=2e-4, atol=2e-5)
    else:  # bf16 gradient wire: the update direction agrees, magnitudes within the wire's rounding
        d_got, d_ref = got - w0, ref - w0
        cos = float(torch.nn.functional.cosine_similarity(d_got, d_ref, dim=0))
        assert cos > 0.99, cos


@pytest.mark.parametrize("meth", ["adagrad_wd", "rmsprop", "adadelta", "adamax", "ftrl", "adam"])
def test_elementwise_methods_sharded_match_serial(meth):
    got, ref, _ = _run("mlp", meth, "fp32")
    torch.testing.assert_close(got, ref, rtol=2e-4, atol=2e-5)


def test_lbfgs_and_lars_stay_replicated():
    from bigdl.optim import LBFGS, LarsSGD, Adagrad, RMSprop, Adadelta, Adamax, Ftrl
    assert not LBFGS.supports_slices and not LarsSGD.supports_slices
    assert all(m.supports_slices for m in (Adagrad, RMSprop, Adadelta, Adamax, Ftrl))
