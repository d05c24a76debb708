"""DistriOptimizer over gloo (CPU, world 2): must produce the same weights as a serial optimizer
on the concatenated global batch (the reference's RefDistriOptimizer check,
TS/optim/DistriOptimizerSpec.scala:378,428)."""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model():
    from bigdl.nn import Sequential, Linear, ReLU, LogSoftMax, BatchNormalization
    from bigdl.utils.random import RNG
    RNG.setSeed(7)
    torch.manual_seed(7)
    return Sequential().add(Linear(8, 16)).add(ReLU()).add(Linear(16, 16)).add(ReLU()).add(Linear(16, 4)).add(
        LogSoftMax())


def _data(n=64):
    g = torch.Generator().manual_seed(3)
    x = torch.randn(n, 8, generator=g)
    y = (torch.randint(0, 4, (n,), generator=g) + 1).float()
    return x, y


def _worker(rank, world, port, mode, comm_dtype, out_q, alias=True):
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bigdl-1_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from bigdl.utils import config
    config.set_property("bigdl.comm.sharded", mode in ("sharded", "parallel"))
    config.set_property("bigdl.comm.dtype", comm_dtype)
    config.set_property("bigdl.comm.bucketMB", 0.0005)  # several buckets even for a tiny model
    config.set_property("bigdl.comm.aliasWorld1", alias)
    from bigdl.utils.engine import Engine
    Engine.init(device="cpu", dist=True, backend="gloo")
    from bigdl.nn import ClassNLLCriterion
    from bigdl.optim import SGD
    from bigdl.parallel import DistriOptimizer
    from bigdl.dataset import MiniBatch
    model = _model()
    x, y = _data()
    per = x.shape[0] // world
    sgd = SGD(learningrate=0.1, momentum=0.9, dampening=0.0, weightdecay=1e-3)
    if mode == "parallel":
        from bigdl.parallel import ParallelOptimizer
        opt = ParallelOptimizer(model, [MiniBatch(x[:per], y[:per])], ClassNLLCriterion(), sgd, parameter_blocks=3)
        last = [m for m in model.modules if m.parameters() and m.parameters()[0]][-1]
        opt.setPriorities({last.get_name(): 100})
    else:
        opt = DistriOptimizer(model, [MiniBatch(x[:per], y[:per])], ClassNLLCriterion(), sgd)
    opt.prepare()
    issued = []
    if world == 1:  # count the collectives the step issues
        import torch.distributed as dist
        from bigdl.parallel import distri_optimizer as D
        for nm in ("reduce_scatter_tensor", "all_gather_into_tensor", "all_reduce"):
            real = getattr(dist, nm)
            setattr(D.dist, nm, (lambda real, nm: lambda *a, **k: (issued.append(nm), real(*a, **k))[1])(real, nm))
    for step in range(4):
        xs = x[rank * per:(rank + 1) * per]
        ys = y[rank * per:(rank + 1) * per]
        opt.train_step(MiniBatch(xs, ys))
    opt._finish()
    w = opt.flat.weight.clone()
    if rank == 0:
        ws = torch.cat([p.reshape(-1) for p in model.parameters()[0]])
        out_q.put((ws.numpy(), len(issued), bool(opt._alias)))
    Engine.shutdown()


def _reference_weights():
    from bigdl.nn import ClassNLLCriterion
    from bigdl.optim import SGD
    from bigdl.optim.optimizer import LocalOptimizer
    from bigdl.dataset import MiniBatch
    from bigdl.utils.engine import Engine
    Engine.init(device="cpu")
    model = _model()
    x, y = _data()
    opt = LocalOptimizer(model, [MiniBatch(x, y)], ClassNLLCriterion(),
                         SGD(learningrate=0.1, momentum=0.9, dampening=0.0, weightdecay=1e-3))
    opt.prepare()
    for _ in range(4):
        opt.train_step(MiniBatch(x, y))
    return torch.cat([p.reshape(-1) for p in model.parameters()[0]])


@pytest.mark.parametrize("mode,comm_dtype", [("sharded", "fp32"), ("replicated", "fp32"), ("sharded", "bf16"),
                                             ("parallel", "fp32")])
def test_distri_matches_serial(mode, comm_dtype):
    ref = _reference_weights()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, mode, comm_dtype, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = torch.from_numpy(q.get(timeout=240)[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    tol = 1e-5 if comm_dtype == "fp32" else 3e-2
    torch.testing.assert_close(got, ref, rtol=tol, atol=tol)


@pytest.mark.parametrize("mode,comm_dtype,alias", [("sharded", "fp32", True), ("sharded", "bf16", True),
                                                   ("parallel", "fp32", True), ("sharded", "fp32", False)])
def test_distri_world1_matches_serial(mode, comm_dtype, alias):
    """One rank: the sharded DistriOptimizer (hooks, buckets, shard update path) must give the serial
    optimizer's weights; with ``bigdl.comm.aliasWorld1`` the shard tensors alias the arena and no
    gradient / weight collective is issued (a bf16 wire is then never used, so the match is fp32-exact)."""
    ref = _reference_weights()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(0, 1, _free_port(), mode, comm_dtype, q, alias))
    p.start()
    w, n_coll, aliased = q.get(timeout=240)
    p.join(timeout=120)
    assert p.exitcode == 0
    assert aliased == alias
    if alias:
        assert n_coll == 0, n_coll
    else:
        assert n_coll > 0
    tol = 1e-5 if (comm_dtype == "fp32" or alias) else 3e-2
    torch.testing.assert_close(torch.from_numpy(w), ref, rtol=tol, atol=tol)


def test_bf16_truncate_golden():
    """Reference wire format: 1.111111 → 1.109375 (TS/parameters/FP16ParameterSpec.scala:50-66)."""
    from bigdl.parallel.comm import bf16_truncate
    t = bf16_truncate(torch.tensor([1.111111]))
    assert float(t.float()) == 1.109375


def test_launcher_runs_ranks(tmp_path):
    """``python -m bigdl.launch --nproc 3 script``: env:// rendezvous, every rank joins, exit 0."""
    import subprocess
    child = tmp_path / "child.py"
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bigdl-1_amd")
    child.write_text(
        "import os, sys\n"
        f"sys.path.insert(0, {root!r})\n"
        "from bigdl.utils.engine import Engine\n"
        "Engine.init(device='cpu', dist=True, backend='gloo')\n"
        "import torch, torch.distributed as dist\n"
        "t = torch.tensor([float(Engine.rank() + 1)])\n"
        "dist.all_reduce(t)\n"
        "assert float(t) == 6.0\n"
        "print('rank', Engine.rank(), 'ok', flush=True)\n"
        "Engine.shutdown()\n")
    env = dict(os.environ, PYTHONPATH=root)
    r = subprocess.run([sys.executable, "-m", "bigdl.launch", "--nproc", "3", "--no-numa-bind", str(child)],
                       capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert sorted(l for l in r.stdout.splitlines() if l.startswith("rank")) == ["rank 0 ok", "rank 1 ok", "rank 2 ok"]


def test_launcher_restarts_all_ranks(tmp_path):
    """``--max-restarts``: a rank that fails on the first attempt makes the launcher stop the others
    and relaunch every rank; the second attempt (BIGDL_RESTART_COUNT=1) succeeds."""
    import subprocess
    child = tmp_path / "child.py"
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bigdl-1_amd")
    child.write_text(
        "import os, sys, time\n"
        "if os.environ['BIGDL_RESTART_COUNT'] == '0' and os.environ['RANK'] == '1':\n"
        "    sys.exit(3)\n"
        "if os.environ['BIGDL_RESTART_COUNT'] == '0':\n"
        "    time.sleep(30)\n"
        "print('attempt', os.environ['BIGDL_RESTART_COUNT'], 'rank', os.environ['RANK'], flush=True)\n")
    env = dict(os.environ, PYTHONPATH=root)
    r = subprocess.run([sys.executable, "-m", "bigdl.launch", "--nproc", "2", "--no-numa-bind", "--max-restarts", "1",
                        str(child)], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert sorted(r.stdout.split("\n"))[-2:] == ["attempt 1 rank 0", "attempt 1 rank 1"]
