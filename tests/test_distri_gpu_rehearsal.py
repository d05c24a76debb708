"""The multi-rank DEVICE path of the DistriOptimizer against a serial oracle on one GPU.

RCCL refuses two ranks on the same card, so the ranks here share ``cuda:0`` and run their
collectives over gloo; everything else is the path the driver's N > 1 bench runs on RCCL: native
kernels, gradient-ready hooks, bf16-truncated wire buckets, the sharded fused update reading the
reduce-scatter output, the all-gather, and SyncBN's native sums contract.  Oracle: a LocalOptimizer
on the concatenated global batch (SyncBN makes the two runs the same mathematics; reference method
``RefDistriOptimizer``, spark/dl/src/test/scala/.../optim/DistriOptimizerSpec.scala:378,428)."""
import os
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

_ROOT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bigdl-1_amd")
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_distri_resnet import _data, _free_port, _model, _sgd, GLOBAL_BATCH  # noqa: E402


def _worker(rank, world, port, comm_dtype, dtype, steps, out_q):
    sys.path.insert(0, _ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), OMP_NUM_THREADS="2")
    from bigdl.utils import config
    config.set_property("bigdl.compute.dtype", dtype)
    config.set_property("bigdl.comm.sharded", True)
    config.set_property("bigdl.comm.dtype", comm_dtype)
    config.set_property("bigdl.comm.bucketMB", 0.05)
    from bigdl.utils.engine import Engine
    Engine.init(device="cuda:0", dist=True, backend="gloo")
    from bigdl.nn import CrossEntropyCriterion
    from bigdl.dataset import MiniBatch
    from bigdl.parallel import DistriOptimizer
    model = _model(world)
    x, y = _data()
    per = GLOBAL_BATCH // world
    xs, ys = x[rank * per:(rank + 1) * per].cuda(), y[rank * per:(rank + 1) * per].cuda()
    opt = DistriOptimizer(model, [MiniBatch(xs, ys)], CrossEntropyCriterion(), _sgd())
    opt.prepare()
    for _ in range(steps):
        opt.train_step(MiniBatch(xs, ys))
    opt._finish()
    torch.cuda.synchronize()
    from bigdl.ops import native_status
    if rank == 0:
        out_q.put((torch.cat([p.detach().reshape(-1).float().cpu() for p in model.parameters()[0]]).numpy(),
                   bool(native_status()["loaded"])))
    Engine.shutdown()


def _serial(dtype, steps):
    """The oracle in the pytest process: the Engine may already be initialised by earlier tests, so
    the compute dtype is switched explicitly and restored afterwards."""
    from bigdl.utils import config
    from bigdl.utils.engine import Engine
    Engine.init(device="cuda:0")
    old_cfg, old_dt = config.get_property("bigdl.compute.dtype"), Engine.compute_dtype()
    config.set_property("bigdl.compute.dtype", dtype)
    Engine.set_compute_dtype(dtype)
    try:
        from bigdl.nn import CrossEntropyCriterion
        from bigdl.optim.optimizer import LocalOptimizer
        from bigdl.dataset import MiniBatch
        model = _model(1)
        w0 = torch.cat([p.detach().reshape(-1).float().cpu() for p in model.parameters()[0]])
        x, y = _data()
        x, y = x.cuda(), y.cuda()
        opt = LocalOptimizer(model, [MiniBatch(x, y)], CrossEntropyCriterion(), _sgd())
        opt.prepare()
        assert opt.compute_dtype == (torch.float32 if dtype == "fp32" else torch.bfloat16)
        for _ in range(steps):
            opt.train_step(MiniBatch(x, y))
        torch.cuda.synchronize()
        return w0, torch.cat([p.detach().reshape(-1).float().cpu() for p in model.parameters()[0]])
    finally:
        config.set_property("bigdl.compute.dtype", old_cfg)
        Engine.set_compute_dtype(old_dt)


# one step: the update differs from the serial one only by summation order and the wire rounding,
# so a gradient-scaling or shard-offset error shows at full size; three momentum steps of a BN net
# amplify the rounding chaotically (tests/test_distri_resnet.py), hence the looser bounds there
_TOL = {(1, "fp32"): (0.03, 0.9995), (1, "bf16"): (0.15, 0.99), (3, "fp32"): (0.12, 0.99), (3, "bf16"): (0.3, 0.97)}


@pytest.mark.parametrize("steps", [1, 3])
@pytest.mark.parametrize("dtype,comm_dtype", [("fp32", "fp32"), ("bf16", "bf16_truncate")])
def test_two_ranks_on_device_match_serial(dtype, comm_dtype, steps):
    w0, ref = _serial(dtype, steps)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, comm_dtype, dtype, steps, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, native = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert native
    got = torch.from_numpy(got)
    rel = float((got - ref).norm() / (ref - w0).norm())
    cos = float(((got - w0) @ (ref - w0)) / ((got - w0).norm() * (ref - w0).norm()))
    print(f"dtype={dtype} comm={comm_dtype} steps={steps} rel={rel:.4f} cos={cos:.5f}")
    lim, cmin = _TOL[(steps, dtype)]
    assert rel < lim and cos > cmin, (rel, cos)
