"""SyncBN (P6) at world 2 over gloo with UNEVEN per-rank batches (an uneven last batch): every rank
must issue the same collectives (the row count rides in the all-reduced sums buffer — no per-shape
cached count), and the result must equal plain training BN over the concatenated batch: outputs,
input gradients, γ/β gradients (summed over ranks, as the data-parallel all-reduce does) and the
running statistics.  Reference: SpatialBatchNormalization.scala:1114-1151,1257-1329."""
import os
import socket
import sys

import torch
import torch.multiprocessing as mp

_ROOT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bigdl-1_amd")
SIZES = [3, 7]  # per-rank batch


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs():
    g = torch.Generator().manual_seed(5)
    x = torch.randn(sum(SIZES), 8, 5, 4, generator=g) * 3 + 10  # |mean| >> std: cancellation-prone
    gy = torch.randn(sum(SIZES), 8, 5, 4, generator=g)
    return x, gy


def _bn():
    from bigdl.nn import SpatialBatchNormalization
    from bigdl.utils.random import RNG
    RNG.setSeed(2)
    m = SpatialBatchNormalization(8)
    with torch.no_grad():
        m.weight.uniform_(0.5, 1.5)
        m.bias.uniform_(-0.5, 0.5)
    return m


def _worker(rank, port, q):
    sys.path.insert(0, _ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=2)
    x, gy = _inputs()
    lo = sum(SIZES[:rank])
    xs, gs = x[lo:lo + SIZES[rank]], gy[lo:lo + SIZES[rank]]
    m = _bn()
    m.setParallism(2)
    m.training()
    for _ in range(2):  # second step: the same shapes again (a cached-count design would diverge here)
        m.zeroGradParameters()
        y = m.forward(xs)
        gi = m.backward(xs, gs)
    gw, gb = m.gradWeight.clone(), m.gradBias.clone()
    dist.all_reduce(gw)
    dist.all_reduce(gb)
    # numpy arrays pickle by value: no shared-memory handles that must outlive this process
    q.put((rank, y.numpy().copy(), gi.numpy().copy(), gw.numpy(), gb.numpy(), m.runningMean.numpy().copy(),
           m.runningVar.numpy().copy(), m._sync_path, m._sync_bwd_path))
    dist.barrier()
    dist.destroy_process_group()


def test_syncbn_uneven_batches_match_global_bn():
    sys.path.insert(0, _ROOT)
    x, gy = _inputs()
    ref = _bn()
    ref.training()
    for _ in range(2):
        ref.zeroGradParameters()
        y = ref.forward(x)
        gi = ref.backward(x, gy)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(2)], key=lambda t: t[0])
    res = [(r[0],) + tuple(torch.from_numpy(a) for a in r[1:7]) + tuple(r[7:]) for r in res]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    ys = torch.cat([r[1] for r in res])
    gis = torch.cat([r[2] for r in res])
    torch.testing.assert_close(ys, y, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(gis, gi, rtol=1e-4, atol=1e-4)
    for r in res:
        torch.testing.assert_close(r[3], ref.gradWeight, rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(r[4], ref.gradBias, rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(r[5], ref.runningMean, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(r[6], ref.runningVar, rtol=1e-4, atol=1e-4)
        assert r[7] == "reference" and r[8] == "reference"
