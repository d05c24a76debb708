"""Observability of the training loop (reference DistriOptimizer.scala:188-196,
246-278, 421-449): per-iteration phase timers, the per-rank JSON metrics stream, roctx ranges,
the P5 straggler monitor (kthLargest threshold over all-gathered step times) and the RCCL
channel cap."""
import json
import os
import socket
import sys
import time

import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _mlp():
    from bigdl.nn import Sequential, Linear, ReLU, LogSoftMax
    return Sequential().add(Linear(8, 16)).add(ReLU()).add(Linear(16, 4)).add(LogSoftMax())


def _batches(n=4, bs=16):
    from bigdl.dataset import MiniBatch
    g = torch.Generator().manual_seed(0)
    return [MiniBatch(torch.randn(bs, 8, generator=g), (torch.randint(0, 4, (bs,), generator=g) + 1).float())
            for _ in range(n)]


def test_local_optimizer_json_metrics_and_phases(tmp_path):
    from bigdl.utils import config
    from bigdl.nn import ClassNLLCriterion
    from bigdl.optim import SGD, MaxIteration
    from bigdl.optim.optimizer import LocalOptimizer
    path = str(tmp_path / "metrics")
    config.set_property("bigdl.metrics.jsonPath", path)
    try:
        bs = _batches()
        opt = LocalOptimizer(_mlp(), bs, ClassNLLCriterion(), SGD(learningrate=0.1), batch_size=16)
        opt.setEndWhen(MaxIteration(5))
        opt.optimize()
    finally:
        config.clear_property("bigdl.metrics.jsonPath")
    lines = [json.loads(l) for l in open(path + ".rank0.jsonl")]
    assert [l["iteration"] for l in lines] == [1, 2, 3, 4, 5]
    for l in lines:
        assert l["rank"] == 0 and l["world"] == 1 and l["batch"] == 16
        ph = l["phases_s"]
        assert set(ph) == {"forward", "backward", "compute weight"}
        assert all(v >= 0 for v in ph.values())
    summary = opt.metrics.summary()
    assert "forward" in summary and "compute weight" in summary


def test_tracing_off_by_default_is_a_noop():
    from bigdl.utils.tracing import StepTracer
    from bigdl.optim.metrics import Metrics
    tr = StepTracer(Metrics())
    assert not tr.enabled
    with tr.phase("forward"):
        pass
    assert tr._cur == [] and tr._cur_host == {}


def test_roctx_ranges_are_balanced():
    """roctx push/pop through ctypes (libroctx64 is in the image; no profiler attached here, the
    calls must still succeed and nest)."""
    from bigdl.utils import tracing
    with tracing.roctx_range("outer"):
        with tracing.roctx_range("inner"):
            tracing.roctx_mark("tick")
    lib = tracing._roctx()
    assert lib is not None


def test_straggler_threshold_matches_kth_largest():
    from bigdl.utils.tracing import StepTracer
    from bigdl.optim.metrics import Metrics
    from bigdl.utils import config
    config.set_property("bigdl.straggler.window", 4)
    try:
        tr = StepTracer(Metrics(), rank=0, world=3)
    finally:
        config.clear_property("bigdl.straggler.window")
    per_rank = [[1.0, 1.1, 0.9, 1.0], [1.0, 1.0, 1.0, 1.05], [2.5, 2.6, 2.4, 2.5]]  # rank 2 straggles
    out = None
    for i, t in enumerate(per_rank[0]):
        out = tr.observe_step_time(i, t, 0.25, allgather=lambda mine: per_rank)
    # k = 0.25 · window 4 · world 3 = 3 → the 3rd largest of the 12 times
    assert abs(tr.threshold - sorted(sum(per_rank, []), reverse=True)[2]) < 1e-6
    assert out == [2] and tr.slow_ranks == [2]


def _straggler_worker(rank, world, port, out_q):
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bigdl-1_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from bigdl.utils import config
    config.set_property("bigdl.straggler.window", 3)
    from bigdl.utils.engine import Engine
    Engine.init(device="cpu", dist=True, backend="gloo")
    from bigdl.nn import ClassNLLCriterion
    from bigdl.optim import SGD, MaxIteration
    from bigdl.parallel import DistriOptimizer
    bs = _batches()
    opt = DistriOptimizer(_mlp(), bs, ClassNLLCriterion(), SGD(learningrate=0.1), batch_size=16)
    opt.setEndWhen(MaxIteration(7))
    opt.setDropModuleProperty(0.2, 0.5, batchsize=3, warmup_iteration=0)
    if rank == 1:  # this rank computes slowly in every iteration
        model = opt.model
        orig = model.forward

        def slow(x):
            time.sleep(0.15)
            return orig(x)
        model.forward = slow
    opt.optimize()
    tr = opt.tracer
    phases = sorted(opt.metrics._host)
    out_q.put((rank, list(tr.slow_ranks), tr.threshold, phases))
    Engine.shutdown()


def test_straggler_monitor_flags_slow_rank_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_straggler_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict((r, (s, t, ph)) for r, s, t, ph in (q.get(timeout=300) for _ in ps))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        slow, thr, phases = res[r]
        assert slow == [1], res
        assert thr is not None and thr > 0.1
        # the distributed phases the reference reports (DistriOptimizer.scala:188-196)
        assert {"forward", "backward", "aggregate gradient", "compute weight"} <= set(phases), phases


def test_comm_channel_cap_env():
    from bigdl.utils import config
    from bigdl.utils.engine import apply_comm_env
    env = {}
    config.set_property("bigdl.comm.channels", 8)
    try:
        apply_comm_env(env)
    finally:
        config.clear_property("bigdl.comm.channels")
    assert env == {"NCCL_MIN_NCHANNELS": "8", "NCCL_MAX_NCHANNELS": "8"}
    env2 = {"NCCL_MAX_NCHANNELS": "4"}
    config.set_property("bigdl.comm.channels", 8)
    try:
        apply_comm_env(env2)
    finally:
        config.clear_property("bigdl.comm.channels")
    assert env2["NCCL_MAX_NCHANNELS"] == "4"  # a user-exported value wins


def test_device_timers_are_noop_on_host():
    from bigdl.utils import config
    config.set_property("bigdl.profile.deviceTimers", True)
    try:
        m = _mlp()
        x = torch.randn(4, 8)
        m.forward(x)
        m.backward(x, torch.randn(4, 4))
        assert all(f == 0.0 and b == 0.0 for _, f, b in m.getDeviceTimes())
    finally:
        config.clear_property("bigdl.profile.deviceTimers")


import pytest  # noqa: E402


@pytest.mark.gpu
def test_device_timers_hip_events():
    """HIP-event per-module timers: resolved lazily, positive for the layers that ran on the device,
    a container's time covers its children's."""
    from bigdl.utils import config
    from bigdl.utils.engine import Engine
    import bigdl.nn as nn
    Engine.init(device="cuda:0")
    config.set_property("bigdl.profile.deviceTimers", True)
    try:
        m = nn.Sequential().add(nn.SpatialConvolution(8, 16, 3, 3, 1, 1, 1, 1)).add(nn.ReLU()) \
            .add(nn.SpatialConvolution(16, 16, 3, 3, 1, 1, 1, 1)).to(device="cuda")
        x = torch.randn(16, 8, 32, 32, device="cuda")
        for _ in range(3):
            y = m.forward(x)
            m.backward(x, torch.ones_like(y))
        times = m.getDeviceTimes()
        top_f, top_b = times[0][1], times[0][2]
        convs = [(f, b) for mod, f, b in times if type(mod).__name__ == "SpatialConvolution"]
        assert len(convs) == 2 and all(f > 0 and b > 0 for f, b in convs)
        assert top_f >= 0.9 * sum(f for f, _ in convs) and top_b >= 0.9 * sum(b for _, b in convs)
        m.resetTimes()
        assert all(f == 0.0 for _, f, _ in m.getDeviceTimes())
    finally:
        config.clear_property("bigdl.profile.deviceTimers")
