"""Native SyncBN (P6, SpatialBatchNormalization.scala:1114-1151,1257-1329) on the HIP kernels over
RCCL at world size 1: the cross-rank path (local shifted sums → all-reduce of 2·C floats → finalize
from global sums → apply; backward likewise) must reproduce plain training BN, and its forward +
backward must launch no torch elementwise kernels (every pass is a bigdl kernel or the
collective).  Multi-rank correctness of the same math is the gloo world-2/4 oracle test
(tests/test_distri_resnet.py)."""
import copy
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"


def _init_world1():
    import torch.distributed as dist
    if dist.is_initialized():
        return
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))


def _block():
    from bigdl.models.resnet import Convolution, Sbn
    from bigdl.nn import Sequential, ReLU
    from bigdl.utils.random import RNG
    RNG.setSeed(3)
    m = Sequential().add(Convolution(64, 64, 3, 3, 1, 1, 1, 1)).add(Sbn(64)).add(ReLU(True))
    m.add(Convolution(64, 128, 1, 1)).add(Sbn(128))
    for mod in m.modules:  # the convs' L2 regularizers are torch adds outside the SyncBN path
        if hasattr(mod, "wRegularizer"):
            mod.wRegularizer = mod.bRegularizer = None
    with torch.no_grad():
        for mod in m.modules:
            if type(mod).__name__ == "SpatialBatchNormalization":
                mod.weight.uniform_(0.5, 1.5)
                mod.bias.uniform_(-0.2, 0.2)
    return m


def _prep(m, sync):
    from bigdl.nn.fusion import fuse
    from bigdl.utils.engine import Engine
    m.cuda()
    m.training()
    for mod in m.modules:
        if type(mod).__name__ == "SpatialBatchNormalization":
            mod.setParallism(1)
            if sync:  # the collective path even at world size 1
                mod.set_sync_group(None, True, force=True)
    fuse(m)
    m.getParameters()
    m.flat_parameters().enable_shadow(Engine.compute_dtype())
    return m


@pytest.fixture
def rehearse_multirank():
    """Run the multi-rank SyncBN kernels at world size 1 (by default a one-rank group runs the
    local BN kernels, bigdl.bn.syncOneRankLocal)."""
    from bigdl.utils import config
    config.set_property("bigdl.bn.syncOneRankLocal", False)
    yield
    config.set_property("bigdl.bn.syncOneRankLocal", True)


def test_syncbn_one_rank_group_runs_local_kernels():
    from bigdl.utils import config
    from bigdl.utils.engine import Engine
    config.set_property("bigdl.compute.dtype", "bf16")
    Engine.init(device="cuda:0")
    _init_world1()
    b = _prep(_block(), True)
    bns = [mod for mod in b.modules if type(mod).__name__ == "SpatialBatchNormalization"]
    assert bns and not any(mod._sync_active() for mod in bns)


def test_syncbn_world1_matches_local_bn_and_runs_native(rehearse_multirank):
    from bigdl.utils import config
    from bigdl.utils.engine import Engine
    config.set_property("bigdl.compute.dtype", "bf16")
    Engine.init(device="cuda:0")
    _init_world1()
    a = _block()
    b = copy.deepcopy(a)
    a, b = _prep(a, False), _prep(b, True)
    assert all(mod._sync_active() for mod in b.modules if type(mod).__name__ == "SpatialBatchNormalization")
    assert not any(mod._sync_active() for mod in a.modules if type(mod).__name__ == "SpatialBatchNormalization")
    g = torch.Generator().manual_seed(0)
    x = torch.randn(16, 64, 28, 28, generator=g).to(dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    gy = torch.randn(16, 128, 28, 28, generator=g).to(dev).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    outs = []
    for m in (a, b):
        m.zeroGradParameters()
        y = m.forward(x)
        gi = m.backward(x, gy)
        torch.cuda.synchronize()
        outs.append((y.float(), gi.float(), [p.clone() for p in m.parameters()[1]],
                     [e.clone() for e in m.getExtraParameter()]))
    (ya, ga, pa, ea), (yb, gb, pb, eb) = outs
    torch.testing.assert_close(yb, ya, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(gb, ga, rtol=5e-2, atol=5e-2)
    assert float((gb - ga).norm() / ga.norm()) < 3e-2
    # a conv bias feeding a training BN has an exactly-zero true gradient (BN is shift-invariant):
    # both paths return rounding noise there, so those entries are compared in absolute terms
    names = [f"{type(m).__name__}.{n}" for (m, n, _g) in a._param_entries()]
    errs = []
    for nm, u, v in zip(names, pb, pa):
        if nm.endswith(".bias") and "Convolution" in nm:
            errs.append((nm, float((u - v).abs().max()), 1e-2))
        else:
            errs.append((nm, float((u - v).norm() / v.norm().clamp_min(1e-12)), 2e-2))
    assert all(e < tol for _, e, tol in errs), errs
    for u, v in zip(eb, ea):  # running statistics
        torch.testing.assert_close(u, v, rtol=1e-3, atol=1e-4)
    # no torch elementwise kernels in the SyncBN forward/backward
    import traceback
    sites = []  # where a torch add ran (named in the failure message)
    orig = {n: getattr(torch.Tensor, n) for n in ("add_", "add", "__add__", "__iadd__")}

    def _spy(n):
        def f(self, *a, **k):
            if self.is_cuda:
                sites.append(n + " @ " + " <- ".join(
                    f"{fs.name}:{fs.lineno}" for fs in traceback.extract_stack(limit=6)[:-1]))
            return orig[n](self, *a, **k)
        return f
    for n in orig:
        setattr(torch.Tensor, n, _spy(n))
    try:
        with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
            b.zeroGradParameters()
            y = b.forward(x)
            b.backward(x, gy)
            torch.cuda.synchronize()
    finally:
        for n, f in orig.items():
            setattr(torch.Tensor, n, f)
    names = {e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA}
    torch_kernels = sorted(n for n in names if "at::native" in n and "Fill" not in n)
    assert not torch_kernels, (torch_kernels, sites)
    ours = sorted(n.split("(")[0] for n in names if "at::native" not in n)
    assert any("k_bn_sum_rows" in n for n in names), " | ".join(ours)


def test_syncbn_resnet_defers_shortcut_bn(rehearse_multirank):
    """The multi-rank SyncBN path keeps the local path's projection-shortcut deferral: the shortcut
    BN only finalizes from the all-reduced sums and the block tail applies it (bigdl_bn_fwd_train_sums
    rcoef) — same loss / gradients as plain local BN on a fused ResNet-50 at 64²."""
    from bigdl.models.resnet import ResNet, DatasetType, model_init
    from bigdl.nn import CrossEntropyCriterion
    from bigdl.nn.fusion import fuse
    from bigdl.ops.reference import BNOut
    from bigdl.utils import config
    from bigdl.utils.engine import Engine
    from bigdl.utils.random import RNG
    config.set_property("bigdl.compute.dtype", "bf16")
    Engine.init(device="cuda:0")
    _init_world1()
    RNG.setSeed(5)
    a = model_init(ResNet(10, depth=50, dataset=DatasetType.ImageNet, image_size=64))
    with torch.no_grad():
        for mod in a.flattened_modules():
            if type(mod).__name__ == "SpatialBatchNormalization" and float(mod.weight.abs().max()) == 0.0:
                mod.weight.fill_(0.2)
    b = copy.deepcopy(a)
    for m, sync in ((a, False), (b, True)):
        m.cuda()
        m.training()
        for mod in m.flattened_modules():
            if type(mod).__name__ == "SpatialBatchNormalization" and sync:
                mod.setParallism(1)
                mod.set_sync_group(None, True, force=True)
        fuse(m)
        m.getParameters()
        m.flat_parameters().enable_shadow(Engine.compute_dtype())
    bns = [mod for mod in b.flattened_modules() if type(mod).__name__ == "SpatialBatchNormalization"]
    assert all(mod._sync_active() for mod in bns)
    g = torch.Generator().manual_seed(1)
    x = torch.randn(8, 3, 64, 64, generator=g).to(dev)
    y = (torch.randint(0, 10, (8,), generator=g) + 1).float().to(dev)
    crit = CrossEntropyCriterion()
    res = []
    for m in (a, b):
        for _ in range(2):  # the second step runs with the statistics shift ring primed
            m.zeroGradParameters()
            out = m.forward(x)
            loss = float(crit.forward(out, y))
            m.backward(x, crit.backward(out, y))
            torch.cuda.synchronize()
        deferred = sum(isinstance(getattr(mod, "output", None), BNOut) for mod in m.flattened_modules()
                       if type(mod).__name__ == "SpatialBatchNormalization")
        res.append((loss, [p.detach().float().clone() for p in m.parameters()[1]], deferred))
    (la, ga, da), (lb, gb, db) = res
    assert db == 4 and da == 4, (da, db)  # one projection shortcut per stage
    # (random-init bf16 ResNet-50 gradients are chaotic at this scale — two runs of the SAME local
    # path differ at gradient cosine ~0.6, tools/syncbn_diag.py — so the end-to-end check is the loss;
    # the deferred kernels themselves are pinned below against the fp32 reference)
    assert abs(la - lb) <= 2e-2 * abs(la), (la, lb)


@pytest.mark.parametrize("C", [256, 1024])
def test_bn_forward_from_sums_deferred_matches_reference(C):
    """bigdl_bn_fwd_train_sums finalize-only (a deferred shortcut BN) and with a deferred residual
    (res·rcoef + shift inside the tail's pass) against ops.reference on the same global sums."""
    from bigdl.ops import native_ops as NO, reference as R
    torch.manual_seed(2)
    M = 4096
    x = (torch.randn(8, C, 16, 32, device=dev) * 1.5 + 0.3).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    xs = (torch.randn(8, C, 16, 32, device=dev) * 0.7 - 0.2).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    assert x.numel() // C == M
    gamma, beta = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
    shift = torch.randn(C, device=dev) * 0.05

    def sums_of(t):
        tf = t.float().permute(0, 2, 3, 1).reshape(-1, C) - shift
        return torch.cat([tf.sum(0), (tf * tf).sum(0), torch.tensor([float(tf.shape[0])], device=dev)])
    # the shortcut BN: finalize only
    coef_n = torch.empty(2 * C, device=dev)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    r = NO.bn_forward_from_sums(xs, sums_of(xs), 0, shift, gamma, beta, rm, rv, 0.1, 1e-3, coef_out=coef_n, apply=False)
    assert r is not NotImplemented and r[0] is None
    coef_r = torch.empty(2 * C, device=dev)
    rm2, rv2 = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    R.bn_forward_from_sums(xs, sums_of(xs), 0, shift, gamma, beta, rm2, rv2, 0.1, 1e-3, coef_out=coef_r, apply=False)
    torch.testing.assert_close(coef_n, coef_r, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(rm, rm2, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(rv, rv2, rtol=1e-5, atol=1e-6)
    # the tail BN: ReLU(BN(x) + BN_s(xs)) with the shortcut applied inside its pass
    res = R.BNOut(xs, coef_n)
    g2, b2 = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
    y, _m, _s = NO.bn_forward_from_sums(x, sums_of(x), 0, shift, g2, b2, torch.zeros(C, device=dev),
                                       torch.ones(C, device=dev), 0.1, 1e-3, relu=True, residual=res)
    yr, _m2, _s2 = R.bn_forward_from_sums(x, sums_of(x), 0, shift, g2, b2, torch.zeros(C, device=dev),
                                          torch.ones(C, device=dev), 0.1, 1e-3, relu=True,
                                          residual=(xs.float() * coef_n[:C].view(1, C, 1, 1)
                                                    + coef_n[C:].view(1, C, 1, 1)))
    torch.testing.assert_close(y.float(), yr.float(), rtol=1.6e-2, atol=2e-2)
