"""fp32 compute mode on the bf16 MFMA kernels (ops/fp32x3.py, csrc/precision.hip): the hi/lo split
is exact against torch's own bf16 rounding, and conv forward / data gradient / weight gradient and
Linear forward / backward match an fp64 reference to fp32-class accuracy (far below bf16 rounding),
through the ops and through the nn modules with ``bigdl.compute.dtype=fp32`` (no torch fallback)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = "cuda"


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def test_split_matches_torch_rounding():
    from bigdl.ops import fp32x3 as F3
    g = torch.Generator().manual_seed(0)
    x = (torch.randn(37, 21, generator=g) * torch.logspace(-3, 3, 21)).to(dev)
    hi = x.bfloat16()
    lo = (x - hi.float()).bfloat16()
    side = F3.split(x, 24, F3.HHL, False).cpu()
    assert torch.equal(side[:, 0:21], hi.cpu()) and torch.equal(side[:, 24:45], hi.cpu())
    assert torch.equal(side[:, 48:69], lo.cpu())
    assert side[:, 21:24].abs().sum() == 0 and side[:, 69:72].abs().sum() == 0
    st = F3.split(x, 24, F3.HLH, True).cpu()
    assert torch.equal(st[0:37, :21], hi.cpu()) and torch.equal(st[37:74, :21], lo.cpu())
    assert torch.equal(st[74:111, :21], hi.cpu())
    two = F3.split2(x, 24).cpu()  # [hi | lo], each zero-padded to 24
    assert torch.equal(two[:, 0:21], hi.cpu()) and torch.equal(two[:, 24:45], lo.cpu())
    assert two.shape == (37, 48) and two[:, 21:24].abs().sum() == 0 and two[:, 45:48].abs().sum() == 0
    rec = hi.double() + lo.double()
    assert float(((rec - x.double()).abs() / x.double().abs().clamp_min(1e-30)).max()) < 2 ** -16


@pytest.mark.parametrize("N,C,K,H,W,k,s,p,d", [
    (4, 64, 128, 14, 14, 3, 1, 1, 1),
    (2, 3, 64, 32, 32, 7, 2, 3, 1),      # RGB stem: C padded to 8, strided dgrad on the lattice
    (3, 32, 48, 9, 11, 1, 2, 0, 1),      # 1x1 stride 2
    (2, 16, 20, 10, 10, 3, 1, 2, 2),     # dilated, K % 8 != 0
    (2, 24, 8, 15, 15, 3, 2, 1, 1),
])
@pytest.mark.parametrize("two", [True, False], ids=["hi_lo", "hi_hi_lo"])
def test_conv_fp32x3_matches_fp64(N, C, K, H, W, k, s, p, d, two):
    from bigdl.ops import fp32x3 as F3
    from bigdl.utils import config
    prev = config.get_property("bigdl.fp32.twoPart")
    config.set_property("bigdl.fp32.twoPart", two)
    try:
        _conv_case(F3, N, C, K, H, W, k, s, p, d)
    finally:
        config.set_property("bigdl.fp32.twoPart", prev)


def _conv_case(F3, N, C, K, H, W, k, s, p, d):
    g = torch.Generator().manual_seed(1)
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(K, C, k, k, generator=g) * (1.0 / (C * k * k) ** 0.5)
    b = torch.randn(K, generator=g)
    xr, wr, br = (t.double().requires_grad_() for t in (x, w, b))
    yr = F.conv2d(xr, wr, br, s, p, d)
    gy = torch.randn(yr.shape, generator=g)
    yr.backward(gy.double())

    y = F3.conv_forward(x.to(dev), w.to(dev), b.to(dev), (s, s), (p, p), (d, d))
    assert y is not NotImplemented and y.dtype == torch.float32 and y.shape == yr.shape
    gw = torch.zeros(K, k, k, C, device=dev).permute(0, 3, 1, 2)  # KRSC arena layout
    gb = torch.zeros(K, device=dev)
    gi = F3.conv_backward(gy.to(dev), x.to(dev), w.to(dev), (s, s), (p, p), (d, d), 1, True, gw, gb, 1.0)
    torch.cuda.synchronize()
    assert _rel(y, yr) < 2e-5, _rel(y, yr)
    assert _rel(gi, xr.grad) < 2e-5, _rel(gi, xr.grad)
    assert _rel(gw, wr.grad) < 2e-5, _rel(gw, wr.grad)
    assert _rel(gb, br.grad) < 1e-6
    # and it is not the bf16 path: plain bf16 operands are ~100x further off
    yb = F.conv2d(x.bfloat16().double(), w.bfloat16().double(), b.double(), s, p, d)
    assert _rel(yb, yr) > 20 * _rel(y, yr)
    # shortcut gradient summed in the data-gradient epilogue (C % 4 == 0) or by the fallback add (C == 3)
    res = torch.randn(N, C, H, W, generator=g)
    gi2 = F3.conv_backward(gy.to(dev), x.to(dev), w.to(dev), (s, s), (p, p), (d, d), 1, True, gw.clone(), gb.clone(),
                           1.0, residual=res.to(dev).contiguous(memory_format=torch.channels_last))
    torch.cuda.synchronize()
    assert _rel(gi2, xr.grad + res.double()) < 2e-5, _rel(gi2, xr.grad + res.double())


@pytest.mark.parametrize("M,K,N",[(64, 256, 128), (33, 100, 10), (7, 24, 36)])
def test_linear_fp32x3_matches_fp64(M, K, N):
    from bigdl.ops import fp32x3 as F3
    g = torch.Generator().manual_seed(2)
    x, w, b = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g) * K ** -0.5, torch.randn(N, generator=g)
    xr, wr, br = (t.double().requires_grad_() for t in (x, w, b))
    yr = F.linear(xr, wr, br)
    gy = torch.randn(M, N, generator=g)
    yr.backward(gy.double())
    y = F3.linear_forward(x.to(dev), w.to(dev), b.to(dev))
    gw, gb = torch.zeros(N, K, device=dev), torch.zeros(N, device=dev)
    gi = F3.linear_backward(gy.to(dev), x.to(dev), w.to(dev), True, gw, gb, 0.5)
    torch.cuda.synchronize()
    assert _rel(y, yr) < 2e-5
    assert _rel(gi, xr.grad) < 2e-5
    assert _rel(gw, 0.5 * wr.grad) < 2e-5
    assert _rel(gb, 0.5 * br.grad) < 1e-6


def test_fp32_modules_run_native_without_fallback():
    from bigdl.utils import config
    from bigdl.utils.engine import Engine
    from bigdl import ops
    from bigdl.nn import Sequential, SpatialConvolution, ReLU, Reshape, Linear
    config.set_property("bigdl.compute.dtype", "fp32")
    try:
        Engine.init(device="cuda:0")
        torch.manual_seed(0)
        m = Sequential().add(SpatialConvolution(8, 16, 3, 3, 1, 1, 1, 1)).add(ReLU()) \
            .add(SpatialConvolution(16, 16, 3, 3, 2, 2, 1, 1)).add(Reshape([16 * 4 * 4])).add(Linear(256, 10))
        ref = [p.detach().double().clone() for p in m.parameters()[0]]
        x = torch.randn(4, 8, 8, 8)
        gy = torch.randn(4, 10)
        m.cuda()
        ops.reset_fallbacks()
        with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
            y = m.forward(x.to(dev))
            m.zeroGradParameters()
            m.backward(x.to(dev), gy.to(dev))
            torch.cuda.synchronize()
        names = {e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA}
        assert any("k_split_bf16x3" in n for n in names) and any("k_conv_fwd" in n for n in names), sorted(names)
        assert any("k_gemm" in n for n in names) and any("k_conv_wgrad" in n for n in names), sorted(names)
        assert not any("miopen" in n.lower() or "Cijk" in n for n in names), sorted(names)
        fb = {k[0] for k in ops.fallback_counts()}
        assert not ({"conv2d_forward", "conv2d_backward", "linear_forward", "linear_backward"} & fb), fb
        w1, b1, w2, b2, wl, bl = ref
        xr = x.double().requires_grad_()
        h = F.relu(F.conv2d(xr, w1.reshape(16, 8, 3, 3), b1, 1, 1))
        h = F.conv2d(h, w2.reshape(16, 16, 3, 3), b2, 2, 1)
        yr = F.linear(h.permute(0, 1, 2, 3).reshape(4, -1), wl.reshape(10, 256), bl)
        yr.backward(gy.double())
        assert _rel(y, yr) < 5e-5
        gin = m.gradInput
        assert _rel(gin, xr.grad) < 5e-5
    finally:
        config.set_property("bigdl.compute.dtype", "bf16")
        Engine.init(device="cuda:0")


@pytest.mark.parametrize("relu,res", [(False, False), (True, False), (True, True)])
def test_bn32_native_matches_reference(relu, res):
    """fp32 BatchNorm kernels (batchnorm.hip k_bn32_*) vs the torch reference ops in fp64."""
    from bigdl.ops import native_ops as NO, reference as R
    g = torch.Generator().manual_seed(3)
    N_, C_, H, W = 4, 48, 9, 7
    x = (torch.randn(N_, C_, H, W, generator=g) * 3 + 5).contiguous(memory_format=torch.channels_last)
    r = torch.randn(N_, C_, H, W, generator=g).contiguous(memory_format=torch.channels_last) if res else None
    gam, bet = torch.rand(C_, generator=g) + 0.5, torch.randn(C_, generator=g)
    rm, rv = torch.zeros(C_), torch.ones(C_)
    y, m, inv = NO.batchnorm_forward_train(x.to(dev), gam.to(dev), bet.to(dev), rm.to(dev), rv.to(dev), 0.1, 1e-3,
                                           relu, None if r is None else r.to(dev))
    rm_d, rv_d = rm.double(), rv.double()
    yr, mr, ir = R.batchnorm_forward_train(x.double(), gam.double(), bet.double(), rm_d, rv_d, 0.1, 1e-3, relu,
                                           None if r is None else r.double())
    assert _rel(y, yr) < 1e-5 and _rel(m, mr) < 1e-6 and _rel(inv, ir) < 1e-5
    gy = torch.randn(N_, C_, H, W, generator=g).contiguous(memory_format=torch.channels_last)
    gg, gb = torch.zeros(C_, device=dev), torch.zeros(C_, device=dev)
    gx, gres = NO.batchnorm_backward(gy.to(dev), x.to(dev), gam.to(dev), m, inv, y, relu, True, gg, gb, 1.0,
                                     want_gres=res)
    ggr, gbr = torch.zeros(C_, dtype=torch.float64), torch.zeros(C_, dtype=torch.float64)
    out = R.batchnorm_backward(gy.double(), x.double(), gam.double(), mr, ir, yr, relu, True, ggr, gbr, 1.0)
    torch.cuda.synchronize()
    assert _rel(gx, out[0]) < 1e-4 and _rel(gg, ggr) < 1e-5 and _rel(gb, gbr) < 1e-5
    if res:
        assert _rel(gres, gy.double() * (yr > 0)) < 1e-6
    if relu:  # the backward read the forward's mask bits; the y-reading path (no bits for a copy of y) agrees exactly
        from bigdl.ops import fp32x3 as F3
        assert F3.producer_bits(y) is not None and F3.producer_bits(y.clone()) is None
        gx2, _ = NO.batchnorm_backward(gy.to(dev), x.to(dev), gam.to(dev), m, inv, y.clone(), relu, True,
                                       torch.zeros(C_, device=dev), torch.zeros(C_, device=dev), 1.0)
        assert torch.equal(gx2, gx)
    # the apply passes also wrote the consuming conv's [hi | lo] operand (producer-side split): it is
    # exactly the split pass's output, and the conv finds it
    from bigdl.ops import fp32x3 as F3
    for t in (y, gx):
        sp = F3._producer_split(t, C_)
        assert sp is not None
        assert torch.equal(sp, F3.split2(F3._nhwc_rows(t), C_))


def test_fp32_conv_uses_producer_split():
    """A BN → conv chain in fp32 gives bit-identical results with the producer-side split on and off,
    and the conv launches one split pass fewer."""
    from bigdl.ops import native_ops as NO, fp32x3 as F3
    from bigdl.utils import config
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 64, 12, 12, generator=g).to(dev).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(32, 64, 3, 3, generator=g) * 0.05).to(dev)
    gam, bet = torch.rand(64, generator=g).to(dev) + 0.5, torch.randn(64, generator=g).to(dev)
    outs = []
    config.set_property("bigdl.fp32.direct", False)  # the split-operand kernels (direct ones need no split)
    for on in (True, False):
        config.set_property("bigdl.fp32.producerSplit", on)
        try:
            h, _, _ = NO.batchnorm_forward_train(x, gam, bet, torch.zeros(64, device=dev), torch.ones(64, device=dev),
                                                 0.1, 1e-5, True)
            hit = F3._producer_split(h, 64) is not None
            with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
                y = F3.conv_forward(h, w, None, (1, 1), (1, 1))
                torch.cuda.synchronize()
            n_split = sum(1 for e in prof.events() if "k_split_bf16x3" in e.name)
            outs.append((y.clone(), hit, n_split))
        finally:
            config.set_property("bigdl.fp32.producerSplit", True)
    config.set_property("bigdl.fp32.direct", True)
    (y1, hit1, n1), (y0, hit0, n0) = outs
    assert hit1 and not hit0 and n1 == n0 - 1, (hit1, hit0, n1, n0)
    assert torch.equal(y1, y0)


@pytest.mark.parametrize("s", [1, 2])
def test_conv_fp32x3_dgrad_in_image_chunks(s, monkeypatch):
    """A data gradient whose dY operand exceeds the kernels' 32-bit offsets (the 224² stem at batch 256)
    runs in image chunks: forced here with a small limit, checked against fp64."""
    from bigdl.ops import fp32x3 as F3
    g = torch.Generator().manual_seed(7)
    N, C, K, H, W = 5, 16, 32, 12, 12
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(K, C, 3, 3, generator=g) * (1.0 / (C * 9) ** 0.5)
    xr, wr = x.double().requires_grad_(), w.double().requires_grad_()
    yr = F.conv2d(xr, wr, None, s, 1)
    gy = torch.randn(yr.shape, generator=g)
    res = torch.randn(N, C, H, W, generator=g)
    yr.backward(gy.double())
    monkeypatch.setattr(F3, "_OPERAND_LIMIT", 2 * H * W * 2 * K * 2 + 7)  # 2 images per launch
    gw = torch.zeros(K, 3, 3, C, device=dev).permute(0, 3, 1, 2)
    gi = F3.conv_backward(gy.to(dev), x.to(dev), w.to(dev), (s, s), (1, 1), (1, 1), 1, True, gw, None, 1.0,
                          residual=res.to(dev).contiguous(memory_format=torch.channels_last))
    torch.cuda.synchronize()
    assert _rel(gi, xr.grad + res.double()) < 2e-5
    assert _rel(gw, wr.grad) < 2e-5


def test_fp32_conv_epilogue_bn_statistics():
    """fp32 conv → BN with the statistics added by the conv's fp32 epilogue into the BN's replicated
    buffer (finalize from 32 rows, cleared after reading) matches the standalone statistics pass."""
    from bigdl.ops import native_ops as NO, fp32x3 as F3
    g = torch.Generator().manual_seed(9)
    N_, C_, K, H = 3, 64, 48, 13  # M = 507 rows: a partial last row tile
    x = (torch.randn(N_, C_, H, H, generator=g) + 0.5).to(dev).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C_, 3, 3, generator=g) * 0.05).to(dev)
    gam, bet = torch.rand(K, generator=g).to(dev) + 0.5, torch.randn(K, generator=g).to(dev)
    rep = 32
    buf = torch.zeros(2 * rep * K, device=dev)
    rm1, rv1 = torch.full((K,), 0.3, device=dev), torch.ones(K, device=dev)
    rm0, rv0 = rm1.clone(), rv1.clone()
    r = NO.conv2d_forward_stats(x, w, None, (1, 1), (1, 1), shift=rm1, sums=(buf, rep))
    assert r is not NotImplemented
    y1, part, G = r
    assert part is buf and G == rep
    out1 = NO.batchnorm_forward_train_partials(y1, part, G, gam, bet, rm1, rv1, 0.1, 1e-5, relu=True, shift=rm1,
                                               rezero=True)
    assert out1 is not NotImplemented
    y0 = F3.conv_forward(x, w, None, (1, 1), (1, 1))
    out0 = NO.batchnorm_forward_train(y0, gam, bet, rm0, rv0, 0.1, 1e-5, relu=True)
    torch.cuda.synchronize()
    assert torch.equal(y1, y0)
    assert _rel(out1[0], out0[0]) < 1e-5 and _rel(out1[1], out0[1]) < 1e-5 and _rel(out1[2], out0[2]) < 1e-5
    assert _rel(rm1, rm0) < 1e-5 and _rel(rv1, rv0) < 1e-5
    assert float(buf.abs().sum()) == 0.0  # cleared by the finalize for the next step


@pytest.mark.parametrize("tail", [False, True], ids=["mid_block", "block_tail"])
def test_fp32_dgrad_epilogue_bn_backward_statistics(tail):
    """The fp32 data gradient of a conv that consumes a BN + ReLU output stores the ReLU-masked gradient
    and adds the BN-backward sums into the BN's replicas (mask recomputed from scale·x + shift, or the
    block tail's forward mask bits with the shortcut gradient summed first); the BN backward from them
    matches the standalone path."""
    from bigdl.ops import native_ops as NO, fp32x3 as F3
    g = torch.Generator().manual_seed(11)
    N_, C_, K, H = 2, 32, 24, 11
    cl = torch.channels_last
    xb = torch.randn(N_, C_, H, H, generator=g).to(dev).contiguous(memory_format=cl)
    gam, bet = (torch.rand(C_, generator=g) + 0.5).to(dev), torch.randn(C_, generator=g).to(dev)
    res = torch.randn(N_, C_, H, H, generator=g).to(dev).contiguous(memory_format=cl) if tail else None
    coef = torch.empty(2 * C_, device=dev)
    y, mean, invstd = NO.batchnorm_forward_train(xb, gam, bet, torch.zeros(C_, device=dev), torch.ones(C_, device=dev),
                                                 0.1, 1e-5, relu=True, residual=res, coef_out=coef)
    w = (torch.randn(K, C_, 3, 3, generator=g) * 0.1).to(dev)
    gy = torch.randn(N_, K, H, H, generator=g).to(dev).contiguous(memory_format=cl)
    sres = torch.randn(N_, C_, H, H, generator=g).to(dev).contiguous(memory_format=cl) if tail else None
    rep = 32
    buf = torch.zeros(2 * rep * C_, device=dev)
    fuse = {"x": xb, "mean": mean, "sums": (buf, rep)}
    if tail:
        fuse["mask"] = y
    else:
        fuse["scale"], fuse["shift"] = coef[:C_], coef[C_:]
    gi1 = F3.conv_backward(gy, y, w, (1, 1), (1, 1), (1, 1), 1, True, None, None, 1.0, residual=sres, bn_fuse=fuse)
    assert fuse.get("partial") is buf and fuse.get("G") == rep
    gg1, gb1 = torch.zeros(C_, device=dev), torch.zeros(C_, device=dev)
    gx1 = NO.batchnorm_backward_partials(gi1, xb, gam, mean, invstd, buf, rep, True, gg1, gb1, 1.0, rezero=True)
    assert gx1 is not NotImplemented
    gi0 = F3.conv_backward(gy, y, w, (1, 1), (1, 1), (1, 1), 1, True, None, None, 1.0, residual=sres)
    gg0, gb0 = torch.zeros(C_, device=dev), torch.zeros(C_, device=dev)
    gx0, _ = NO.batchnorm_backward(gi0, xb, gam, mean, invstd, y.clone(), True, True, gg0, gb0, 1.0)
    torch.cuda.synchronize()
    assert torch.equal(gi1, gi0 * (y > 0))
    assert _rel(gx1, gx0) < 1e-5 and _rel(gg1, gg0) < 1e-5 and _rel(gb1, gb0) < 1e-5
    assert float(buf.abs().sum()) == 0.0
