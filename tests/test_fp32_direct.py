"""fp32 compute mode, direct-operand kernels (csrc/conv_x3.hip, conv_wgrad.hip F32): the conv reads the
fp32 activations / gradients itself and splits each MFMA fragment into bf16 hi / lo while reading it, so
no [hi | lo] split tensor exists.  Forward, sub-pixel strided data gradient, weight gradient and the fused
BN epilogues (forward statistics, BN-backward statistics with the ReLU mask, compact strided residual) are
checked against fp64 torch references of the same ops (reference: SpatialConvolution updateOutput /
updateGradInput / accGradParameters in fp32, DL/nn/SpatialConvolution.scala:253-505)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = "cuda"
cl = torch.channels_last


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _targs(name):
    """Template arguments of a demangled kernel name ("k<a, b>(...)" → ["a", "b"])."""
    head = name.split("(")[0]
    return head.split("<", 1)[1].rstrip(">").split(", ") if "<" in head else []


def _kernels(fn):
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
        out = fn()
        torch.cuda.synchronize()
    return out, [e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA]


@pytest.mark.parametrize("N,C,K,H,W,k,s,p", [
    (4, 64, 128, 14, 14, 3, 1, 1),
    (3, 128, 64, 13, 9, 1, 1, 0),     # pointwise, partial last pixel tile
    (2, 64, 64, 15, 15, 3, 2, 1),     # strided 3x3: four parity classes in the dgrad
    (2, 64, 256, 14, 14, 1, 2, 0),    # 1x1 stride 2: one parity class, the rest zero
    (2, 96, 200, 7, 7, 3, 1, 1),      # K not a multiple of the 128-channel tile
    (1, 32, 32, 5, 6, 5, 1, 2),       # 25 taps
])
def test_direct_conv_matches_fp64(N, C, K, H, W, k, s, p):
    from bigdl.ops import fp32x3 as F3
    g = torch.Generator().manual_seed(1)
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(K, C, k, k, generator=g) * (1.0 / (C * k * k) ** 0.5)
    b = torch.randn(K, generator=g)
    xr, wr, br = (t.double().requires_grad_() for t in (x, w, b))
    yr = F.conv2d(xr, wr, br, s, p)
    gy = torch.randn(yr.shape, generator=g)
    yr.backward(gy.double())
    xd = x.to(dev).contiguous(memory_format=cl)
    gyd = gy.to(dev).contiguous(memory_format=cl)
    y, names = _kernels(lambda: F3.conv_forward(xd, w.to(dev), b.to(dev), (s, s), (p, p)))
    assert any("k_conv_x3" in n for n in names), names
    assert _rel(y, yr) < 2e-5, _rel(y, yr)
    gw = torch.zeros(K, k, k, C, device=dev).permute(0, 3, 1, 2)
    gb = torch.zeros(K, device=dev)
    gi, names = _kernels(lambda: F3.conv_backward(gyd, xd, w.to(dev), (s, s), (p, p), (1, 1), 1, True, gw, gb, 1.0))
    # the fp32-operand wgrad (8 template arguments: F32 = true), one launch
    # (template argument 8: F32; 9: the BN prologue, off here)
    assert sum("k_conv_wgrad" in n and _targs(n)[7:] == ["true", "false"] for n in names) == 1, names
    if K % 32 == 0:  # (a dgrad over K % 32 != 0 channels takes the split-operand kernels)
        assert any("k_conv_x3" in n for n in names), names
        # no activation / gradient split: the only split launches are the weight chunks
        assert sum("k_split_bf16x3" in n for n in names) <= (1 if s == 1 else 4), names
    assert _rel(gi, xr.grad) < 2e-5, _rel(gi, xr.grad)
    assert _rel(gw, wr.grad) < 2e-5, _rel(gw, wr.grad)
    assert _rel(gb, br.grad) < 1e-6
    # the shortcut gradient summed in the epilogue (dense residual)
    res = torch.randn(N, C, H, W, generator=g)
    gi2 = F3.conv_backward(gyd, xd, w.to(dev), (s, s), (p, p), (1, 1), 1, True, None, None, 1.0,
                           residual=res.to(dev).contiguous(memory_format=cl))
    torch.cuda.synchronize()
    assert _rel(gi2, xr.grad + res.double()) < 2e-5


def test_direct_split_is_round_to_nearest():
    """The in-kernel split keeps hi = rne(v), lo = rne(v − hi): a 1×1 conv with a one-hot filter of 1.0
    returns hi + lo of its input, which must equal the host-side split's reconstruction exactly."""
    from bigdl.ops import fp32x3 as F3
    g = torch.Generator().manual_seed(2)
    x = (torch.randn(1, 32, 4, 8, generator=g) * torch.logspace(-3, 3, 32).reshape(1, 32, 1, 1)).to(dev)
    x = x.contiguous(memory_format=cl)
    w = torch.eye(32).reshape(32, 32, 1, 1).to(dev)
    y = F3.conv_forward(x, w, None, (1, 1), (0, 0))
    hi = x.bfloat16().float()
    lo = (x - hi).bfloat16().float()
    torch.cuda.synchronize()
    # the 1.0 weight's lo part is 0: y = hi + lo exactly (fp32 accumulation of two terms)
    assert torch.equal(y, hi + lo)


def test_direct_stats_epilogue_matches_standalone():
    from bigdl.ops import native_ops as NO, fp32x3 as F3
    g = torch.Generator().manual_seed(9)
    N_, C_, K, H = 3, 64, 96, 13
    x = (torch.randn(N_, C_, H, H, generator=g) + 0.5).to(dev).contiguous(memory_format=cl)
    w = (torch.randn(K, C_, 3, 3, generator=g) * 0.05).to(dev)
    gam, bet = torch.rand(K, generator=g).to(dev) + 0.5, torch.randn(K, generator=g).to(dev)
    rep = 32
    buf = torch.zeros(2 * rep * K, device=dev)
    rm1, rv1 = torch.full((K,), 0.3, device=dev), torch.ones(K, device=dev)
    rm0, rv0 = rm1.clone(), rv1.clone()
    r = NO.conv2d_forward_stats(x, w, None, (1, 1), (1, 1), shift=rm1, sums=(buf, rep))
    assert r is not NotImplemented
    y1, part, G = r
    out1 = NO.batchnorm_forward_train_partials(y1, part, G, gam, bet, rm1, rv1, 0.1, 1e-5, relu=True, shift=rm1,
                                               rezero=True)
    y0 = F3.conv_forward(x, w, None, (1, 1), (1, 1))
    out0 = NO.batchnorm_forward_train(y0, gam, bet, rm0, rv0, 0.1, 1e-5, relu=True)
    torch.cuda.synchronize()
    assert torch.equal(y1, y0)
    assert _rel(out1[0], out0[0]) < 1e-5 and _rel(out1[1], out0[1]) < 1e-5 and _rel(out1[2], out0[2]) < 1e-5
    assert _rel(rm1, rm0) < 1e-5 and _rel(rv1, rv0) < 1e-5
    assert float(buf.abs().sum()) == 0.0
    # the BN wrote fp32 only: no producer split registered for a direct-kernel consumer
    assert F3._producer_split(out1[0], K) is None


@pytest.mark.parametrize("tail,st", [(False, 1), (True, 1), (False, 2)], ids=["mid_block", "block_tail", "strided"])
def test_direct_bnbwd_epilogue(tail, st):
    from bigdl.ops import native_ops as NO, fp32x3 as F3
    g = torch.Generator().manual_seed(11)
    N_, C_, K, H = 2, 64, 64, 11
    xb = torch.randn(N_, C_, H, H, generator=g).to(dev).contiguous(memory_format=cl)
    gam, bet = (torch.rand(C_, generator=g) + 0.5).to(dev), torch.randn(C_, generator=g).to(dev)
    res = torch.randn(N_, C_, H, H, generator=g).to(dev).contiguous(memory_format=cl) if tail else None
    coef = torch.empty(2 * C_, device=dev)
    y, mean, invstd = NO.batchnorm_forward_train(xb, gam, bet, torch.zeros(C_, device=dev), torch.ones(C_, device=dev),
                                                 0.1, 1e-5, relu=True, residual=res, coef_out=coef)
    w = (torch.randn(K, C_, 3, 3, generator=g) * 0.1).to(dev)
    P = (H - 1) // st + 1
    gy = torch.randn(N_, K, P, P, generator=g).to(dev).contiguous(memory_format=cl)
    sres = torch.randn(N_, C_, H, H, generator=g).to(dev).contiguous(memory_format=cl) if tail else None
    rep = 32
    buf = torch.zeros(2 * rep * C_, device=dev)
    fuse = {"x": xb, "mean": mean, "sums": (buf, rep)}
    if tail:
        fuse["mask"] = y
    else:
        fuse["scale"], fuse["shift"] = coef[:C_], coef[C_:]
    gi1, names = _kernels(lambda: F3.conv_backward(gy, y, w, (st, st), (1, 1), (1, 1), 1, True, None, None, 1.0,
                                                   residual=sres, bn_fuse=fuse))
    assert any("k_conv_x3" in n for n in names), names
    assert fuse.get("partial") is buf and fuse.get("G") == rep
    gg1, gb1 = torch.zeros(C_, device=dev), torch.zeros(C_, device=dev)
    gx1 = NO.batchnorm_backward_partials(gi1, xb, gam, mean, invstd, buf, rep, True, gg1, gb1, 1.0, rezero=True)
    gi0 = F3.conv_backward(gy, y, w, (st, st), (1, 1), (1, 1), 1, True, None, None, 1.0, residual=sres)
    gg0, gb0 = torch.zeros(C_, device=dev), torch.zeros(C_, device=dev)
    gx0, _ = NO.batchnorm_backward(gi0, xb, gam, mean, invstd, y.clone(), True, True, gg0, gb0, 1.0)
    torch.cuda.synchronize()
    assert torch.equal(gi1, gi0 * (y > 0))
    assert _rel(gx1, gx0) < 1e-5 and _rel(gg1, gg0) < 1e-5 and _rel(gb1, gb0) < 1e-5
    assert float(buf.abs().sum()) == 0.0


def test_direct_lazy_strided_shortcut_gradient():
    """A 1×1 stride-2 shortcut's data gradient handed back compactly (StridedGrad) and summed by the
    block's first conv as a strided residual equals the dense computation."""
    from bigdl.ops import fp32x3 as F3
    from bigdl.ops.reference import StridedGrad
    g = torch.Generator().manual_seed(13)
    N_, C_, H = 2, 64, 10
    x = torch.randn(N_, C_, H, H, generator=g).to(dev).contiguous(memory_format=cl)
    ws = (torch.randn(128, C_, 1, 1, generator=g) * 0.1).to(dev)
    gys = torch.randn(N_, 128, H // 2, H // 2, generator=g).to(dev).contiguous(memory_format=cl)
    sg = F3.conv_backward(gys, x, ws, (2, 2), (0, 0), (1, 1), 1, True, None, None, 1.0, lazy_strided=True)
    assert isinstance(sg, StridedGrad)
    dense = F3.conv_backward(gys, x, ws, (2, 2), (0, 0), (1, 1), 1, True, None, None, 1.0)
    assert _rel(sg.dense(), dense) < 1e-6
    w1 = (torch.randn(64, C_, 1, 1, generator=g) * 0.1).to(dev)
    gy1 = torch.randn(N_, 64, H, H, generator=g).to(dev).contiguous(memory_format=cl)
    gi_lazy = F3.conv_backward(gy1, x, w1, (1, 1), (0, 0), (1, 1), 1, True, None, None, 1.0, residual=sg)
    gi_dense = F3.conv_backward(gy1, x, w1, (1, 1), (0, 0), (1, 1), 1, True, None, None, 1.0, residual=dense)
    torch.cuda.synchronize()
    assert _rel(gi_lazy, gi_dense) < 1e-6


def test_direct_off_falls_back_to_split_path():
    from bigdl.ops import fp32x3 as F3
    from bigdl.utils import config
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 64, 9, 9, generator=g).to(dev).contiguous(memory_format=cl)
    w = (torch.randn(64, 64, 3, 3, generator=g) * 0.05).to(dev)
    y1 = F3.conv_forward(x, w, None, (1, 1), (1, 1))
    config.set_property("bigdl.fp32.direct", False)
    try:
        y0, names = _kernels(lambda: F3.conv_forward(x, w, None, (1, 1), (1, 1)))
    finally:
        config.set_property("bigdl.fp32.direct", True)
    assert not any("k_conv_x3" in n for n in names)
    assert _rel(y1, y0) < 2e-5


@pytest.mark.parametrize("c4,C,K,H,k,st,pd", [(False, 3, 64, 30, 7, 2, 3), (True, 3, 64, 30, 7, 2, 3),
                                             (True, 3, 64, 31, 7, 2, 3), (True, 4, 32, 9, 3, 1, 1),
                                             (True, 1, 16, 12, 5, 1, 0)],
                         ids=["s2d", "c4", "c4_odd", "c4_3x3", "c4_gray5x5"])
def test_direct_stem(c4, C, K, H, k, st, pd):
    """The fp32 RGB stem (≤ 4 input channels) on the direct kernels — either the 4-channel gather
    (bigdl.fp32.stemC4: conv_x3 MODE 2, 8 taps × 4 channels per k-tile; the C4 fp32 weight gradient
    folded onto the master's taps) or the space-to-depth image (a 4×4 stride-1 conv): forward (+ BN
    statistics epilogue) and weight gradient against fp64."""
    from bigdl.ops import fp32x3 as F3, native_ops as NO
    from bigdl.utils import config
    config.set_property("bigdl.fp32.stemC4", c4)
    try:
        g = torch.Generator().manual_seed(17)
        N_ = 2
        x = torch.randn(N_, C, H, H, generator=g)
        w = torch.randn(K, C, k, k, generator=g) * 0.1
        xr, wr = x.double(), w.double().requires_grad_()
        yr = F.conv2d(xr, wr, None, st, pd)
        gy = torch.randn(yr.shape, generator=g)
        yr.backward(gy.double())
        xd = x.to(dev).contiguous(memory_format=cl)
        slot = [None]
        y, names = _kernels(lambda: F3.conv_forward(xd, w.to(dev), None, (st, st), (pd, pd), slot=slot))
        prep = "k_pad4_f32" if c4 else "k_s2d_f32"
        assert any(prep in n for n in names) and any("k_conv_x3" in n for n in names), names
        assert _rel(y, yr) < 2e-5, _rel(y, yr)
        gw = torch.zeros(K, k, k, C, device=dev).permute(0, 3, 1, 2)
        for rep_ in range(2):  # twice: the persistent accumulation buffer is cleared by the fold
            gw.zero_()
            r, names = _kernels(lambda: F3.conv_backward(gy.to(dev).contiguous(memory_format=cl), xd, w.to(dev),
                                                         (st, st), (pd, pd), (1, 1), 1, False, gw, None, 1.0,
                                                         slot=slot))
            assert r is None and (rep_ == 1 or not any(prep in n for n in names)), names  # forward's image reused
            assert _rel(gw, wr.grad) < 2e-5, _rel(gw, wr.grad)
        # the statistics epilogue through the stem path
        rep = 8
        buf = torch.zeros(2 * rep * K, device=dev)
        shift = torch.zeros(K, device=dev)
        out = NO.conv2d_forward_stats(xd, w.to(dev), None, (st, st), (pd, pd), shift=shift, sums=(buf, rep))
        assert out is not NotImplemented
        torch.cuda.synchronize()
        ys = out[0].double().cpu()
        assert _rel(ys, yr) < 2e-5
        assert _rel(buf.reshape(2, rep, K).sum(1)[0], ys.sum((0, 2, 3))) < 1e-5
    finally:
        config.clear_property("bigdl.fp32.stemC4")


def test_weight_operand_cache_matches_host_forms():
    """csrc/weight_x3.hip: every cached fp32-mode weight operand (forward chunks, flipped dgrad chunks,
    parity sub-filters, the s2d stem filter, Linear [hi | lo | hi] rows) equals the host-side form
    bit for bit, and goes stale exactly when the weight changes (torch in-place write, or a native
    update reported by mark_dirty)."""
    from bigdl.ops import fp32x3 as F3
    g = torch.Generator().manual_seed(5)
    base = torch.randn(64, 3, 3, 96, generator=g).to(dev)   # KRSC physical, like the arena
    w4 = base.permute(0, 3, 1, 2)                             # logical [K][C][R][S]
    k, c, r, s = w4.shape
    ref_fwd = F3.chunk_split(w4.float().permute(0, 2, 3, 1).reshape(k, -1).contiguous())
    got = F3._wprep(w4, ("fwd",))
    torch.cuda.synchronize()
    assert torch.equal(got.reshape(-1), ref_fwd.reshape(-1))
    classes = [((2, 0), (2, 0)), ((1,), (2, 0)), ((2, 0), (1,)), ((1,), (1,))]
    subs = F3._w_dgrad(w4, classes)
    for (a, b), sub in zip(classes, subs):
        ref = F3.chunk_split(w4[:, :, list(a)][:, :, :, list(b)].permute(1, 2, 3, 0).reshape(c, -1).contiguous())
        assert torch.equal(sub.reshape(-1), ref.reshape(-1)), (a, b)
    # stem: [64][3][7][7] → s2d [64][4][4][32]
    ws = torch.randn(64, 7, 7, 3, generator=g).to(dev).permute(0, 3, 1, 2)
    got = F3._wprep(ws, ("s2d",))
    ref = F3.chunk_split(F3._stem_weights(ws).reshape(64, -1))
    assert torch.equal(got.reshape(-1), ref.reshape(-1))
    # stem: [64][3][7][7] → C4 [64][7][64] (8 taps × 4 channels per chunk, zero past 49 taps / 3 channels)
    got = F3._wprep(ws, ("c4",))
    w4p = torch.zeros(64, 56, 4, device=dev)
    w4p[:, :49, :3] = ws.permute(0, 2, 3, 1).reshape(64, 49, 3)
    ref = F3.chunk_split(w4p.reshape(64, -1))
    assert torch.equal(got.reshape(-1), ref.reshape(-1))
    # Linear rows, plain and transposed, with padded rows / columns
    wl = torch.randn(10, 20, generator=g).to(dev)
    got = F3._wprep(wl, ("rows3", 12, 24, False))
    ref = F3.split(wl, 24, F3.HLH, False, out=torch.zeros((12, 72), dtype=torch.bfloat16, device=dev))
    assert torch.equal(got, ref)
    got = F3._wprep(wl, ("rows3", 20, 16, True))
    ref = F3.split(wl.t().contiguous(), 16, F3.HLH, False, out=torch.zeros((20, 48), dtype=torch.bfloat16, device=dev))
    assert torch.equal(got, ref)
    # staleness: a torch in-place write bumps the version counter
    before = F3._wprep(w4, ("fwd",)).clone()
    assert torch.equal(F3._wprep(w4, ("fwd",)), before)      # cached: same contents
    base.mul_(2.0)
    assert torch.equal(F3._wprep(w4, ("fwd",)).reshape(-1),
                       F3.chunk_split(w4.permute(0, 2, 3, 1).reshape(k, -1).contiguous()).reshape(-1))
    # a write torch does not see (the fused SGD kernel) is reported through mark_dirty
    from bigdl.ops import native_ops as NO
    flat = base.view(-1)
    grad = torch.randn(flat.shape, generator=g).to(dev)
    assert NO.sgd_step(flat, grad, None, 0.5, 0.0, 0.0, 0.0, False, True) is not NotImplemented
    torch.cuda.synchronize()
    assert torch.equal(F3._wprep(w4, ("fwd",)).reshape(-1),
                       F3.chunk_split(w4.permute(0, 2, 3, 1).reshape(k, -1).contiguous()).reshape(-1))


def test_fp32_threshold_and_colsum_kernels():
    """fp32 ReLU / Threshold (elementwise.hip k_threshold_*_f32) and the fp32 column sum (gemm.hip
    k_colsum_f32) against torch, including an odd tail."""
    from bigdl.ops import native_ops as NO
    g = torch.Generator().manual_seed(6)
    x = torch.randn(1001, generator=g).to(dev)
    y, names = _kernels(lambda: NO.relu_forward(x, 0.1, -0.5))
    assert any("k_threshold_fwd_f32" in n for n in names), names
    assert torch.equal(y, torch.where(x > 0.1, x, torch.full_like(x, -0.5)))
    gy = torch.randn(1001, generator=g).to(dev)
    gx = NO.relu_backward(gy, x, 0.1)
    assert torch.equal(gx, torch.where(x > 0.1, gy, torch.zeros_like(gy)))
    m = torch.randn(777, 1000, generator=g).to(dev)
    out = torch.ones(1000, device=dev)
    NO.colsum_acc(m, out, 0.5)
    torch.cuda.synchronize()
    assert _rel(out, 1.0 + 0.5 * m.double().sum(0)) < 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("C,K,H", [(256, 1024, 14), (512, 2048, 7)])
def test_conv_epilogue_statistics_are_exact_every_time(C, K, H):
    """The fp32 conv's BN-statistics epilogue, repeated: every launch's Σ(y − K), Σ(y − K)² must match
    fp64 sums of the output it wrote.  (The epilogue's LDS staging once synchronised with a raw
    s_barrier, which on gfx950 does not drain the writing wave's ds_writes: a few launches in a hundred
    folded stale partials — BN variances off by up to 65 % on some training steps.)"""
    from bigdl.ops import fp32x3 as F3
    torch.manual_seed(0)
    x = torch.randn(128, C, H, H, device=dev).contiguous(memory_format=torch.channels_last)
    w = torch.randn(K, C, 1, 1, device=dev) * (2.0 / C) ** 0.5
    shift = torch.randn(K, device=dev) * 0.1
    rep = 32
    buf = torch.zeros(2 * rep * K, device=dev)
    bad = []
    for it in range(120):
        buf.zero_()
        y, _b, _r = F3.conv_forward_stats(x, w, (1, 1), (0, 0), (1, 1), (buf, rep), shift)
        yd = y.double().permute(0, 2, 3, 1).reshape(-1, K) - shift.double()
        b = buf.double().reshape(2, rep, K).sum(1)
        e2 = float(((b[1] - (yd * yd).sum(0)).abs() / (yd * yd).sum(0)).max())
        if e2 > 1e-5:
            bad.append((it, e2))
    assert not bad, bad[:5]
