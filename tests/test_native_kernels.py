"""Numerics of the native HIP kernels vs the fp32 reference ops (bigdl/ops/reference.py).

Each test asserts the native library is loaded and the op actually dispatched natively (so a
silent fallback to the reference path fails the test)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

dev = "cuda"


def _native():
    from bigdl.ops import native, native_status
    st = native_status()
    assert st["loaded"], st
    return native


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def test_native_loaded_and_ops_registered():
    N = _native()
    for op in ["cast_copy", "relu_forward", "batchnorm_forward_train", "batchnorm_backward", "cross_entropy_fused",
               "sgd_step"]:
        assert N.has(op), op


@pytest.mark.parametrize("n", [8, 1000, 4099, 1 << 20])
def test_cast(n):
    N = _native()
    x = torch.randn(n, device=dev)
    b = torch.empty(n, dtype=torch.bfloat16, device=dev)
    assert N.cast_copy(b, x) is not NotImplemented
    torch.testing.assert_close(b, x.to(torch.bfloat16), rtol=0, atol=0)
    f = torch.empty(n, device=dev)
    N.cast_copy(f, b)
    torch.testing.assert_close(f, b.float(), rtol=0, atol=0)


def test_relu_fwd_bwd():
    N = _native()
    x = _cl(torch.randn(4, 64, 7, 7, device=dev).bfloat16())
    y = N.relu_forward(x)
    torch.testing.assert_close(y, torch.relu(x))
    gy = _cl(torch.randn_like(x))
    gx = N.relu_backward(gy, y)
    torch.testing.assert_close(gx, gy * (x > 0).to(gy.dtype))


@pytest.mark.parametrize("shape", [(8, 64, 14, 14), (4, 256, 7, 7), (2, 2048, 7, 7), (3, 24, 5, 5), (64, 512)])
@pytest.mark.parametrize("relu,res", [(False, False), (True, False), (True, True)])
def test_bn_forward_backward(shape, relu, res):
    N = _native()
    from bigdl.ops import reference as R
    C = shape[1]
    x = torch.randn(*shape, device=dev) * 3 + 1.5
    x = (_cl(x) if len(shape) == 4 else x).bfloat16()
    if len(shape) == 4:
        x = _cl(x)
    gamma = torch.rand(C, device=dev) + 0.5
    beta = torch.randn(C, device=dev)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    rm2, rv2 = rm.clone(), rv.clone()
    r = None
    if res:
        r = torch.randn(*shape, device=dev).bfloat16()
        r = _cl(r) if len(shape) == 4 else r
    out = N.batchnorm_forward_train(x, gamma, beta, rm, rv, 0.1, 1e-5, relu=relu, residual=r)
    assert out is not NotImplemented
    y, mean, invstd = out
    yr, meanr, invr = R.batchnorm_forward_train(x.float(), gamma, beta, rm2, rv2, 0.1, 1e-5, relu=relu,
                                                residual=None if r is None else r.float())
    torch.testing.assert_close(mean, meanr, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(invstd, invr, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(rm, rm2, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(rv, rv2, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(y.float(), yr.float(), rtol=2e-2, atol=3e-2)
    # backward
    gy = torch.randn(*shape, device=dev).bfloat16()
    gy = _cl(gy) if len(shape) == 4 else gy
    gg, gb = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    gg2, gb2 = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    cb, cb2 = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    out = N.batchnorm_backward(gy, x, gamma, mean, invstd, y=y, relu=relu, gg_acc=gg, gb_acc=gb, scale=0.5,
                               cbias_acc=cb, cbias_scale=1.0, want_gres=res)
    assert out is not NotImplemented
    gx, gres = out
    gxr, gresr = R.batchnorm_backward(gy.float(), x.float(), gamma, mean, invstd, y=y.float(), relu=relu,
                                      gg_acc=gg2, gb_acc=gb2, scale=0.5, cbias_acc=cb2, want_gres=res)
    torch.testing.assert_close(cb, cb2, rtol=0, atol=5e-2)
    if res:
        torch.testing.assert_close(gres.float(), gresr.float())
    torch.testing.assert_close(gg, gg2, rtol=2e-3, atol=2e-2)
    torch.testing.assert_close(gb, gb2, rtol=2e-3, atol=2e-2)
    torch.testing.assert_close(gx.float(), gxr.float(), rtol=3e-2, atol=3e-2)


def test_bn_infer():
    N = _native()
    from bigdl.ops import reference as R
    x = _cl(torch.randn(4, 128, 9, 9, device=dev).bfloat16())
    C = 128
    g, b, m, v = torch.rand(C, device=dev), torch.randn(C, device=dev), torch.randn(C, device=dev), torch.rand(C, device=dev) + .5
    y = N.batchnorm_forward_infer(x, g, b, m, v, 1e-5, relu=True)
    yr = R.batchnorm_forward_infer(x.float(), g, b, m, v, 1e-5, relu=True)
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("n", [1, 7, 4096, 25557032])
def test_zero_fill(n):
    """The gradient-arena clear: native 16-B store kernel, tail and all (no torch fill kernel)."""
    N = _native()
    from bigdl import ops
    t = torch.randn(n + 1, device=dev)[:n] if n % 4 == 0 else torch.randn(n, device=dev)
    assert N.zero_fill(t) is not NotImplemented
    assert int(torch.count_nonzero(t)) == 0
    g = torch.randn(n + 3, device=dev)
    ops.zero_fill(g)
    assert int(torch.count_nonzero(g)) == 0


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("weights", [False, True])
@pytest.mark.parametrize("tdtype", [torch.float32, torch.int64])
def test_cross_entropy(dtype, weights, tdtype):
    """float labels on the device go to the float-target kernel (no per-step int cast), others to
    the int32 one; both against the fp32 reference."""
    N = _native()
    from bigdl.ops import reference as R
    B, K = 37, 1000
    x = (torch.randn(B, K, device=dev) * 4).to(dtype)
    t = torch.randint(1, K + 1, (B,), device=dev).to(tdtype)
    t[3] = -1  # padding value -> skipped
    w = torch.rand(K, device=dev) if weights else None
    loss, g = N.cross_entropy_fused(x, t, w, True, -1)
    lr, gr = R.cross_entropy_fused(x.float(), t.float(), w, True, -1)
    torch.testing.assert_close(loss, lr, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(g.float(), gr.float(), rtol=2e-2, atol=2e-4 if dtype == torch.float32 else 2e-3)


def test_logsoftmax():
    N = _native()
    from bigdl.ops import reference as R
    x = torch.randn(33, 100, device=dev)
    y = N.log_softmax_forward(x)
    torch.testing.assert_close(y, R.log_softmax_forward(x), rtol=1e-5, atol=1e-5)
    gy = torch.randn_like(x)
    torch.testing.assert_close(N.log_softmax_backward(gy, y), R.log_softmax_backward(gy, y), rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("nesterov,first", [(True, True), (True, False), (False, False)])
def test_sgd(nesterov, first):
    N = _native()
    from bigdl.ops import reference as R
    n = 4096 + 64
    w = torch.randn(n, device=dev)
    g = torch.randn(n, device=dev)
    buf = torch.randn(n, device=dev)
    w2, buf2 = w.clone(), buf.clone()
    sh = torch.empty(n, dtype=torch.bfloat16, device=dev)
    damp = 0.0 if nesterov else 0.1
    N.sgd_step(w, g, buf, 0.1, 0.9, damp, 1e-4, nesterov, first, 0.5, sh)
    R.sgd_step(w2, g, buf2, 0.1, 0.9, damp, 1e-4, nesterov, first, 0.5)
    torch.testing.assert_close(w, w2, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(buf, buf2, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(sh, w.bfloat16(), rtol=0, atol=0)


def test_adam():
    N = _native()
    from bigdl.ops import reference as R
    n = 1024
    w, g = torch.randn(n, device=dev), torch.randn(n, device=dev)
    m, v = torch.zeros(n, device=dev), torch.zeros(n, device=dev)
    w2, m2, v2 = w.clone(), m.clone(), v.clone()
    for step in (1, 2, 3):
        N.adam_step(w, g, m, v, 1e-3, 0.9, 0.999, 1e-8, step)
        R.adam_step(w2, g, m2, v2, 1e-3, 0.9, 0.999, 1e-8, step)
    torch.testing.assert_close(w, w2, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("graph_counter", [False, True])
def test_adagrad_fused_matches_optim_method(graph_counter):
    """k_adagrad (one pass over w, g, the accumulator and the bf16 shadow) against the torch form
    of Adagrad.optimize (DL/optim/Adagrad.scala), with weight decay and a gradient scale, host or
    device iteration counter."""
    N = _native()
    n = 1003  # a tail past the float4 body
    w = torch.randn(n, device=dev)
    g = torch.randn(n, device=dev)
    s = torch.zeros(n, device=dev)
    shadow = torch.empty(n, dtype=torch.bfloat16, device=dev)
    w2, s2 = w.clone(), s.clone()
    lr, dec, wd, sc = 0.01, 0.001, 1e-3, 0.5
    nt = torch.zeros(1, device=dev)
    for it in range(3):
        N.adagrad_step(w, g, s, lr, dec, it, wd, sc, shadow, dev_n=nt if graph_counter else None)
        nt.add_(1)
        gg = g * sc + wd * w2
        s2.addcmul_(gg, gg)
        w2.addcdiv_(gg, s2.sqrt().add_(1e-10), value=-lr / (1 + it * dec))
    torch.testing.assert_close(w, w2, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(s, s2, rtol=1e-5, atol=1e-6)
    assert torch.equal(shadow, w.bfloat16())


def test_layers_use_native_path():
    """Spatial BN + ReLU layers on bf16 NHWC activations go through the native kernels."""
    _native()
    from bigdl.nn import SpatialBatchNormalization, ReLU, Sequential
    from bigdl.utils.engine import Engine
    from bigdl.utils import config
    config.set_property("bigdl.compute.dtype", "bf16")
    Engine.init(device="cuda:0")
    m = Sequential().add(SpatialBatchNormalization(64)).add(ReLU(True)).cuda()
    x = _cl(torch.randn(2, 64, 8, 8, device=dev).bfloat16())
    y = m.forward(x)
    g = m.backward(x, torch.ones_like(y))
    assert y.dtype == torch.bfloat16 and g.dtype == torch.bfloat16
    assert torch.isfinite(g.float()).all()


# ---------------------------------------------------------------------------------------- conv
CONV_CASES = [
    # N, C, H, W, K, R, S, stride, pad
    (2, 64, 14, 14, 256, 1, 1, 1, 0),     # 1x1 expand
    (2, 256, 14, 14, 64, 1, 1, 1, 0),     # 1x1 reduce (K=64 tile)
    (2, 64, 15, 13, 64, 3, 3, 1, 1),      # 3x3 s1, odd spatial
    (2, 128, 16, 16, 128, 3, 3, 2, 1),    # 3x3 s2 (ResNet v1.5 downsample)
    (2, 256, 14, 14, 512, 1, 1, 2, 0),    # 1x1 s2 projection shortcut
    (2, 3, 32, 32, 64, 7, 7, 2, 3),       # stem (C=3 padded to 4: two-tap C4 gather)
    (2, 3, 17, 19, 16, 3, 3, 1, 1),       # RGB 3x3 (C4, R·S odd → half-chunk tail)
    (2, 4, 12, 12, 32, 5, 5, 2, 2),       # C = 4 exactly
    (2, 1, 28, 28, 6, 5, 5, 1, 0),        # LeNet conv1 (C=1 → 4, K=6: per-element epilogue tail)
    (3, 24, 9, 9, 40, 5, 5, 1, 2),        # Inception-ish odd channels
]


def _conv_ref(x, w4, stride, pad):
    return torch.nn.functional.conv2d(x.float(), w4.float(), None, stride, pad)


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_forward(case):
    N = _native()
    n, c, h, w, k, r, s, st, pd = case
    x = _cl(torch.randn(n, c, h, w, device=dev).bfloat16())
    w4 = _cl(torch.randn(k, c, r, s, device=dev).bfloat16() * 0.1)
    b = torch.randn(k, device=dev)
    y = N.conv2d_forward(x, w4, b, (st, st), (pd, pd))
    assert y is not NotImplemented
    ref = _conv_ref(x, w4, (st, st), (pd, pd)) + b.view(1, -1, 1, 1)
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_backward(case):
    N = _native()
    n, c, h, w, k, r, s, st, pd = case
    if k % 8:
        pytest.skip("K % 8")
    x = _cl(torch.randn(n, c, h, w, device=dev).bfloat16())
    w4 = _cl(torch.randn(k, c, r, s, device=dev).bfloat16() * 0.1)
    xr = x.float().requires_grad_(True)
    wr = w4.float().requires_grad_(True)
    yr = torch.nn.functional.conv2d(xr, wr, None, (st, st), (pd, pd))
    gy = _cl(torch.randn_like(yr).bfloat16())
    yr.backward(gy.float())
    gw = torch.zeros(k, r, s, c, device=dev).permute(0, 3, 1, 2)  # KRSC physical like the arena
    gw.fill_(0.5)
    gi = N.conv2d_backward(gy, x, w4, (st, st), (pd, pd), (1, 1), 1, True, gw, None, 2.0)
    assert gi is not NotImplemented
    torch.testing.assert_close(gi.float(), xr.grad, rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(gw, 0.5 + 2.0 * wr.grad, rtol=2e-2, atol=5e-2)


@pytest.mark.parametrize("case", [(4, 64, 28, 28, 64, 3, 3, 1, 1), (2, 256, 14, 14, 1024, 1, 1, 1, 0),
                                  (2, 128, 16, 16, 128, 3, 3, 2, 1), (2, 3, 32, 32, 64, 7, 7, 2, 3),
                                  (3, 24, 9, 9, 40, 5, 5, 1, 2)])
def test_conv_wgrad_lds_staged_epilogue(case, monkeypatch):
    """BIGDL_WGRAD_EPI=1: split-K partial tiles staged in LDS and added with 256-B atomic
    wave-instructions — same weight gradient as the register epilogue and the fp32 reference."""
    N = _native()
    n, c, h, w, k, r, s, st, pd = case
    if k % 8:
        pytest.skip("K % 8")
    x = _cl(torch.randn(n, c, h, w, device=dev).bfloat16())
    w4 = _cl(torch.randn(k, c, r, s, device=dev).bfloat16() * 0.1)
    wr = w4.float().requires_grad_(True)
    yr = torch.nn.functional.conv2d(x.float(), wr, None, (st, st), (pd, pd))
    gy = _cl(torch.randn_like(yr).bfloat16())
    yr.backward(gy.float())
    out = {}
    for epi in ("0", "1"):
        monkeypatch.setenv("BIGDL_WGRAD_EPI", epi)
        gw = torch.zeros(k, r, s, c, device=dev).permute(0, 3, 1, 2)
        N.conv2d_backward(gy, x, w4, (st, st), (pd, pd), (1, 1), 1, False, gw, None, 1.0)
        out[epi] = gw.clone()
    torch.testing.assert_close(out["1"], wr.grad, rtol=2e-2, atol=5e-2)
    torch.testing.assert_close(out["1"], out["0"], rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_lstm_cell_kernels(dtype):
    from bigdl.ops import reference as R
    N = _native()
    B, H, Tn = 5, 40, 3
    seq = torch.randn(B, Tn, 4 * H, device=dev).to(dtype)
    hg = torch.randn(B, 4 * H, device=dev).to(dtype)
    c0 = torch.randn(B, H, device=dev)
    out = torch.zeros(B, Tn, H, device=dev, dtype=dtype)
    r = N.lstm_cell_forward(seq[:, 1], hg, c0, h_out=out[:, 1])
    assert r is not NotImplemented
    e = R.lstm_cell_forward(seq[:, 1], hg, c0)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    for a, b in zip(r, e):
        torch.testing.assert_close(a.float(), b.float(), rtol=tol, atol=tol)
    torch.testing.assert_close(out[:, 1].float(), e[0].float(), rtol=tol, atol=tol)
    gy = torch.randn(B, Tn, H, device=dev).to(dtype)
    gh2 = torch.randn(B, H, device=dev).to(dtype)
    gc = torch.randn(B, H, device=dev)
    dgs = torch.zeros(B, Tn, 4 * H, device=dev, dtype=dtype)
    rb = N.lstm_cell_backward(gy[:, 2], gh2, gc, e[2], e[3], c0, dg_out=dgs[:, 2])
    assert rb is not NotImplemented
    eb = R.lstm_cell_backward(gy[:, 2], gh2, gc, e[2], e[3], c0)
    for a, b in zip(rb, eb):
        torch.testing.assert_close(a.float(), b.float(), rtol=tol, atol=tol)


def test_recurrent_lstm_gpu_vs_cpu():
    """Recurrent(LSTM) on the GPU (bf16 GEMMs + native cell) vs the CPU fp32 path."""
    import copy
    from bigdl.nn import Recurrent, LSTM
    _native()
    torch.manual_seed(0)
    cpu = Recurrent().add(LSTM(32, 64))
    gpu = copy.deepcopy(cpu).cuda()
    x = torch.randn(8, 10, 32)
    y = cpu.forward(x)
    yg = gpu.forward(x.cuda())
    torch.testing.assert_close(yg.float().cpu(), y, rtol=3e-2, atol=3e-2)
    gy = torch.randn_like(y)
    gi = cpu.backward(x, gy)
    gig = gpu.backward(x.cuda(), gy.cuda())
    torch.testing.assert_close(gig.float().cpu(), gi, rtol=5e-2, atol=5e-2)
    for a, b in zip(gpu.parameters()[1], cpu.parameters()[1]):
        torch.testing.assert_close(a.float().cpu(), b, rtol=5e-2, atol=5e-2 * float(b.abs().max()))


@pytest.mark.parametrize("case", [c for c in CONV_CASES if c[4] % 8 == 0])
def test_conv_forward_residual_and_stats(case):
    """Epilogue extras: residual add (used by the dgrad gradient-sum fold) and per-row-tile Σy/Σy²
    partials that replace the following BN's statistics pass."""
    N = _native()
    from bigdl.ops import native_ops as NO
    n, c, h, w, k, r, s, st, pd = case
    x = _cl(torch.randn(n, c, h, w, device=dev).bfloat16())
    w4 = _cl(torch.randn(k, c, r, s, device=dev).bfloat16() * 0.1)
    y, part, G = NO.conv2d_forward_stats(x, w4, None, (st, st), (pd, pd))
    ref = _conv_ref(x, w4, (st, st), (pd, pd))
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)
    # the partials are taken from the fp32 accumulators (before the bf16 store), so they match the
    # fp32 convolution of the same bf16 operands to summation-order rounding
    s1 = part.view(2, G, k).sum(1)
    torch.testing.assert_close(s1[0], ref.sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
    torch.testing.assert_close(s1[1], (ref * ref).sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
    res = _cl(torch.randn_like(ref).bfloat16())
    y2 = NO._conv_fwd_impl(x, w4, None, (st, st), (pd, pd), res=res)
    torch.testing.assert_close(y2.float(), ref + res.float(), rtol=2e-2, atol=3e-2)


def test_bn_forward_from_conv_partials():
    N = _native()
    from bigdl.ops import native_ops as NO, reference as R
    x = _cl(torch.randn(4, 64, 14, 14, device=dev).bfloat16())
    w4 = _cl(torch.randn(128, 64, 3, 3, device=dev).bfloat16() * 0.05)
    y, part, G = NO.conv2d_forward_stats(x, w4, None, (1, 1), (1, 1))
    g = torch.rand(128, device=dev) + 0.5
    b = torch.randn(128, device=dev)
    rm1, rv1 = torch.zeros(128, device=dev), torch.ones(128, device=dev)
    rm2, rv2 = rm1.clone(), rv1.clone()
    ib = torch.randn(128, device=dev)
    out, mean, invstd = NO.batchnorm_forward_train_partials(y, part, G, g, b, rm1, rv1, 0.1, 1e-3, relu=True,
                                                            in_bias=ib)
    ro, rmean, rinv = R.batchnorm_forward_train(y, g, b, rm2, rv2, 0.1, 1e-3, relu=True, in_bias=ib)
    torch.testing.assert_close(mean, rmean, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(invstd, rinv, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(rm1, rm2, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(rv1, rv2, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(out.float(), ro.float(), rtol=2e-2, atol=2e-2)


def test_bn_from_conv_partials_large_mean():
    """Conv-epilogue statistics with outputs of mean ≈ 64 and std ≈ 0.5 over a 56²-sized batch
    (thousands of 128-row partials): the fp64 combine of the unshifted Σy, Σy² partials must keep
    the variance of the stored values (fp32 two-pass reference)."""
    _native()
    from bigdl.ops import native_ops as NO
    C, K = 64, 64
    x = _cl(torch.randn(80, C, 32, 32, device=dev).bfloat16())
    w4 = _cl((torch.randn(K, C, 1, 1, device=dev) * 0.06).bfloat16())
    bias = torch.full((K,), 64.0, device=dev)
    y, part, G = NO.conv2d_forward_stats(x, w4, bias, (1, 1), (0, 0))
    assert G > 512  # exercises the fp64 pre-fold
    g, b = torch.ones(K, device=dev), torch.zeros(K, device=dev)
    rm, rv = torch.zeros(K, device=dev), torch.ones(K, device=dev)
    out, mean, invstd = NO.batchnorm_forward_train_partials(y, part, G, g, b, rm, rv, 0.1, 1e-5)
    yf = y.float()
    ref_mean = yf.mean((0, 2, 3))
    ref_var = yf.var((0, 2, 3), unbiased=False)
    torch.testing.assert_close(mean, ref_mean, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(1.0 / invstd ** 2 - 1e-5, ref_var, rtol=1e-2, atol=1e-4)


def test_dgrad_residual_fold():
    N = _native()
    x = _cl(torch.randn(2, 64, 14, 14, device=dev).bfloat16())
    w4 = _cl(torch.randn(128, 64, 3, 3, device=dev).bfloat16() * 0.1)
    gy = _cl(torch.randn(2, 128, 14, 14, device=dev).bfloat16())
    res = _cl(torch.randn(2, 64, 14, 14, device=dev).bfloat16())
    gi0 = N.conv2d_backward(gy, x, w4, (1, 1), (1, 1), (1, 1), 1, True, None, None, 0.0)
    gi1 = N.conv2d_backward(gy, x, w4, (1, 1), (1, 1), (1, 1), 1, True, None, None, 0.0, residual=res)
    torch.testing.assert_close(gi1.float(), gi0.float() + res.float(), rtol=2e-2, atol=3e-2)


@pytest.mark.parametrize("case", [(2, 64, 15, 13, 128, 3, 3, 2, 1), (2, 64, 14, 14, 64, 1, 1, 2, 0),
                                  (1, 32, 11, 12, 64, 5, 5, 2, 2), (2, 16, 9, 9, 32, 3, 3, 3, 1)])
def test_strided_dgrad_subpixel(case):
    """Sub-pixel strided backward-data (sh·sw stride-1 launches with output scatter) vs autograd,
    with and without the fused residual-gradient sum."""
    N = _native()
    n, c, h, w, k, r, s, st, pd = case
    x = _cl(torch.randn(n, c, h, w, device=dev).bfloat16())
    w4 = _cl(torch.randn(k, c, r, s, device=dev).bfloat16() * 0.1)
    xr = x.float().requires_grad_(True)
    yr = torch.nn.functional.conv2d(xr, w4.float(), None, (st, st), (pd, pd))
    gy = _cl(torch.randn_like(yr).bfloat16())
    yr.backward(gy.float())
    gi = N.conv2d_backward(gy, x, w4, (st, st), (pd, pd), (1, 1), 1, True, None, None, 0.0)
    torch.testing.assert_close(gi.float(), xr.grad, rtol=3e-2, atol=3e-2)
    res = _cl(torch.randn_like(x))
    gi2 = N.conv2d_backward(gy, x, w4, (st, st), (pd, pd), (1, 1), 1, True, None, None, 0.0, residual=res)
    torch.testing.assert_close(gi2.float(), xr.grad + res.float(), rtol=3e-2, atol=4e-2)


@pytest.mark.parametrize("shape", [(2, 16, 13, 11), (2, 64, 28, 28), (1, 8, 9, 12)])
@pytest.mark.parametrize("cfg", [((3, 3), (2, 2), (1, 1), False), ((2, 2), (2, 2), (0, 0), True),
                                 ((3, 3), (2, 2), (0, 0), True), ((3, 3), (1, 1), (1, 1), False),
                                 ((3, 3), (2, 2), (1, 1), True)])
def test_maxpool_native(cfg, shape):
    """Generic and 3×3 / stride-2 (all window loads in flight) kernels against the reference,
    forward values and argmax-routed backward, with ceil-mode overhang."""
    N = _native()
    from bigdl.ops import reference as R
    k, s, p, ceil = cfg
    x = _cl(torch.randn(*shape, device=dev).bfloat16())
    y, idx = N.maxpool2d_forward(x, k, s, p, ceil)
    yr, idr = R.maxpool2d_forward(x.float(), k, s, p, ceil)
    torch.testing.assert_close(y.float(), yr)
    gy = _cl(torch.randn_like(yr).bfloat16())
    gx = N.maxpool2d_backward(gy, x, idx, k, s, p, ceil)
    gr = R.maxpool2d_backward(gy.float(), x.float(), idr, k, s, p, ceil)
    torch.testing.assert_close(gx.float(), gr, rtol=1e-2, atol=1e-2)


def test_block_tail_bn_backward_fused_into_next_dgrad():
    """Two ImageNet bottlenecks on bf16: the second block's first conv applies the first block's
    tail ReLU mask and produces its BN reductions in the dgrad epilogue; gradients must match the
    same fused model with that tail fusion switched off."""
    _native()
    import copy
    from bigdl.models.resnet import Convolution, Sbn
    from bigdl.nn import ConcatTable, Identity, Sequential, ReLU, CAddTable, SpatialConvolution, \
        SpatialBatchNormalization
    from bigdl.nn.fusion import fuse
    from bigdl.utils.engine import Engine
    from bigdl.utils import config
    config.set_property("bigdl.compute.dtype", "bf16")
    Engine.init(device="cuda:0")
    torch.manual_seed(0)

    def block(n_in, n, proj):
        s = Sequential().add(Convolution(n_in, n, 1, 1)).add(Sbn(n)).add(ReLU(True))
        s.add(Convolution(n, n, 3, 3, 1, 1, 1, 1)).add(Sbn(n)).add(ReLU(True))
        s.add(Convolution(n, n * 4, 1, 1)).add(Sbn(n * 4))
        sc = Sequential().add(Convolution(n_in, n * 4, 1, 1)).add(Sbn(n * 4)) if proj else Identity()
        return Sequential().add(ConcatTable().add(s).add(sc)).add(CAddTable(True)).add(ReLU(True))
    a = Sequential().add(block(64, 16, True)).add(block(64, 16, False)).add(block(64, 16, False))
    for m in a.flattened_modules():
        if isinstance(m, SpatialBatchNormalization):
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.2, 0.2)
    b = copy.deepcopy(a)
    fuse(a)
    fuse(b)
    heads = [m for m in a.flattened_modules() if isinstance(m, SpatialConvolution) and m._tail_candidates]
    assert len(heads) == 3
    for m in b.flattened_modules():
        if isinstance(m, SpatialConvolution):
            m._tail_candidates = None
    a.cuda()
    b.cuda()
    hits = []
    orig = SpatialConvolution._tail_target
    SpatialConvolution._tail_target = lambda self, x: (lambda r: (hits.append(r), r)[1])(orig(self, x))
    try:
        x = _cl(torch.randn(4, 64, 12, 12, device=dev).bfloat16())
        gy = _cl(torch.randn(4, 64, 12, 12, device=dev).bfloat16())
        for m in (a, b):
            m.zeroGradParameters()
        ya, yb = a.forward(x), b.forward(x)
        ga, gb = a.backward(x, gy), b.backward(x, gy)
    finally:
        SpatialConvolution._tail_target = orig
    assert sum(h is not None for h in hits) == 2  # blocks 2 and 3 consume a tail
    torch.testing.assert_close(ya.float(), yb.float())
    # both paths accumulate the BN reductions with fp32 atomics (order varies run to run): an element
    # left small by cancellation can differ by a bf16 ulp of the large terms, so compare to the scale
    d, ref = (ga.float() - gb.float()).abs(), gb.float().abs()
    assert float(d.max()) <= 2e-2 * float(ref.max()) + 5e-2, (float(d.max()), float(ref.max()))
    assert float((d > 5e-2 + 5e-2 * ref).float().mean()) < 1e-3
    # parameter gradients to the scale of each tensor (a conv bias feeding a training BN has an
    # exactly-zero true gradient: both paths hold rounding noise there, skipped by the scale floor)
    for u, v in zip(a.parameters()[1], b.parameters()[1]):
        scale = float(v.float().abs().max())
        if scale > 1e-3:
            assert float((u.float() - v.float()).abs().max()) <= 1e-2 * scale + 1e-2, scale


@pytest.mark.parametrize("case", [(8, 64, 14, 14, 128, 3, 3, 1, 1), (4, 64, 28, 28, 256, 1, 1, 1, 0),
                                  (2, 3, 32, 32, 64, 7, 7, 2, 3)])
def test_conv_stats_shifted_partials(case):
    """Shifted statistics partials Σ(y−K), Σ(y−K)² (K = a per-channel shift such as the BN running
    mean) against the fp32 convolution; and the BN built on them recovers mean/variance of a
    large-mean output where raw Σy² − (Σy)²/M would cancel."""
    _native()
    from bigdl.ops import native_ops as NO
    n, c, h, w, k, r, s, st, pd = case
    x = _cl((torch.randn(n, c, h, w, device=dev) + 3.0).bfloat16())
    w4 = _cl((torch.randn(k, c, r, s, device=dev) * 0.05 + 0.02).bfloat16())
    ref = _conv_ref(x, w4, (st, st), (pd, pd)).double()
    K = ref.mean((0, 2, 3)).float() + 0.1 * torch.randn(k, device=dev)
    y, part, G = NO.conv2d_forward_stats(x, w4, None, (st, st), (pd, pd), shift=K)
    s1 = part.view(2, G, k).double().sum(1)
    d = ref - K.double().view(1, k, 1, 1)
    torch.testing.assert_close(s1[0], d.sum((0, 2, 3)), rtol=1e-3, atol=1e-1)
    torch.testing.assert_close(s1[1], (d * d).sum((0, 2, 3)), rtol=1e-3, atol=1e-1)
    g = torch.ones(k, device=dev)
    b = torch.zeros(k, device=dev)
    rm, rv = K.clone(), torch.ones(k, device=dev)
    out, mean, invstd = NO.batchnorm_forward_train_partials(y, part, G, g, b, rm, rv, 0.1, 1e-5, shift=K)
    torch.testing.assert_close(mean.double(), ref.mean((0, 2, 3)), rtol=1e-4, atol=1e-3)
    var = ref.var((0, 2, 3), unbiased=False)
    torch.testing.assert_close((1.0 / invstd.double() ** 2 - 1e-5), var, rtol=2e-3, atol=1e-4)


@pytest.mark.parametrize("groups,C,K,st,R", [(2, 32, 64, 1, 3), (4, 32, 32, 2, 3), (2, 16, 16, 1, 1), (8, 64, 64, 1, 3)])
def test_grouped_conv_native(groups, C, K, st, R):
    """Grouped convolution (reference nGroup) on the native kernels, one launch per group, vs the
    fp32 torch grouped conv; no torch fallback."""
    N = _native()
    from bigdl.ops import native_ops as NO
    from bigdl.ops import native
    native.reset_fallbacks()
    pd = R // 2
    x = _cl(torch.randn(4, C, 12, 12, device=dev).bfloat16())
    w4 = (torch.randn(K, C // groups, R, R, device=dev) * 0.1).bfloat16()
    b = torch.randn(K, device=dev)
    y = NO.conv2d_forward(x, w4, b, (st, st), (pd, pd), groups=groups)
    assert y is not NotImplemented
    ref = torch.nn.functional.conv2d(x.float(), w4.float(), b, (st, st), (pd, pd), groups=groups)
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=3e-2)
    gy = _cl(torch.randn_like(ref).bfloat16())
    gw = torch.zeros(K, C // groups, R, R, device=dev)
    gb = torch.zeros(K, device=dev)
    gi = NO.conv2d_backward(gy, x, w4, (st, st), (pd, pd), groups=groups, need_input=True, gw_acc=gw, gb_acc=gb)
    assert gi is not NotImplemented
    xr = x.float().requires_grad_(True)
    wr = w4.float().requires_grad_(True)
    out = torch.nn.functional.conv2d(xr, wr, None, (st, st), (pd, pd), groups=groups)
    out.backward(gy.float())
    torch.testing.assert_close(gi.float(), xr.grad, rtol=2e-2, atol=5e-2)
    torch.testing.assert_close(gw, wr.grad, rtol=2e-2, atol=5e-2 * float(wr.grad.abs().max()))
    torch.testing.assert_close(gb, gy.float().sum((0, 2, 3)), rtol=1e-2, atol=1e-1)
    assert not any(k[0].startswith("conv") for k in native.fallback_counts()), native.fallback_counts()


@pytest.mark.parametrize("C,R,st,dil", [(32, 3, 1, 1), (64, 3, 2, 1), (16, 5, 1, 1), (48, 3, 1, 2), (24, 1, 1, 1)])
def test_depthwise_conv_native(C, R, st, dil):
    """Depthwise convolution (groups == C == K) on the stencil kernels vs torch fp32."""
    _native()
    from bigdl.ops import native_ops as NO
    from bigdl.ops import native
    native.reset_fallbacks()
    pd = dil * (R // 2)
    x = _cl(torch.randn(4, C, 15, 17, device=dev).bfloat16())
    w4 = (torch.randn(C, 1, R, R, device=dev) * 0.3).bfloat16()
    b = torch.randn(C, device=dev)
    y = NO.conv2d_forward(x, w4, b, (st, st), (pd, pd), (dil, dil), groups=C)
    assert y is not NotImplemented
    xr = x.float().requires_grad_(True)
    wr = w4.float().requires_grad_(True)
    ref = torch.nn.functional.conv2d(xr, wr, b, (st, st), (pd, pd), (dil, dil), groups=C)
    torch.testing.assert_close(y.float(), ref.detach(), rtol=2e-2, atol=3e-2)
    gy = _cl(torch.randn_like(ref).bfloat16())
    ref.backward(gy.float())
    gw = torch.zeros(C, 1, R, R, device=dev)
    gb = torch.zeros(C, device=dev)
    gi = NO.conv2d_backward(gy, x, w4, (st, st), (pd, pd), (dil, dil), groups=C, need_input=True, gw_acc=gw, gb_acc=gb)
    torch.testing.assert_close(gi.float(), xr.grad, rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(gw, wr.grad, rtol=1e-2, atol=1e-2 * float(wr.grad.abs().max()))
    assert not any(k[0].startswith("conv") for k in native.fallback_counts())


@pytest.mark.parametrize("shape,k,s,p,ceil", [((4, 64, 28, 28), 3, 1, 1, False), ((2, 192, 56, 56), 3, 2, 0, True),
                                              ((3, 16, 13, 11), 2, 2, 0, False), ((2, 8, 9, 9), 5, 1, 2, False)])
def test_maxpool_inference_rows_kernel(shape, k, s, p, ceil):
    """Inference max-pool (no argmax, row-reuse kernel) vs torch."""
    _native()
    from bigdl.ops import native_ops as NO
    x = _cl(torch.randn(shape, device=dev).bfloat16())
    y, idx = NO.maxpool2d_forward(x, (k, k), (s, s), (p, p), ceil, need_indices=False)
    assert idx is None
    ref = torch.nn.functional.max_pool2d(x.float(), k, s, p, 1, ceil)
    assert torch.equal(y.float(), ref)


@pytest.mark.parametrize("Cin,Cout,R,st,pd,adj", [(32, 16, 3, 1, 1, 0), (16, 32, 4, 2, 1, 0), (64, 32, 3, 2, 1, 1),
                                                  (32, 32, 2, 2, 0, 0)])
def test_transposed_conv_native(Cin, Cout, R, st, pd, adj):
    """SpatialFullConvolution's math (transposed conv) on the conv kernels: forward = conv dgrad,
    backward-data = conv forward, weight gradient = conv wgrad with roles exchanged — vs torch."""
    _native()
    from bigdl.ops import native_ops as NO
    x = _cl(torch.randn(3, Cin, 9, 11, device=dev).bfloat16())
    w = (torch.randn(Cin, Cout, R, R, device=dev) * 0.1).requires_grad_(True)
    b = torch.randn(Cout, device=dev).requires_grad_(True)
    xg = x.detach().requires_grad_(True)
    y = NO.conv_transpose2d(xg, w, b, (st, st), (pd, pd), (adj, adj))
    assert y is not NotImplemented
    xr = x.float().requires_grad_(True)
    wr = w.detach().bfloat16().float().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True)
    ref = torch.nn.functional.conv_transpose2d(xr, wr, br, st, pd, adj)
    torch.testing.assert_close(y.float(), ref.detach(), rtol=2e-2, atol=3e-2)
    gy = torch.randn_like(ref)
    y.float().backward(gy)
    ref.backward(gy)
    torch.testing.assert_close(xg.grad.float(), xr.grad, rtol=3e-2, atol=5e-2)
    torch.testing.assert_close(w.grad, wr.grad, rtol=3e-2, atol=3e-2 * float(wr.grad.abs().max()))
    # the output is bf16, so the incoming gradient is bf16-rounded before the bias sum
    torch.testing.assert_close(b.grad, gy.bfloat16().float().sum((0, 2, 3)), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("K,taps,C,cp,ldw", [(64, 49, 3, 4, 200), (16, 9, 5, 8, 72), (32, 1, 3, 8, 8)])
def test_pad_taps(K, taps, C, cp, ldw):
    """Narrow-channel conv weights padded per tap and per row in one native pass (the stem's C4
    operand) == the zero-fill + strided-copy construction."""
    _native()
    from bigdl.ops import native_ops as NO
    wk = torch.randn(K, taps, C, device=dev).bfloat16()
    got = NO._pad_taps(wk, K, taps, C, cp, ldw)
    ref = torch.zeros(K, ldw, dtype=torch.bfloat16, device=dev)
    ref[:, :taps * cp].view(K, taps, cp)[..., :C] = wk
    assert torch.equal(got, ref)
