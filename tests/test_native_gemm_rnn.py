"""Numerics of the round-2 HIP kernels vs plain fp32 torch references of the same ops:
MFMA GEMM (gemm.hip) with its epilogues, transpose / column sums, the Linear layer on them,
softmax (K12), avg-pool (K11), embedding gather / scatter-add (K16) and the fused recurrent
step (rnn_step.hip: LSTM K14, GRU K15) through ``Recurrent``.

Every test also asserts that no device op fell back to the torch reference."""
import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = "cuda"
bf = torch.bfloat16


@pytest.fixture(autouse=True)
def _no_fallback():
    from bigdl import ops
    st = ops.native_status()
    assert st["loaded"], st
    ops.reset_fallbacks()
    yield
    assert ops.fallback_counts() == {}, ops.fallback_counts()


def _NO():
    from bigdl.ops import native_ops
    return native_ops


@pytest.mark.parametrize("M,N,K", [(1, 4, 8), (20, 800, 200), (37, 100, 72), (400, 10000, 200), (1024, 1024, 1024),
                                   (513, 260, 136)])
@pytest.mark.parametrize("act", [0, 1])
def test_gemm_bf16_out(M, N, K, act):
    NO = _NO()
    a = torch.randn(M, K, device=dev).to(bf)
    b = torch.randn(N, K, device=dev).to(bf)
    bias = torch.randn(N, device=dev)
    y = NO.gemm(a, b, bias, act=act)
    ref = a.float() @ b.float().t() + bias
    if act:
        ref = torch.relu(ref)
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2 * float(ref.abs().max()) / 10 + 1e-2)


def test_gemm_fp32_accumulate_strided_and_addend():
    NO = _NO()
    M, N, K = 70, 96, 48
    big = torch.randn(M, 3 * K, device=dev).to(bf)
    a = big[:, K:2 * K]  # strided view (row stride 3K)
    b = torch.randn(N, K, device=dev).to(bf)
    d = torch.randn(M, N, device=dev).to(bf)
    c = torch.randn(M, N, device=dev)
    c0 = c.clone()
    NO.gemm(a, b, None, out=c, d=d, alpha=0.5, beta=2.0)
    ref = 0.5 * (a.float() @ b.float().t()) + d.float() + 2.0 * c0
    torch.testing.assert_close(c, ref, rtol=1e-2, atol=5e-2)


@pytest.mark.parametrize("M,N,K", [(128, 4096, 25088), (128, 1000, 4096), (37, 100, 2056), (3, 12, 8192)])
@pytest.mark.parametrize("act", [0, 1])
def test_gemm_split_k(M, N, K, act):
    """Small-M, long-K GEMMs take the split-K path (fp32 partial slabs summed by the epilogue kernel)."""
    NO = _NO()
    assert NO._gemm_splits(M, N, K) > 1
    a = torch.randn(M, K, device=dev).to(bf)
    b = (torch.randn(N, K, device=dev) * 0.05).to(bf)
    bias = torch.randn(N, device=dev)
    y = NO.gemm(a, b, bias, act=act)
    ref = a.float() @ b.float().t() + bias
    if act:
        ref = torch.relu(ref)
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2 * float(ref.abs().max()) / 10 + 1e-2)
    # fp32 output with addend and beta through the split epilogue
    d = torch.randn(M, N, device=dev).to(bf)
    c = torch.randn(M, N, device=dev)
    c0 = c.clone()
    NO.gemm(a, b, None, out=c, d=d, alpha=0.5, beta=2.0)
    ref2 = 0.5 * (a.float() @ b.float().t()) + d.float() + 2.0 * c0
    torch.testing.assert_close(c, ref2, rtol=1e-2, atol=5e-2 * float(ref2.abs().max()) / 10 + 5e-2)


def test_transpose_and_colsum():
    NO = _NO()
    x = torch.randn(130, 72, device=dev).to(bf)
    torch.testing.assert_close(NO.transpose_bf16(x), x.t().contiguous(), rtol=0, atol=0)
    out = torch.ones(72, device=dev)
    NO.colsum_acc(x, out, 0.5)
    torch.testing.assert_close(out, 1 + 0.5 * x.float().sum(0), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("M,IN,OUT", [(64, 200, 800), (400, 200, 10000), (8, 16, 24)])
def test_linear_layer_native_vs_fp32(M, IN, OUT):
    from bigdl.nn import Linear
    from bigdl.utils.engine import Engine
    Engine.init(device="cuda:0")
    lin = Linear(IN, OUT)
    cpu = copy.deepcopy(lin)
    lin = lin.cuda() if hasattr(lin, "cuda") else lin.to(dev)
    x = torch.randn(M, IN)
    y = lin.forward(x.to(dev))
    yr = cpu.forward(x)
    torch.testing.assert_close(y.float().cpu(), yr, rtol=3e-2, atol=3e-2)
    gy = torch.randn(M, OUT)
    gi = lin.backward(x.to(dev), gy.to(dev))
    gir = cpu.backward(x, gy)
    torch.testing.assert_close(gi.float().cpu(), gir, rtol=3e-2, atol=5e-2)
    (gw, gb), (gwr, gbr) = lin.parameters()[1], cpu.parameters()[1]
    torch.testing.assert_close(gw.float().cpu(), gwr, rtol=3e-2, atol=3e-2 * float(gwr.abs().max()))
    torch.testing.assert_close(gb.float().cpu(), gbr, rtol=3e-2, atol=3e-2 * float(gbr.abs().max()))


@pytest.mark.parametrize("shape", [(16, 10), (3, 1000), (7, 33)])
@pytest.mark.parametrize("dtype", [bf, torch.float32])
def test_softmax_rows(shape, dtype):
    NO = _NO()
    x = (torch.randn(*shape, device=dev) * 3).to(dtype)
    y = NO.softmax_forward(x)
    ref = torch.softmax(x.float(), -1)
    tol = 1e-2 if dtype == bf else 1e-5
    torch.testing.assert_close(y.float(), ref, rtol=tol, atol=tol)
    gy = torch.randn(*shape, device=dev).to(dtype)
    gx = NO.softmax_backward(gy, y)
    gref = ref * (gy.float() - (gy.float() * ref).sum(-1, keepdim=True))
    torch.testing.assert_close(gx.float(), gref, rtol=3 * tol, atol=3 * tol)


def test_softmax_layer_channels_nhwc():
    from bigdl.nn import SoftMax
    m = SoftMax()
    x = torch.randn(2, 16, 5, 5, device=dev).to(bf).contiguous(memory_format=torch.channels_last)
    y = m.forward(x)
    ref = torch.softmax(x.float(), 1)
    torch.testing.assert_close(y.float(), ref, rtol=1e-2, atol=1e-2)
    gy = torch.randn_like(x)
    gx = m.backward(x, gy)
    gref = ref * (gy.float() - (gy.float() * ref).sum(1, keepdim=True))
    torch.testing.assert_close(gx.float(), gref, rtol=3e-2, atol=3e-2)


AVG_CASES = [
    # (N, C, H, W, k, s, p, ceil, count_include_pad, divisor)
    (4, 64, 7, 7, (7, 7), (1, 1), (0, 0), False, True, None),  # global (ResNet head)
    (2, 32, 14, 14, (3, 3), (1, 1), (1, 1), False, True, None),
    (2, 32, 14, 14, (3, 3), (1, 1), (1, 1), False, False, None),
    (2, 16, 15, 15, (3, 3), (2, 2), (1, 1), True, True, None),
    (2, 16, 15, 13, (2, 2), (2, 2), (0, 0), True, False, None),
    (1, 8, 9, 9, (5, 5), (3, 3), (2, 2), False, True, 7),
]


@pytest.mark.parametrize("case", AVG_CASES)
def test_avgpool_native(case):
    NO = _NO()
    n, c, h, w, k, s, p, ceil, cip, div = case
    x = torch.randn(n, c, h, w, device=dev).to(bf).contiguous(memory_format=torch.channels_last)
    y = NO.avgpool2d_forward(x, k, s, p, ceil, cip, div)
    assert y is not NotImplemented
    # fp32 oracle on the host (contiguous NCHW): ROCm torch's channels-last avg_pool2d backward on
    # the device disagreed with it on the padded 3×3 cases
    xr = x.float().cpu().contiguous().requires_grad_(True)
    yr = F.avg_pool2d(xr, k, s, p, ceil, cip, div)
    torch.testing.assert_close(y.float().cpu(), yr, rtol=1e-2, atol=1e-2)
    gy = torch.randn(yr.shape).to(bf)
    gx = NO.avgpool2d_backward(gy.to(dev).contiguous(memory_format=torch.channels_last), x, k, s, p, ceil, cip, div)
    yr.backward(gy.float())
    torch.testing.assert_close(gx.float().cpu(), xr.grad, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("itype", [torch.float32, torch.int64, torch.int32])
@pytest.mark.parametrize("D,wdt", [(200, bf), (33, torch.float32), (64, torch.float32)])
def test_embedding_native(itype, D, wdt):
    NO = _NO()
    V = 50
    w = torch.randn(V, D, device=dev).to(wdt)
    idx = torch.randint(1, V + 1, (6, 7), device=dev)
    idx[0, 0] = 3  # padding value below
    idx = idx.to(itype)
    y = NO.embedding_forward(w, idx, 0)
    torch.testing.assert_close(y, w[idx.long() - 1], rtol=0, atol=0)
    gw = torch.zeros(V, D, device=dev)
    gy = torch.randn(6, 7, D, device=dev).to(wdt)
    NO.embedding_backward(gw, idx, gy, 0.5, 3)
    ref = torch.zeros(V, D, device=dev)
    keep = idx.reshape(-1).long() != 3
    ref.index_add_(0, (idx.reshape(-1).long() - 1)[keep], 0.5 * gy.reshape(-1, D).float()[keep])
    torch.testing.assert_close(gw, ref, rtol=1e-5, atol=1e-4)


def _rec_cmp(cell_fn, B=20, T=12, IN=48, H=64, tol=5e-2):
    from bigdl.nn import Recurrent
    torch.manual_seed(0)
    cpu = Recurrent().add(cell_fn(IN, H))
    gpu = copy.deepcopy(cpu).cuda()
    x = torch.randn(B, T, IN)
    y = cpu.forward(x)
    yg = gpu.forward(x.cuda())
    torch.testing.assert_close(yg.float().cpu(), y, rtol=tol, atol=tol)
    gy = torch.randn_like(y)
    gi = cpu.backward(x, gy)
    gig = gpu.backward(x.cuda(), gy.cuda())
    torch.testing.assert_close(gig.float().cpu(), gi, rtol=tol, atol=tol)
    for a, b in zip(gpu.parameters()[1], cpu.parameters()[1]):
        torch.testing.assert_close(a.float().cpu(), b, rtol=tol, atol=tol * float(b.abs().max()))
    return gpu


def test_recurrent_lstm_fused_step_vs_cpu():
    from bigdl.nn import LSTM
    g = _rec_cmp(LSTM)
    assert g._rec is None


def test_recurrent_gru_fused_step_vs_cpu():
    from bigdl.nn import GRU
    _rec_cmp(GRU)


def test_ptb_lstm_fused_inference_matches_train_forward():
    from bigdl.nn import LSTM, Recurrent
    rec = Recurrent().add(LSTM(32, 40)).cuda()
    x = torch.randn(4, 9, 32, device=dev)
    y_train = rec.forward(x).float()
    rec.evaluate()
    y_eval = rec.forward(x).float()
    torch.testing.assert_close(y_eval, y_train, rtol=0, atol=0)


@pytest.mark.parametrize("dtype", [bf, torch.float32])
@pytest.mark.parametrize("weighted,avg,pad", [(False, True, -1), (True, True, 3), (False, False, 2)])
def test_class_nll_native(dtype, weighted, avg, pad):
    from bigdl.ops import native_ops as NO, reference as R
    B, K = 37, 10
    lp = torch.log_softmax(torch.randn(B, K, device=dev), -1).to(dtype)
    t = (torch.randint(0, K, (B,), device=dev) + 1).float()
    w = torch.rand(K, device=dev) if weighted else None
    l = NO.class_nll_forward(lp, t, w, avg, pad)
    lr = R.class_nll_forward(lp, t, w, avg, pad)
    torch.testing.assert_close(l.float(), lr.float(), rtol=1e-4, atol=1e-4)
    g = NO.class_nll_backward(lp, t, w, avg, pad)
    gr = R.class_nll_backward(lp, t, w, avg, pad)
    torch.testing.assert_close(g.float(), gr.float(), rtol=1e-3, atol=1e-5)


@pytest.mark.parametrize("n", [22278, 5, 1024])
def test_sgd_adam_odd_lengths(n):
    from bigdl.ops import native_ops as NO, reference as R
    w = torch.randn(n, device=dev)
    g = torch.randn(n, device=dev)
    buf = torch.randn(n, device=dev)
    w2, buf2 = w.clone(), buf.clone()
    NO.sgd_step(w, g, buf, 0.1, 0.9, 0.0, 1e-4, True, False)
    R.sgd_step(w2, g, buf2, 0.1, 0.9, 0.0, 1e-4, True, False)
    torch.testing.assert_close(w, w2, rtol=1e-5, atol=1e-6)
    m, v = torch.zeros(n, device=dev), torch.zeros(n, device=dev)
    w3, m3, v3 = w.clone(), m.clone(), v.clone()
    NO.adam_step(w, g, m, v, 1e-3, 0.9, 0.999, 1e-8, 1)
    R.adam_step(w3, g, m3, v3, 1e-3, 0.9, 0.999, 1e-8, 1)
    torch.testing.assert_close(w, w3, rtol=1e-5, atol=1e-6)
