"""int8 implicit-GEMM convolution (ops/csrc/conv_i8.hip) for quantized inference.

* Kernel exactness: the per-image quantisation is reproduced on the host and the int8 products are
  summed in fp64 — the kernel must match to bf16 output rounding (the int32 accumulation is exact).
* Accuracy vs fp32 (the verdict's cosine > 0.99): VGG16 and ResNet-50 layer shapes, the quantized
  SpatialConvolution layer, and a whole quantized VGG16 forward.
Reference: DL/nn/quantized/SpatialConvolution.scala:163-208 (ConvDataInit + MixPrecisionGEMM)."""
import pytest
import os
import sys

import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = "cuda"

SHAPES = [  # N, C, H, K, R, stride, pad, dilation
    (2, 64, 28, 64, 3, 1, 1, 1),      # VGG conv1_2 / conv2_1 class: two taps per k-tile
    (2, 64, 30, 128, 3, 1, 1, 1),
    (2, 128, 14, 256, 3, 1, 1, 1),    # one tap per k-tile
    (2, 256, 14, 256, 3, 2, 1, 1),
    (1, 512, 7, 512, 3, 1, 1, 1),
    (2, 256, 14, 64, 1, 1, 0, 1),     # ResNet-50 pointwise
    (2, 1024, 14, 256, 1, 1, 0, 1),
    (2, 512, 14, 1024, 1, 2, 0, 1),
    (3, 64, 17, 72, 3, 1, 2, 2),      # dilated, M and K tails
    (2, 64, 9, 64, 5, 1, 2, 1),       # R·S = 25: odd tap count → half-empty last k-tile
    (2, 480, 14, 192, 1, 1, 0, 1),    # C % 128 != 0 (Inception concats): partial last k-tile per tap
    (2, 528, 14, 160, 1, 1, 0, 1),
    (2, 832, 7, 384, 1, 1, 0, 1),
    (2, 96, 15, 128, 3, 1, 1, 1),     # … and with padded taps
    (2, 16, 12, 32, 5, 1, 2, 1),
    (2, 64, 28, 256, 1, 1, 0, 1),     # short reductions (≤ 2 k-tiles): 128 × 128 tiles, 2-deep ring
    (2, 128, 14, 512, 1, 1, 0, 1),
    (3, 256, 14, 520, 1, 2, 0, 1),    # … strided, K tail
]


def _native():
    from bigdl.ops import native_status
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert native_status()["loaded"]
    from bigdl.ops import native_ops as NO, reference as R
    return NO, R


def _cos(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return float(a @ b / (a.norm() * b.norm()))


@pytest.mark.parametrize("shape", SHAPES)
def test_conv_i8_exact_and_accurate(shape):
    NO, R = _native()
    N, C, H, K, Rk, st, pd, dl = shape
    torch.manual_seed(C + K + H)
    x = torch.relu(torch.randn(N, C, H, H, device=dev)).bfloat16().contiguous(memory_format=torch.channels_last)
    w = torch.randn(K, C, Rk, Rk, device=dev) * 0.05
    b = torch.randn(K, device=dev)
    qw, sw = R.quant_rows(w.reshape(K, -1).float())
    wq, ldw = NO.conv_i8_weight(qw, K, C, Rk, Rk)
    P = (H + 2 * pd - dl * (Rk - 1) - 1) // st + 1
    y = NO.conv2d_i8_forward(x, wq, ldw, sw.float(), b, K, Rk, Rk, (st, st), (pd, pd), (dl, dl), (P, P))
    assert y is not NotImplemented
    # host emulation of the same quantisation: scale amax/127 per image, round-to-nearest-even
    amax = x.float().abs().amax(dim=(1, 2, 3))
    sx = torch.where(amax > 0, amax / 127.0, torch.ones_like(amax))
    xq = torch.clamp(torch.round(x.float() / sx.view(-1, 1, 1, 1)), -127, 127)
    wqf = qw[:, :C * Rk * Rk].double().reshape(K, C, Rk, Rk)
    acc = F.conv2d(xq.double(), wqf, None, st, pd, dl)
    ref = acc * sx.double().view(-1, 1, 1, 1) * sw.double().view(1, -1, 1, 1) + b.double().view(1, -1, 1, 1)
    torch.testing.assert_close(y.double(), ref, rtol=1e-2, atol=1e-2 * float(ref.abs().max()))
    f32 = F.conv2d(x.float(), w, b, st, pd, dl)
    assert _cos(y.float(), f32) > 0.99


def test_quantized_layer_native_path_vs_float():
    NO, R = _native()
    from bigdl import nn
    from bigdl.nn import quantized as Q
    torch.manual_seed(1)
    conv = nn.SpatialConvolution(128, 256, 3, 3, 1, 1, 1, 1)
    conv.evaluate()
    x = torch.relu(torch.randn(4, 128, 20, 20))
    y = conv.forward(x).clone()
    q = Q.SpatialConvolution.from_float(conv).cuda()
    called = {}
    orig = NO.conv2d_i8_forward

    def spy(*a, **k):
        called["n"] = called.get("n", 0) + 1
        return orig(*a, **k)
    NO.conv2d_i8_forward = spy
    try:
        yq = q.forward(x.cuda())
    finally:
        NO.conv2d_i8_forward = orig
    assert called.get("n") == 1  # the int8 kernel ran, not the unfold path
    assert _cos(yq.float().cpu(), y) > 0.99


def test_quantized_vgg16_forward_vs_fp32():
    """VGG16 quantized end to end on the int8 kernels: against the host int8 path (the same
    quantisation semantics — one symmetric activation scale per image, per-channel weight scales)
    and against fp32 (what int8 costs in accuracy: the per-image
    scales compound over 13 convs + 3 FCs; the host path measures 0.974 on this net)."""
    _native()
    from bigdl.models.vgg import Vgg_16
    from bigdl.utils.engine import Engine
    Engine.init(device="cuda:0")
    torch.manual_seed(0)
    m = Vgg_16(1000, has_dropout=False)
    m.evaluate()
    x = torch.randn(4, 3, 224, 224)
    # data-dependent init (tools/bench_configs.py:_lsuv): without it a random-init VGG16's log-probs
    # are one image-independent vector and any comparison of them passes trivially
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from bench_configs import _lsuv
    _lsuv(m, x)
    q = m.quantize()
    with torch.no_grad():
        ref = m.forward(x).float().clone()
        host = q.forward(x).float().clone()
        yq = q.cuda().forward(x.cuda()).float().cpu()
    r = lambda t: t - t.mean(1, keepdim=True)  # noqa: E731 - log-probs → centred logits
    assert float((r(ref) - r(ref).mean(0)).std()) > 0.1  # the logits do carry image-dependent signal
    # the kernels see bf16 activations (the host path fp32): that rounding alone moves the centred
    # logits as much as int8 does, so both comparisons carry the same tolerance
    assert _cos(r(yq), r(host)) > 0.95
    assert _cos(r(yq), r(ref)) > 0.95


@pytest.mark.gpu
@pytest.mark.parametrize("k,s,p,H,u8", [(3, 2, 0, 15, False), (3, 2, 1, 14, True), (2, 2, 0, 16, False),
                                        (3, 1, 1, 9, True), (3, 2, 0, 112, True)])
def test_maxpool_i8_matches_torch(k, s, p, H, u8):
    """int8 max pooling (fixed-window kernels for 3x3 / 2x2, ceil-mode output sizes as Caffe's) against
    torch's max pool of the same codes; the unsigned (offset) code keeps its padding tail."""
    import math
    from bigdl.ops import native_ops as NO
    torch.manual_seed(3)
    N, C = 2, 48
    P = int(math.ceil((H + 2 * p - k) / s)) + 1
    if p > 0 and (P - 1) * s >= H + p:
        P -= 1
    codes = torch.randint(-128, 128, (N, C, H, H), dtype=torch.int8, device="cuda")
    if u8:
        x = NO._i8_act(N, C, H, H, "cuda", True)
        x.copy_(codes)
        x.untyped_storage()[x.numel():].fill_(0x80)
        x = NO._tag(x, 0.1, True)
    else:
        x = NO._tag(codes.contiguous(memory_format=torch.channels_last), 0.1, False)
    y = NO.maxpool_i8(x, k, k, s, s, p, p, P, P)
    assert y is not NotImplemented
    ref = torch.nn.functional.max_pool2d(codes.float(), k, s, p, ceil_mode=True)[:, :, :P, :P]
    assert torch.equal(y.float(), ref)
    if u8:
        raw = torch.empty(0, dtype=torch.uint8, device="cuda").set_(y.untyped_storage())
        assert bool((raw[y.numel():y.numel() + 16] == 0x80).all())


@pytest.mark.gpu
@pytest.mark.parametrize("K,res", [(256, False), (256, True), (64, False)])
def test_i8_pixel_pair_path_matches_plain(K, res):
    """64-channel 1×1 int8 convs run as the GEMM of pixel pairs with a block-diagonal weight: the same
    int32 sums, so the codes match the plain 64-channel k-tile path exactly (with and without the
    int8 residual of a block tail)."""
    import bigdl.nn as nn
    from bigdl.nn.quantized import layers as Q
    from bigdl.ops import native_ops as NO
    torch.manual_seed(5)
    conv = nn.SpatialConvolution(64, K, 1, 1)
    q = Q.SpatialConvolution.from_float(conv).cuda()
    q.static_scale = 0.05
    q._out_qscale, q._out_u8, q._relu_fused = 0.04, True, True
    N, H = 4, 14
    xc = NO._i8_act(N, 64, H, H, "cuda", True)
    xc.copy_(torch.randint(-128, 128, (N, 64, H, H), dtype=torch.int8, device="cuda"))
    xc.untyped_storage()[xc.numel():].fill_(0x80)
    x = NO._tag(xc, 0.05, True)
    r = None
    if res:
        rc = torch.randint(-128, 128, (N, K, H, H), dtype=torch.int8, device="cuda").contiguous(memory_format=torch.channels_last)
        r = NO._tag(rc, 0.03, True)
    assert q._pair_ok(x, (0, 0, 0, 0), r)
    if res:
        y1 = q.forward_residual(x, r, out_scale=0.04, out_u8=True)
    else:
        y1 = q._native_static(x, (0, 0, 0, 0))
    q._pair_ok = lambda *a, **k: False
    if res:
        y0 = q.forward_residual(x, r, out_scale=0.04, out_u8=True)
    else:
        y0 = q._native_static(x, (0, 0, 0, 0))
    torch.cuda.synchronize()
    assert y1.shape == y0.shape and y1._qscale == y0._qscale and y1._qzero == y0._qzero
    assert torch.equal(y1.contiguous(), y0.contiguous())
