"""The 8-wave 32x32x16 / LDS-DMA conv family (ops/csrc/conv_mfma32.hip) against an fp32 PyTorch
reference of the same bf16 operands: every instantiated tile, both gathers (tap-uniform 3x3 / 5x5 /
dilated, pointwise stride 1 and 2), row (M) and channel (K) tails, bias + ReLU, residual and
shifted BN-statistics partials.  The tile is pinned per geometry
through the kernel-selection table, the same path the compile phase uses."""
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"

X8_TILES = [(128, 1, 128), (64, 1, 256), (128, 1, 256), (256, 1, 256)]

CASES = [  # N, C, H, W, K, R, S, stride, pad, dilation
    (2, 64, 14, 14, 128, 3, 3, 1, 1, 1),
    (3, 128, 15, 13, 96, 3, 3, 1, 1, 1),     # odd spatial, M tail, K tail vs BN 128
    (2, 128, 16, 16, 128, 3, 3, 2, 1, 1),    # strided 3x3
    (2, 64, 12, 12, 64, 3, 3, 1, 2, 2),      # dilated
    (2, 64, 11, 11, 72, 5, 5, 1, 2, 1),      # 5x5, K tail not a multiple of 64
    (4, 256, 14, 14, 256, 1, 1, 1, 0, 1),    # pointwise, direct rows
    (2, 256, 14, 14, 512, 1, 1, 2, 0, 1),    # pointwise stride 2
    (1, 512, 7, 7, 2048, 1, 1, 1, 0, 1),     # deep pointwise, M < one tile
]


def _native():
    from bigdl.ops import native_status
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    st = native_status()
    assert st["loaded"], st
    from bigdl.ops import native_ops as NO
    return NO


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def _key(x, w4, st, pd, dl):
    N, C, H, W = x.shape
    K, _, R, S = w4.shape
    return (N, H, W, C, K, R, S, (st, st), (pd, pd), (dl, dl))


def _ref(x, w4, st, pd, dl):
    return torch.nn.functional.conv2d(x.float(), w4.float(), None, st, pd, dl)


@pytest.mark.parametrize("tile", X8_TILES)
@pytest.mark.parametrize("case", CASES)
def test_x8_forward_bias_relu(case, tile):
    NO = _native()
    n, c, h, w, k, r, s, st, pd, dl = case
    x = _cl(torch.randn(n, c, h, w, device=dev).bfloat16())
    w4 = _cl(torch.randn(k, c, r, s, device=dev).bfloat16() * 0.05)
    b = torch.randn(k, device=dev)
    key = _key(x, w4, st, pd, dl)
    NO._TILE["table"][key] = tile
    try:
        y = NO.conv2d_forward(x, w4, b, (st, st), (pd, pd), (dl, dl), relu=True)
    finally:
        NO._TILE["table"].pop(key, None)
    assert y is not NotImplemented
    ref = torch.relu(_ref(x, w4, st, pd, dl) + b.view(1, -1, 1, 1))
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("tile", X8_TILES)
@pytest.mark.parametrize("case", [c for c in CASES if c[9] == 1 and c[4] % 8 == 0])
def test_x8_stats_and_residual(case, tile):
    NO = _native()
    n, c, h, w, k, r, s, st, pd, dl = case
    x = _cl(torch.randn(n, c, h, w, device=dev).bfloat16())
    w4 = _cl(torch.randn(k, c, r, s, device=dev).bfloat16() * 0.05)
    key = _key(x, w4, st, pd, dl)
    ref = _ref(x, w4, st, pd, dl)
    shift = torch.randn(k, device=dev) * 0.1
    NO._TILE["table"][key] = tile
    try:
        y, part, G = NO.conv2d_forward_stats(x, w4, None, (st, st), (pd, pd), shift=shift)
        res = _cl(torch.randn_like(ref).bfloat16())
        y2 = NO._conv_fwd_impl(x, w4, None, (st, st), (pd, pd), res=res)
    finally:
        NO._TILE["table"].pop(key, None)
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)
    # partials of the stored (bf16) values minus the shift
    yb = y.float() - shift.view(1, -1, 1, 1)
    s1 = part.view(2, G, k).sum(1)
    torch.testing.assert_close(s1[0], yb.sum((0, 2, 3)), rtol=1e-3, atol=2e-2)
    torch.testing.assert_close(s1[1], (yb * yb).sum((0, 2, 3)), rtol=1e-3, atol=2e-2)
    torch.testing.assert_close(y2.float(), ref + res.float(), rtol=2e-2, atol=3e-2)


def test_x8_tile_validation():
    NO = _native()
    lib = NO._lib()
    for t in X8_TILES:
        assert lib.bigdl_conv_tile_ok(*t) == 0
    assert lib.bigdl_conv_tile_ok(64, 1, 128) != 0
    assert lib.bigdl_conv_tile_ok(32, 1, 256) != 0
