"""The persistent halo-patch 3×3 conv (ops/csrc/conv_patch.hip: 64 → 64 channels, stride 1, pad 1 —
the filter resident in the LDS, each input pixel staged once per tile instead of once per tap)
against an fp32 PyTorch reference of the same bf16 operands: forward with bias + ReLU, residual,
BN-statistics partials, and the data gradient (the same kernel with the flipped filter), on image
sizes whose 128-pixel tiles cross image rows and image boundaries."""
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"

SHAPES = [(2, 56, 56), (3, 14, 14), (2, 13, 17), (1, 28, 28), (5, 9, 8)]


@pytest.fixture(autouse=True)
def _patch_on():
    """The kernel is opt-in (slower than the implicit GEMM inside the training step): switch it on."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from bigdl.ops import native_ops as NO
    old = NO._lib().bigdl_conv_patch_enable(1)
    yield
    NO._lib().bigdl_conv_patch_enable(old)


def _native():
    from bigdl.ops import native_status
    st = native_status()
    assert st["loaded"], st
    from bigdl.ops import native_ops as NO
    return NO


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("shape", SHAPES)
def test_patch_forward_bias_relu_residual(shape):
    NO = _native()
    n, h, w = shape
    x = _cl(torch.randn(n, 64, h, w, device=dev).bfloat16())
    w4 = _cl(torch.randn(64, 64, 3, 3, device=dev).bfloat16() * 0.05)
    b = torch.randn(64, device=dev)
    ref = torch.nn.functional.conv2d(x.float(), w4.float(), None, 1, 1)
    y = NO.conv2d_forward(x, w4, b, (1, 1), (1, 1), relu=True)
    assert y is not NotImplemented
    torch.testing.assert_close(y.float(), torch.relu(ref + b.view(1, -1, 1, 1)), rtol=2e-2, atol=2e-2)
    res = _cl(torch.randn_like(ref).bfloat16())
    y2 = NO._conv_fwd_impl(x, w4, None, (1, 1), (1, 1), res=res)
    torch.testing.assert_close(y2.float(), ref + res.float(), rtol=2e-2, atol=3e-2)


@pytest.mark.parametrize("shape", SHAPES)
def test_patch_forward_stats(shape):
    NO = _native()
    n, h, w = shape
    x = _cl(torch.randn(n, 64, h, w, device=dev).bfloat16())
    w4 = _cl(torch.randn(64, 64, 3, 3, device=dev).bfloat16() * 0.05)
    shift = torch.randn(64, device=dev) * 0.1
    ref = torch.nn.functional.conv2d(x.float(), w4.float(), None, 1, 1)
    y, part, G = NO.conv2d_forward_stats(x, w4, None, (1, 1), (1, 1), shift=shift)
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)
    yb = y.float() - shift.view(1, -1, 1, 1)
    s1 = part.view(2, G, 64).sum(1)
    torch.testing.assert_close(s1[0], yb.sum((0, 2, 3)), rtol=1e-3, atol=2e-2)
    torch.testing.assert_close(s1[1], (yb * yb).sum((0, 2, 3)), rtol=1e-3, atol=2e-2)


@pytest.mark.parametrize("shape", SHAPES[:3])
def test_patch_data_gradient(shape):
    NO = _native()
    n, h, w = shape
    x = _cl(torch.randn(n, 64, h, w, device=dev).bfloat16())
    w4 = _cl(torch.randn(64, 64, 3, 3, device=dev).bfloat16() * 0.05)
    gy = _cl(torch.randn(n, 64, h, w, device=dev).bfloat16())
    gx = NO.conv2d_backward(gy, x, w4, (1, 1), (1, 1), need_input=True)
    gx = gx[0] if isinstance(gx, tuple) else gx
    xr = x.float().requires_grad_(True)
    torch.nn.functional.conv2d(xr, w4.float(), None, 1, 1).backward(gy.float())
    torch.testing.assert_close(gx.float(), xr.grad, rtol=2e-2, atol=3e-2)


def test_patch_matches_igemm_family():
    """The same launch with the kernel switched off (the implicit-GEMM family): both accumulate in
    fp32, so the bf16 outputs agree to rounding."""
    NO = _native()
    x = _cl(torch.randn(2, 64, 56, 56, device=dev).bfloat16())
    w4 = _cl(torch.randn(64, 64, 3, 3, device=dev).bfloat16() * 0.05)
    y = NO.conv2d_forward(x, w4, None, (1, 1), (1, 1))
    NO._lib().bigdl_conv_patch_enable(0)
    y0 = NO.conv2d_forward(x, w4, None, (1, 1), (1, 1))
    NO._lib().bigdl_conv_patch_enable(1)
    torch.testing.assert_close(y.float(), y0.float(), rtol=1e-2, atol=1e-2)
