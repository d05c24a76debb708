"""ResizeBilinear with the reference's TensorFlow-style sampling (``nn/ResizeBilinear.scala:266-284,
406-412``: src = dst·in/out, lower = ⌊src⌋, upper = min(lower+1, in−1), no half-pixel offset), checked
against the expected tensors of the reference's ``ResizeBilinearSpec.scala`` (double height / double
width, NHWC), alignCorners, NCHW/NHWC agreement and gradients; the native NHWC kernels
(``resize.hip``) against the same math on the GPU."""
import pytest
import torch

X = [[[[1, 2, 3], [4, 5, 6]], [[7, 8, 9], [2, 3, 1]], [[4, 8, 2], [5, 3, 0]]]]


def test_reference_spec_double_height_and_width():
    from bigdl.nn import ResizeBilinear
    x = torch.tensor(X, dtype=torch.float32)
    assert ResizeBilinear(3, 2, data_format="NHWC").forward(x).tolist() == X
    exp_h = [[[1, 2, 3], [4, 5, 6]], [[4, 5, 6], [3, 4, 3.5]], [[7, 8, 9], [2, 3, 1]], [[5.5, 8, 5.5], [3.5, 3, 0.5]],
             [[4, 8, 2], [5, 3, 0]], [[4, 8, 2], [5, 3, 0]]]
    assert ResizeBilinear(6, 2, data_format="NHWC").forward(x)[0].tolist() == exp_h
    exp_w = [[[1, 2, 3], [2.5, 3.5, 4.5], [4, 5, 6], [4, 5, 6]], [[7, 8, 9], [4.5, 5.5, 5], [2, 3, 1], [2, 3, 1]],
             [[4, 8, 2], [4.5, 5.5, 1], [5, 3, 0], [5, 3, 0]]]
    assert ResizeBilinear(3, 4, data_format="NHWC").forward(x)[0].tolist() == exp_w


@pytest.mark.parametrize("ih,iw,oh,ow,align", [(3, 2, 3, 2, True), (3, 2, 6, 2, True), (3, 2, 3, 4, True),
                                                (3, 2, 6, 2, False), (5, 7, 3, 4, False), (4, 4, 9, 9, True)])
def test_nchw_nhwc_agree_and_gradcheck(ih, iw, oh, ow, align):
    from bigdl.nn import ResizeBilinear
    torch.manual_seed(0)
    x = torch.rand(1, 3, ih, iw, dtype=torch.float64)
    gy = torch.rand(1, 3, oh, ow, dtype=torch.float64)
    cf = ResizeBilinear(oh, ow, align, data_format="NCHW")
    cl = ResizeBilinear(oh, ow, align, data_format="NHWC")
    yf = cf.forward(x)
    gf = cf.backward(x, gy)
    yl = cl.forward(x.permute(0, 2, 3, 1).contiguous())
    gl = cl.backward(x.permute(0, 2, 3, 1).contiguous(), gy.permute(0, 2, 3, 1).contiguous())
    torch.testing.assert_close(yl.permute(0, 3, 1, 2), yf)
    torch.testing.assert_close(gl.permute(0, 3, 1, 2), gf)
    from bigdl.ops.reference import resize_bilinear
    assert torch.autograd.gradcheck(lambda v: resize_bilinear(v, oh, ow, align), (x.clone().requires_grad_(),))
    if align and oh > 1:  # corners map onto corners
        torch.testing.assert_close(yf[..., 0, 0], x[..., 0, 0])
        torch.testing.assert_close(yf[..., -1, -1], x[..., -1, -1])


@pytest.mark.gpu
@pytest.mark.parametrize("N,C,H,W,oh,ow,align", [(2, 64, 13, 17, 26, 34, False), (2, 32, 20, 20, 7, 9, True),
                                                  (1, 8, 5, 5, 5, 5, False)])
def test_native_resize_matches_reference(N, C, H, W, oh, ow, align):
    from bigdl.ops import native_ops as NO
    from bigdl.ops.reference import resize_bilinear
    g = torch.Generator().manual_seed(0)
    x = torch.randn(N, C, H, W, generator=g).bfloat16()
    gy = torch.randn(N, C, oh, ow, generator=g).bfloat16()
    xr = x.float().requires_grad_()
    yr = resize_bilinear(xr, oh, ow, align)
    yr.backward(gy.float())
    xc = x.cuda().contiguous(memory_format=torch.channels_last).requires_grad_()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
        y = NO.resize_bilinear(xc, oh, ow, align)
        assert y is not NotImplemented
        y.backward(gy.cuda())
        torch.cuda.synchronize()
    names = [e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA]
    assert any("k_resize_bilinear_fwd" in n for n in names) and any("k_resize_bilinear_bwd" in n for n in names)
    torch.testing.assert_close(y.float().cpu(), yr.detach(), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(xc.grad.float().cpu(), xr.grad, rtol=2e-2, atol=2e-2)


@pytest.mark.gpu
def test_resize_module_runs_native():
    from bigdl.nn import ResizeBilinear
    m = ResizeBilinear(12, 14)
    x = torch.randn(2, 16, 5, 7).bfloat16().cuda()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
        y = m.forward(x)
        m.backward(x, torch.ones_like(y))
        torch.cuda.synchronize()
    names = [e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA]
    assert any("k_resize_bilinear_fwd" in n for n in names) and any("k_resize_bilinear_bwd" in n for n in names)
    from bigdl.ops.reference import resize_bilinear
    torch.testing.assert_close(y.float().cpu(), resize_bilinear(x.float().cpu(), 12, 14), rtol=1e-2, atol=1e-2)
