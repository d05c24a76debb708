"""fp32 NHWC max / average pooling (csrc/pooling.hip fp32 instantiations; the reference's precision,
SpatialMaxPooling / SpatialAveragePooling, DL/nn/NNPrimitive.scala:654-748,
DL/nn/SpatialAveragePooling.scala:115-700) against torch's fp64 pooling of the same tensors."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = "cuda"
cl = torch.channels_last


@pytest.mark.parametrize("N,C,H,k,s,p,ceil", [(4, 64, 112, 3, 2, 1, False), (2, 24, 13, 3, 2, 0, True),
                                               (3, 16, 9, 2, 2, 0, False), (16, 6, 24, 2, 2, 0, False),
                                               (4, 12, 8, 2, 2, 0, False), (2, 3, 11, 3, 2, 1, True)])
def test_maxpool32_matches_torch(N, C, H, k, s, p, ceil):
    from bigdl.ops import native_ops as NO
    g = torch.Generator().manual_seed(0)
    x = torch.randn(N, C, H, H, generator=g)
    xr = x.double().requires_grad_()
    yr = F.max_pool2d(xr, k, s, p, ceil_mode=ceil)
    gy = torch.randn(yr.shape, generator=g)
    yr.backward(gy.double())
    xd = x.to(dev).contiguous(memory_format=cl)
    r = NO.maxpool2d_forward(xd, (k, k), (s, s), (p, p), ceil)
    assert r is not NotImplemented
    y, idx = r
    assert y.dtype == torch.float32 and torch.equal(y.cpu().double(), yr.detach())
    gx = NO.maxpool2d_backward(gy.to(dev).contiguous(memory_format=cl), xd, idx, (k, k), (s, s), (p, p), ceil)
    assert gx is not NotImplemented and gx.dtype == torch.float32
    torch.cuda.synchronize()
    assert torch.allclose(gx.cpu().double(), xr.grad, atol=1e-6, rtol=1e-6)


@pytest.mark.parametrize("N,C,H,k,s,p,cip", [(4, 2048, 7, 7, 1, 0, True), (2, 32, 14, 3, 2, 1, False),
                                              (2, 32, 14, 3, 2, 1, True)])
def test_avgpool32_matches_torch(N, C, H, k, s, p, cip):
    from bigdl.ops import native_ops as NO
    g = torch.Generator().manual_seed(1)
    x = torch.randn(N, C, H, H, generator=g)
    xr = x.double().requires_grad_()
    yr = F.avg_pool2d(xr, k, s, p, count_include_pad=cip)
    gy = torch.randn(yr.shape, generator=g)
    yr.backward(gy.double())
    xd = x.to(dev).contiguous(memory_format=cl)
    y = NO.avgpool2d_forward(xd, (k, k), (s, s), (p, p), False, cip)
    assert y is not NotImplemented and y.dtype == torch.float32
    gx = NO.avgpool2d_backward(gy.to(dev), xd, (k, k), (s, s), (p, p), False, cip)
    assert gx is not NotImplemented and gx.dtype == torch.float32
    torch.cuda.synchronize()
    assert torch.allclose(y.cpu().double(), yr.detach(), atol=1e-6, rtol=1e-5)
    assert torch.allclose(gx.cpu().double(), xr.grad, atol=1e-6, rtol=1e-5)
