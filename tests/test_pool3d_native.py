"""Native 3-D max / average pooling (pool3d.hip; VolumetricMaxPooling.scala /
VolumetricAveragePooling.scala) against F.max_pool3d / F.avg_pool3d on the same bf16 values:
outputs (max exact, average to bf16 rounding) and input gradients (fp32-accumulated scatter)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("N,C,T,H,W,k,s,p,ceil,cip", [
    (2, 16, 8, 10, 10, (2, 2, 2), (2, 2, 2), (0, 0, 0), False, True),
    (2, 32, 7, 9, 11, (3, 3, 3), (2, 2, 2), (1, 1, 1), False, True),
    (1, 8, 5, 7, 7, (3, 3, 3), (2, 2, 2), (1, 1, 1), True, False),
    (2, 64, 4, 6, 6, (1, 3, 3), (1, 1, 1), (0, 1, 1), False, False),
])
def test_pool3d_matches_torch(mode, N, C, T, H, W, k, s, p, ceil, cip):
    from bigdl.ops import native_ops as NO
    g = torch.Generator().manual_seed(0)
    x = torch.randn(N, C, T, H, W, generator=g).bfloat16()
    xr = x.float().requires_grad_()
    yr = F.max_pool3d(xr, k, s, p, ceil_mode=ceil) if mode == 0 else F.avg_pool3d(xr, k, s, p, ceil, cip)
    gy = torch.randn(yr.shape, generator=g).bfloat16()
    yr.backward(gy.float())
    xc = x.cuda().contiguous(memory_format=torch.channels_last_3d).requires_grad_()
    y = NO.pool3d(xc, mode, k, s, p, ceil, cip)
    assert y is not NotImplemented and y.shape == yr.shape
    y.backward(gy.cuda())
    torch.cuda.synchronize()
    if mode == 0:
        torch.testing.assert_close(y.float().cpu(), yr.detach().bfloat16().float(), rtol=0, atol=0)
    else:
        torch.testing.assert_close(y.float().cpu(), yr.detach(), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(xc.grad.float().cpu(), xr.grad, rtol=1e-2, atol=1e-2)


def test_volumetric_pooling_modules_native():
    from bigdl.nn import VolumetricAveragePooling, VolumetricMaxPooling
    x = torch.randn(2, 16, 6, 8, 8).bfloat16().cuda()
    for m in (VolumetricMaxPooling(2, 2, 2, 2, 2, 2), VolumetricAveragePooling(2, 2, 2, 2, 2, 2)):
        with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
            y = m.forward(x)
            m.backward(x, torch.ones_like(y))
            torch.cuda.synchronize()
        names = [e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA]
        assert any("k_pool3d_fwd" in n for n in names) and any("k_pool3d_bwd" in n for n in names), names
