"""Native 3-D convolution (VolumetricConvolution.scala) on the implicit-GEMM kernels
(conv_igemm.hip k_conv_fwd<…, D3>, conv_wgrad.hip k_conv_wgrad<…, D3>): forward, data gradient
(stride 1 and strided via the stride lattice) and weight / bias gradients against an fp32
F.conv3d reference of the same bf16-rounded operands."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = "cuda"


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


@pytest.mark.parametrize("N,C,K,T,H,W,k,s,p,d", [
    (2, 16, 32, 6, 10, 10, (3, 3, 3), (1, 1, 1), (1, 1, 1), (1, 1, 1)),
    (2, 3, 64, 8, 12, 12, (3, 5, 5), (1, 2, 2), (1, 2, 2), (1, 1, 1)),   # C = 3 (padded to 8), strided
    (1, 64, 64, 5, 9, 7, (2, 3, 3), (2, 2, 1), (0, 1, 1), (1, 1, 1)),
    (2, 32, 16, 7, 8, 8, (3, 3, 3), (1, 1, 1), (2, 2, 2), (2, 2, 2)),   # dilated
    (1, 8, 8, 4, 5, 5, (1, 1, 1), (1, 1, 1), (0, 0, 0), (1, 1, 1)),
    (2, 128, 136, 3, 6, 6, (3, 3, 3), (1, 1, 1), (1, 1, 1), (1, 1, 1)),  # K-tail tile, Kg > 512
])
def test_conv3d_native_matches_fp32(N, C, K, T, H, W, k, s, p, d):
    from bigdl.ops import native_ops as NO
    g = torch.Generator().manual_seed(0)
    x = torch.randn(N, C, T, H, W, generator=g).to(torch.bfloat16)
    w = (torch.randn(K, C, *k, generator=g) * 0.1).to(torch.bfloat16)
    b = torch.randn(K, generator=g)
    xr, wr, br = x.float().requires_grad_(), w.float().requires_grad_(), b.clone().requires_grad_()
    yr = F.conv3d(xr, wr, br, s, p, d)
    gy = torch.randn(yr.shape, generator=g).to(torch.bfloat16)
    yr.backward(gy.float())

    xc = x.to(dev).contiguous(memory_format=torch.channels_last_3d).requires_grad_()
    wc = w.float().to(dev).requires_grad_()
    bc = b.to(dev).requires_grad_()
    y = NO.conv3d_autograd(xc, wc, bc, s, p, d)
    assert y is not NotImplemented
    assert y.shape == yr.shape
    y.backward(gy.to(dev))
    torch.cuda.synchronize()
    assert _rel(y.cpu(), yr) < 1e-2
    assert _rel(xc.grad.cpu(), xr.grad) < 1e-2
    assert _rel(wc.grad.cpu(), wr.grad) < 1e-2
    assert _rel(bc.grad.cpu(), br.grad) < 1e-3


def test_volumetric_convolution_module_native_and_same_padding():
    from bigdl.nn import VolumetricConvolution
    from bigdl.utils import config
    from bigdl.utils.engine import Engine
    config.set_property("bigdl.compute.dtype", "bf16")
    Engine.init(device="cuda:0")
    torch.manual_seed(0)
    for pads in ((1, 1, 1), (-1, -1, -1)):
        m = VolumetricConvolution(8, 16, 3, 3, 3, 2, 2, 2, *pads)
        ref = VolumetricConvolution(8, 16, 3, 3, 3, 2, 2, 2, *pads)
        ref.weight.copy_(m.weight.bfloat16().float())
        ref.bias.copy_(m.bias)
        x = torch.randn(2, 8, 7, 9, 9).bfloat16()
        yr = ref.forward(x.float())
        gy = torch.randn(yr.shape).bfloat16()
        gr = ref.backward(x.float(), gy.float())
        m.cuda()
        with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
            y = m.forward(x.to(dev))
            gi = m.backward(x.to(dev), gy.to(dev))
            torch.cuda.synchronize()
        names = {e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA}
        assert any("k_conv_fwd" in n for n in names) and any("k_conv_wgrad" in n for n in names), sorted(names)
        assert not any("miopen" in n.lower() or "conv3d" in n.lower() for n in names), sorted(names)
        assert _rel(y.cpu(), yr) < 1e-2
        assert _rel(gi.cpu(), gr) < 1e-2
        assert _rel(m.parameters()[1][0].cpu(), ref.parameters()[1][0]) < 2e-2
