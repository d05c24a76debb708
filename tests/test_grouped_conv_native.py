"""Grouped convolution in one launch (SpatialConvolution.scala:93-98 nGroup): the groups are packed
onto block-diagonal filters and the pack index is the grid's y (forward, data gradient) / z (weight
gradient) dimension of the implicit-GEMM kernels — no per-group slice copies or launches.
Numerics vs an fp32 F.conv2d(groups=G) of the same bf16 operands; a ResNeXt-style 32-group block
must launch exactly one conv kernel per pass."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = "cuda"


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


@pytest.mark.parametrize("N,C,K,G,H,R,st", [
    (4, 128, 128, 32, 14, 3, 1),   # ResNeXt-50 32x4d stage-1 width (Cg = Kg = 4)
    (4, 256, 256, 32, 14, 3, 2),   # Cg = Kg = 8, strided (stride-lattice data gradient)
    (2, 96, 256, 2, 13, 5, 1),     # AlexNet-style 2 groups
    (2, 64, 64, 4, 9, 3, 2),
    (2, 1024, 1024, 32, 7, 3, 1),  # Cg = Kg = 32
])
def test_grouped_conv_single_launch_matches_fp32(N, C, K, G, H, R, st):
    from bigdl.ops import native_ops as NO
    g = torch.Generator().manual_seed(0)
    pd = R // 2
    x = torch.randn(N, C, H, H, generator=g).bfloat16()
    w = (torch.randn(K, C // G, R, R, generator=g) * 0.1).bfloat16()
    b = torch.randn(K, generator=g)
    xr, wr, br = x.float().requires_grad_(), w.float().requires_grad_(), b.clone().requires_grad_()
    yr = F.conv2d(xr, wr, br, st, pd, 1, G)
    gy = torch.randn(yr.shape, generator=g).bfloat16()
    yr.backward(gy.float())
    xc = x.to(dev).contiguous(memory_format=torch.channels_last)
    wc = w.to(dev)
    gyc = gy.to(dev).contiguous(memory_format=torch.channels_last)
    gw = torch.zeros(w.shape, device=dev)
    gb = torch.zeros(K, device=dev)
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
        y = NO.conv2d_forward(xc, wc, b.to(dev), (st, st), (pd, pd), groups=G)
        gi = NO.conv2d_backward(gyc, xc, wc, (st, st), (pd, pd), groups=G, need_input=True, gw_acc=gw, gb_acc=gb)
        torch.cuda.synchronize()
    assert y is not NotImplemented and gi is not NotImplemented
    ev = [e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA]
    assert sum("k_conv_fwd" in n for n in ev) == 2, ev       # forward + data gradient
    assert sum("k_conv_wgrad" in n for n in ev) == 1, ev
    assert _rel(y.cpu(), yr) < 1e-2
    assert _rel(gi.cpu(), xr.grad) < 1e-2
    assert _rel(gw.cpu(), wr.grad) < 1e-2
    assert _rel(gb.cpu(), br.grad) < 1e-3


def test_resnext_block_grouped_conv_module():
    """SpatialConvolution(nGroup=32) inside a bottleneck trains on the single-launch path."""
    from bigdl.nn import ReLU, Sequential, SpatialBatchNormalization, SpatialConvolution
    from bigdl.utils import config
    from bigdl.utils.engine import Engine
    config.set_property("bigdl.compute.dtype", "bf16")
    Engine.init(device="cuda:0")
    torch.manual_seed(0)
    m = (Sequential().add(SpatialConvolution(256, 128, 1, 1)).add(SpatialBatchNormalization(128)).add(ReLU())
         .add(SpatialConvolution(128, 128, 3, 3, 1, 1, 1, 1, n_group=32)).add(SpatialBatchNormalization(128))
         .add(ReLU()).add(SpatialConvolution(128, 256, 1, 1)))
    ref = m.cloneModule()
    x = torch.randn(4, 256, 14, 14)
    yr = ref.forward(x)
    gy = torch.randn(yr.shape)
    gr = ref.backward(x, gy)
    m.cuda()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
        y = m.forward(x.cuda())
        gi = m.backward(x.cuda(), gy.cuda())
        torch.cuda.synchronize()
    ev = [e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA]
    assert sum("k_conv_fwd" in n for n in ev) <= 6, ev
    assert _rel(y.float().cpu(), yr) < 3e-2
    assert _rel(gi.float().cpu(), gr) < 1e-1  # bf16 through two training BNs at 784 rows per channel


@pytest.mark.parametrize("N,Cin,Cout,G,H,R,st,pd,adj", [
    (2, 64, 32, 4, 9, 3, 2, 1, 1),
    (2, 128, 128, 32, 7, 4, 2, 1, 0),
    (2, 32, 64, 2, 8, 3, 1, 1, 0),
])
def test_grouped_transposed_conv_matches_fp32(N, Cin, Cout, G, H, R, st, pd, adj):
    """SpatialFullConvolution nGroup > 1 on the single-launch grouped kernels vs F.conv_transpose2d."""
    from bigdl.ops import native_ops as NO
    g = torch.Generator().manual_seed(1)
    x = torch.randn(N, Cin, H, H, generator=g).bfloat16()
    w = (torch.randn(Cin, Cout // G, R, R, generator=g) * 0.1).bfloat16()
    b = torch.randn(Cout, generator=g)
    xr, wr, br = x.float().requires_grad_(), w.float().requires_grad_(), b.clone().requires_grad_()
    yr = F.conv_transpose2d(xr, wr, br, st, pd, adj, G)
    gy = torch.randn(yr.shape, generator=g).bfloat16()
    yr.backward(gy.float())
    xc = x.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_()
    wc = w.float().to(dev).requires_grad_()
    bc = b.to(dev).requires_grad_()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
        y = NO.conv_transpose2d(xc, wc, bc, (st, st), (pd, pd), (adj, adj), G)
        assert y is not NotImplemented
        y.backward(gy.to(dev))
        torch.cuda.synchronize()
    ev = [e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA]
    assert sum("k_conv_fwd" in n for n in ev) == 2 and sum("k_conv_wgrad" in n for n in ev) == 1, ev
    assert y.shape == yr.shape
    assert _rel(y.cpu(), yr) < 1e-2
    assert _rel(xc.grad.cpu(), xr.grad) < 1e-2
    assert _rel(wc.grad.cpu(), wr.grad) < 1e-2
    assert _rel(bc.grad.cpu(), br.grad) < 1e-3
