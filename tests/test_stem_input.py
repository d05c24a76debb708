"""The RGB model input enters the stem conv through ONE cast + relayout + channel-pad pass
(elementwise.hip k_nchw_to_nhwc_pad): forward and weight gradient of a 7×7/2 stem on an fp32 NCHW
batch match torch's fp32 conv of the bf16-rounded operands, and the padded operand is the one the
kernel read (no second pad pass)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_rgb_stem_padded_conversion_matches_torch():
    from bigdl.utils.engine import Engine
    from bigdl.utils import config
    import bigdl.nn as nn
    from bigdl import ops
    config.set_property("bigdl.compute.dtype", "bf16")
    Engine.init(device="cuda:0")
    ops.reset_fallbacks()
    torch.manual_seed(0)
    m = nn.SpatialConvolution(3, 64, 7, 7, 2, 2, 3, 3, propagate_back=False).to(device="cuda")  # as the ResNet stem
    x = torch.randn(4, 3, 32, 32, device="cuda")
    y = m.forward(x)
    slot = m._pad_slot_()[0]
    assert slot is not None and slot[3].shape[1] == 4  # the padded operand came from the conversion
    assert float(slot[3][:, 3].abs().max()) == 0.0
    xb = x.bfloat16().float()
    wb = m.weight.detach().float().view(64, 3, 7, 7).bfloat16().float()
    ref = torch.nn.functional.conv2d(xb, wb, m.bias.detach().float(), 2, 3)
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=3e-2)
    gy = torch.randn_like(ref)
    m.zeroGradParameters()
    m.backward(x, gy.bfloat16().contiguous(memory_format=torch.channels_last))
    xr = xb.clone().requires_grad_(False)
    wr = wb.clone().requires_grad_(True)
    torch.nn.functional.conv2d(xr, wr, None, 2, 3).backward(gy.bfloat16().float())
    gw = m.gradWeight.float().view(64, 3, 7, 7)
    torch.testing.assert_close(gw, wr.grad, rtol=3e-2, atol=3e-2 * float(wr.grad.abs().max()))
    assert ops.fallback_counts() == {}
    config.set_property("bigdl.compute.dtype", "auto")
