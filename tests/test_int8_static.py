"""Calibrated (static) int8 inference chains (``MklInt8Convertible.calcScales`` → ``quantize``):
quantised convs that feed each other through ReLU / max pooling hand over int8 NHWC activations
requantised in the producer's epilogue (ops/csrc/conv_i8.hip ``bigdl_conv_i8_fwd2``), the pooling
runs on int8, and the logits stay close to the float model."""
import pytest
import torch


def _net():
    import bigdl.nn as nn
    m = nn.Sequential()
    m.add(nn.SpatialConvolution(3, 64, 3, 3, 1, 1, 1, 1)).add(nn.ReLU())
    m.add(nn.SpatialConvolution(64, 64, 3, 3, 1, 1, 1, 1)).add(nn.ReLU())
    m.add(nn.SpatialMaxPooling(2, 2, 2, 2))
    m.add(nn.SpatialConvolution(64, 128, 3, 3, 1, 1, 1, 1)).add(nn.ReLU())
    m.add(nn.SpatialConvolution(128, 128, 3, 3, 1, 1, 1, 1)).add(nn.ReLU())
    m.add(nn.SpatialMaxPooling(2, 2, 2, 2))
    m.add(nn.View(128 * 4 * 4)).add(nn.Linear(128 * 4 * 4, 10))
    return m


def test_int8_chain_links_after_calibration():
    from bigdl.nn.quantized import layers as Q
    torch.manual_seed(0)
    m = _net()
    m.evaluate()
    x = torch.randn(4, 3, 16, 16)
    m.forward(x)
    m.calcScales(x)
    q = m.quantize()
    convs = [c for c in q.modules if isinstance(c, Q.SpatialConvolution)]
    assert all(c.static_scale is not None and c.static_scale > 0 for c in convs)
    # conv1 → conv2 → (pool) → conv3 → conv4: three producers write int8 for their consumer
    assert [c._out_qscale is not None for c in convs] == [True, True, True, False]
    assert all(c._relu_fused for c in convs[:3])
    assert convs[0]._out_qscale == convs[1].static_scale


@pytest.mark.gpu
def test_int8_static_chain_matches_float_on_gpu():
    from bigdl.utils import config
    from bigdl.utils.engine import Engine
    from bigdl.nn.quantized import layers as Q
    from bigdl import ops
    config.set_property("bigdl.compute.dtype", "bf16")
    Engine.init(device="cuda:0")
    torch.manual_seed(0)
    m = _net().to(device="cuda")
    m.evaluate()
    xc = torch.randn(8, 3, 16, 16, device="cuda")
    with torch.no_grad():
        m.forward(xc)
    m.calcScales(xc)
    q = m.quantize()
    x = torch.randn(16, 3, 16, 16, device="cuda")
    convs = [c for c in q.modules if isinstance(c, Q.SpatialConvolution)]
    ops.reset_fallbacks()
    with torch.no_grad():
        yq = q.forward(x).float()
        yf = m.forward(x).float()
    outs = [c.output.dtype for c in convs]
    assert outs[:3] == [torch.int8] * 3 and outs[3] == torch.bfloat16, outs
    a, b = yq.flatten().double(), yf.flatten().double()
    cos = float(a @ b / (a.norm() * b.norm()))
    assert cos >= 0.99, cos
    assert ops.fallback_counts() == {}
