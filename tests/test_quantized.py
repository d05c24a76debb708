"""int8 quantization (nn/quantized): per-window math golden values, model rewrite, CPU accuracy,
and the native int8 MFMA GEMM vs the exact int32 reference on GPU."""
import pytest
import torch

from bigdl import nn
from bigdl.ops import reference as R


def test_quantize_math_matches_reference_formula():
    # Quantization.quantize: round(v / max(|max|,|min|) * 127), Math.round = half-up
    x = torch.tensor([[1.0, -2.0, 0.5, 0.0], [0.1, 0.2, 0.3, 0.4]])
    q, s = R.quant_rows(x, 64)
    assert q[0, :4].tolist() == [64, -127, 32, 0]  # 63.5 rounds up to 64
    assert q[1, :4].tolist() == [32, 64, 95, 127]
    assert (q[:, 4:] == 0).all()
    torch.testing.assert_close(s, torch.tensor([2.0 / 127, 0.4 / 127]))


def _net():
    m = nn.Sequential()
    m.add(nn.SpatialConvolution(3, 16, 3, 3, 1, 1, 1, 1)).add(nn.ReLU())
    m.add(nn.SpatialDilatedConvolution(16, 16, 3, 3, 1, 1, 2, 2, 2, 2)).add(nn.ReLU())
    m.add(nn.SpatialConvolution(16, 8, 3, 3, 2, 2, 1, 1, 2)).add(nn.ReLU())
    m.add(nn.View([8 * 4 * 4])).add(nn.Linear(128, 10))
    return m


def test_quantize_model_rewrite_and_accuracy():
    from bigdl.nn import quantized as Q
    m = _net().evaluate()
    x = torch.randn(4, 3, 8, 8)
    y = m.forward(x).clone()
    q = m.quantize()
    kinds = [type(c) for c in q.modules]
    assert Q.SpatialConvolution in kinds and Q.SpatialDilatedConvolution in kinds and Q.Linear in kinds
    assert isinstance(m.modules[0], nn.SpatialConvolution)  # original untouched (cloned)
    yq = q.forward(x)
    rel = (yq - y).abs().max() / y.abs().max()
    assert rel < 0.05, rel
    with pytest.raises(Exception):
        q.backward(x, torch.ones_like(yq))


def test_quantize_graph_model():
    inp = nn.Input()
    c = nn.SpatialConvolution(3, 4, 3, 3)(inp)
    r = nn.ReLU()(c)
    g = nn.Graph([inp], [r]).evaluate()
    x = torch.randn(2, 3, 6, 6)
    y = g.forward(x).clone()
    q = g.quantize()
    torch.testing.assert_close(q.forward(x), y, rtol=0.05, atol=0.05)


@pytest.mark.gpu
def test_gemm_i8_native_exact():
    from bigdl.ops import native_status, native_ops as NO
    assert native_status()["loaded"]
    torch.manual_seed(0)
    for (M, N, K) in [(37, 50, 70), (256, 384, 1152), (1, 10, 16)]:
        a = torch.randn(M, K, device="cuda")
        b = torch.randn(N, K, device="cuda")
        qa, sa = NO.quant_rows(a)
        ra, rsa = R.quant_rows(a)
        assert torch.equal(qa, ra), (M, N, K)
        torch.testing.assert_close(sa, rsa)
        qb, sb = R.quant_rows(b)
        bias = torch.randn(N, device="cuda")
        out = NO.gemm_i8(qa, sa, qb, sb, bias)
        ref = R.gemm_i8(qa, sa, qb, sb, bias)
        torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-4)
        outb = NO.gemm_i8(qa, sa, qb, sb, bias, out_dtype=torch.bfloat16)
        torch.testing.assert_close(outb.float(), ref, rtol=1e-2, atol=1e-2)


@pytest.mark.gpu
def test_quantized_model_gpu_matches_cpu():
    m = _net().evaluate()
    x = torch.randn(4, 3, 8, 8)
    q = m.quantize()
    ycpu = q.forward(x).clone()
    qg = q.cuda()
    yg = qg.forward(x.cuda()).float().cpu()
    torch.testing.assert_close(yg, ycpu, rtol=1e-3, atol=1e-3)


def test_mkl_int8_convertible_calc_scales_and_serialization(tmp_path):
    """``MklInt8Convertible.calcScales`` on a Sequential (``MklInt8ConvertibleSpec``): input/output/
    weight max-abs per mask; the scales survive a .bigdl round trip (proto fields 17-23)."""
    import torch
    from bigdl.nn import Sequential, Linear, ReLU, SpatialConvolution, View
    from bigdl.nn.module import Module
    from bigdl.nn.int8_convertible import calc_tensor_scale
    torch.manual_seed(0)
    m = Sequential().add(SpatialConvolution(2, 4, 3, 3)).add(ReLU()).add(View(4 * 3 * 3)).add(Linear(36, 5))
    conv, lin = m.modules[0], m.modules[3]
    conv.setWeightDimMask(1)
    conv.setOutputDimMask(2)
    x = torch.randn(3, 2, 5, 5)
    m.evaluate()
    m.forward(x)
    m.calcScales(x)
    assert m.getInputScales() == [[float(x.abs().max())]]
    assert conv.getWeightScales()[0] == [float(v) for v in conv.weight.reshape(4, -1).abs().amax(1)]
    assert len(conv.getOutputScales()[0]) == 4  # per output channel (mask bit of dim 1)
    assert lin.getInputScales()[0] == [float(m.modules[2].output.abs().max())]
    assert calc_tensor_scale(torch.tensor([[1.0, -3.0], [2.0, 0.5]]), 3) == [1.0, 3.0, 2.0, 0.5]
    assert calc_tensor_scale(torch.tensor([[1.0, -3.0], [2.0, 0.5]]), 2) == [2.0, 3.0]
    p = str(tmp_path / "s.bigdl")
    m.saveModule(p, over_write=True)
    m2 = Module.loadModule(p)
    assert m2.modules[0].getWeightScales() == conv.getWeightScales()
    assert m2.modules[0].getWeightDimMask() == 1 and m2.modules[0].getOutputDimMask() == 2
    assert m2.getInputScales() == m.getInputScales()
