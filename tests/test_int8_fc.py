"""int8 classifier head (the reference's quantized/Linear.scala with MKL-DNN's static scales): a
calibrated quantised Linear takes the int8 activation of the chain as is (through max pooling and
the flatten), runs the int8 MFMA GEMM split over K for small-M long-K products, and writes the next
quantised Linear's int8 input from its epilogue (bias, ReLU, requantisation; unsigned code after a
ReLU).  Checked against the fp32 GEMM of the dequantised operands and, end to end, the fp32 net."""
import pytest
import torch

from bigdl.nn.quantized import layers as Q


def _head_net():
    import bigdl.nn as nn
    m = nn.Sequential()
    m.add(nn.SpatialConvolution(3, 32, 3, 3, 1, 1, 1, 1)).add(nn.ReLU())
    m.add(nn.SpatialConvolution(32, 64, 3, 3, 1, 1, 1, 1)).add(nn.ReLU())
    m.add(nn.SpatialMaxPooling(2, 2, 2, 2))
    m.add(nn.View(64 * 8 * 8)).add(nn.Linear(64 * 8 * 8, 256)).add(nn.ReLU()).add(nn.Dropout(0.5))
    m.add(nn.Linear(256, 128)).add(nn.ReLU()).add(nn.Linear(128, 10))
    return m


def test_int8_fc_head_links_after_calibration():
    torch.manual_seed(0)
    m = _head_net()
    m.evaluate()
    x = torch.randn(4, 3, 16, 16)
    m.forward(x)
    m.calcScales(x)
    q = m.quantize()
    convs = [c for c in q.modules if isinstance(c, Q.SpatialConvolution)]
    fcs = [c for c in q.modules if isinstance(c, Q.Linear)]
    assert len(fcs) == 3 and all(f.static_scale is not None for f in fcs)
    # conv → conv → pool → flatten → fc1 → ReLU → dropout → fc2 → ReLU → fc3: int8 all the way
    assert all(c._out_qscale is not None for c in convs)
    assert [f._out_qscale is not None for f in fcs] == [True, True, False]
    assert fcs[0]._relu_fused and fcs[0]._out_u8 and fcs[1]._relu_fused
    assert fcs[0]._out_qscale == pytest.approx(fcs[1].static_scale * 127 / 255)


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(128, 512, 25088), (16, 1000, 2048), (256, 96, 64)])
@pytest.mark.parametrize("mode", ["bf16", "i8", "u8"])
def test_gemm_i8_static_matches_fp32(M, N, K, mode):
    from bigdl.ops import native_ops as NO
    torch.manual_seed(1)
    qa = torch.randint(-127, 128, (M, K), dtype=torch.int8, device="cuda")
    qb = torch.randint(-127, 128, (N, K), dtype=torch.int8, device="cuda")
    sa0 = 0.013
    sb = torch.rand(N, device="cuda") * 1e-3 + 1e-4
    bias = torch.randn(N, device="cuda")
    ref = (qa.double() @ qb.double().t()) * sa0 * sb.double() + bias.double()
    relu = mode == "u8"
    if relu:
        ref = ref.clamp_min(0)
    if mode == "bf16":
        y = NO.gemm_i8_static(qa, sa0, qb, sb, bias)
        assert y.dtype == torch.bfloat16
        err = float((y.double() - ref).norm() / ref.norm())
        assert err < 4e-3, err
        return
    osc = float(ref.abs().max()) / (255.0 if relu else 127.0)
    y = NO.gemm_i8_static(qa, sa0, qb, sb, bias, relu=relu, out_scale=osc, out_u8=relu)
    assert y.dtype == torch.int8 and y._qscale == osc and y._qzero == (128 if relu else 0)
    deq = (y.double() + y._qzero) * osc
    assert float((deq - ref).abs().max()) <= 0.5 * osc * (1 + 1e-3) + 1e-6


@pytest.mark.gpu
def test_int8_fc_head_matches_fp32_and_runs_int8():
    torch.manual_seed(0)
    m = _head_net()
    m.evaluate()
    x = torch.randn(32, 3, 16, 16)
    y32 = m.forward(x).clone()
    m.calcScales(x)
    q = m.quantize()
    q.cuda()
    q.evaluate()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
        yq = q.forward(x.cuda())
        torch.cuda.synchronize()
    names = [e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA]
    assert sum("k_gemm_i8" in n for n in names) >= 3, names
    assert not any("quant_rows" in n for n in names), names  # static scales: no per-row pass
    a, b = yq.float().cpu().reshape(-1), y32.float().reshape(-1)
    cos = float(a @ b / (a.norm() * b.norm()))
    assert cos > 0.99, cos
