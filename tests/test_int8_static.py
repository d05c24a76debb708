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
    # conv1 → conv2 → (pool) → conv3 → conv4 → (pool, flatten) → fc: every conv writes int8 for
    # its consumer, the last one for the int8 classifier head
    fc = [c for c in q.modules if isinstance(c, Q.Linear)]
    assert len(fc) == 1 and fc[0].static_scale is not None and fc[0]._out_qscale is None
    assert [c._out_qscale is not None for c in convs] == [True, True, True, True]
    assert all(c._relu_fused for c in convs)
    # ReLU'd producers write the unsigned (offset −128) code: clip / 255 instead of clip / 127
    assert all(c._out_u8 for c in convs[:3])
    assert convs[0]._out_qscale == pytest.approx(convs[1].static_scale * 127 / 255)


def test_int8_chain_signed_when_unsigned_disabled():
    from bigdl.nn.quantized import layers as Q
    from bigdl.utils import config
    torch.manual_seed(0)
    m = _net()
    m.evaluate()
    x = torch.randn(4, 3, 16, 16)
    m.forward(x)
    m.calcScales(x)
    old = config.get_property("bigdl.int8.unsignedActivations")
    config.set_property("bigdl.int8.unsignedActivations", False)
    try:
        q = m.quantize()
    finally:
        config.set_property("bigdl.int8.unsignedActivations", old)
    convs = [c for c in q.modules if isinstance(c, Q.SpatialConvolution)]
    assert not any(c._out_u8 for c in convs)
    assert convs[0]._out_qscale == convs[1].static_scale


@pytest.mark.gpu
@pytest.mark.parametrize("stride,pad,k", [(1, 1, 3), (2, 1, 3), (1, 0, 1), (2, 0, 1)])
def test_conv_i8_unsigned_input_matches_fp32(stride, pad, k):
    """Unsigned (offset −128) int8 input: the kernel's per-tap weight-sum correction (border pixels
    sum their in-image taps only) reproduces the fp32 conv of the dequantised operands."""
    from bigdl.ops import native_ops as NO
    from bigdl.ops import reference as R
    torch.manual_seed(0)
    N, C, H, W, K = 2, 64, 9, 11, 32
    x = torch.rand(N, C, H, W, device="cuda") * 3.0
    w = torch.randn(K, C, k, k, device="cuda")
    bias = torch.randn(K, device="cuda")
    q, ws = R.quant_rows(w.reshape(K, -1).cpu())
    q, ws = q.cuda(), ws.cuda().float()
    wq, ldw = NO.conv_i8_weight(q, K, C, k, k)
    P = (H + 2 * pad - k) // stride + 1
    Q_ = (W + 2 * pad - k) // stride + 1
    sx = 3.0 / 255
    xc = x.contiguous(memory_format=torch.channels_last)
    xq = NO.quant_static(xc, sx, u8=True)
    assert xq._qzero == 128 and xq._qtail
    tail = torch.empty(0, dtype=torch.int8, device="cuda").set_(xq.untyped_storage(), xq.numel(), (16,), (1,))
    assert bool((tail == -128).all())
    xd = (xq.float() + 128) * sx
    assert float((xd - x).abs().max()) <= sx / 2 + 1e-6
    wd = (q[:, :C * k * k].float() * ws[:, None]).reshape(K, C, k, k)
    ref = torch.nn.functional.conv2d(xd, wd, bias, stride, pad)
    for relu, out_u8 in ((False, False), (True, True)):
        y = NO.conv2d_i8_forward_static(xq, wq, ldw, ws, bias, K, k, k, (stride, stride), (pad, pad), (1, 1),
                                        (P, Q_), relu=relu, out_scale=0.05 if out_u8 else None, out_u8=out_u8)
        assert y is not NotImplemented
        if out_u8:
            r = torch.relu(ref)
            assert y._qtail
            got = (y.float() + 128) * 0.05
            exp = (r / 0.05).round().clamp(0, 255) * 0.05
            assert float((got - exp).abs().max()) <= 0.05 + 1e-4
        else:
            err = float((y.float() - ref).abs().max() / ref.abs().max())
            assert err < 1e-2, err


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
    # every conv hands int8 on, the last one to the int8 classifier head (tests/test_int8_fc.py)
    assert outs == [torch.int8] * 4, outs
    a, b = yq.flatten().double(), yf.flatten().double()
    cos = float(a @ b / (a.norm() * b.norm()))
    assert cos >= 0.99, cos
    assert ops.fallback_counts() == {}


@pytest.mark.parametrize("stride,pad,k,dil", [(1, 1, 3, 1), (2, 1, 3, 1), (1, 0, 1, 1), (2, 3, 7, 1), (1, 2, 3, 2)])
def test_u8_offset_bias_reproduces_float_conv(stride, pad, k, dil):
    """The unsigned-input int8 conv's arithmetic — integer conv of the stored codes whose padded taps
    read the code of 0 (−128, the input's tail), scaled, plus the bias with the offset term folded in
    (``conv_i8_u8_bias``) — equals the float conv of the dequantised input on every pixel."""
    from bigdl.ops import native_ops as NO
    torch.manual_seed(0)
    N, C, H, W, K = 2, 16, 9, 10, 8
    q = torch.randint(-128, 128, (N, C, H, W)).double()
    wi = torch.randint(-127, 128, (K, C, k, k))
    ldw = k * k * C + 32
    wq = torch.zeros(K, ldw, dtype=torch.int8)
    wq[:, :k * k * C] = wi.permute(0, 2, 3, 1).reshape(K, -1).to(torch.int8)
    sx, sw, bias = 0.01, torch.rand(K) * 0.02, torch.randn(K)
    b2 = NO.conv_i8_u8_bias(wq, ldw, K, k, k, C, sx, sw, bias)
    qp = torch.nn.functional.pad(q, (pad, pad, pad, pad), value=-128.0)
    acc = torch.nn.functional.conv2d(qp, wi.double(), None, stride, 0, dil)
    got = acc * sx * sw.double()[:, None, None] + b2.double()[:, None, None]
    ref = torch.nn.functional.conv2d((q + 128) * sx, wi.double() * sw.double()[:, None, None, None], bias.double(),
                                     stride, pad, dil)
    assert torch.allclose(got, ref, rtol=1e-5, atol=1e-4), float((got - ref).abs().max())


@pytest.mark.gpu
@pytest.mark.parametrize("u8", [False, True])
def test_stem_conv_int8_epilogue_matches_two_pass(u8):
    """The RGB stem's int8 output written by the conv epilogue equals the bf16 conv followed by
    the static quantisation pass (same bf16-rounded values, same rounding), tail included."""
    from bigdl.ops import native_ops as NO
    torch.manual_seed(0)
    x = torch.randn(2, 3, 30, 34, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(64, 3, 3, 3, device="cuda") * 0.2).bfloat16()
    b = torch.randn(64, device="cuda")
    for relu in (True, False):
        if u8 and not relu:
            continue
        y = NO.conv2d_forward(x, w, b, (1, 1), (1, 1), relu=relu)
        scale = float(y.float().abs().max()) / (255 if u8 else 127)
        ref = NO.quant_static(y, scale, u8=u8)
        got = NO.conv2d_forward_q(x, w, b, (1, 1), (1, 1), relu, scale, u8=u8)
        assert got is not NotImplemented
        assert got._qscale == ref._qscale and got._qzero == ref._qzero
        assert torch.equal(got, ref)
        if u8:
            tail = torch.empty(0, dtype=torch.int8, device="cuda").set_(got.untyped_storage(), got.numel(), (16,), (1,))
            assert bool((tail == -128).all())


def _resnet50_calibrated(size=64, seed=3):
    from bigdl.models.resnet import ResNet, DatasetType, model_init
    from bigdl.nn import SpatialBatchNormalization
    from bigdl.utils.random import RNG
    RNG.setSeed(seed)
    torch.manual_seed(seed)
    m = model_init(ResNet(10, depth=50, dataset=DatasetType.ImageNet, image_size=size))
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for bn in m.flattened_modules():
            if isinstance(bn, SpatialBatchNormalization):
                bn.weight.uniform_(0.2, 1.0, generator=g)
                bn.bias.normal_(0.0, 0.1, generator=g)
        m.training()
        for _ in range(2):
            m.forward(torch.randn(4, 3, size, size, generator=g))
    m.evaluate()
    xc = torch.randn(4, 3, size, size, generator=g)
    with torch.no_grad():
        m.forward(xc)
    m.calcScales(xc)
    return m, g


def test_resnet50_int8_residual_blocks_link():
    """quantize() on a calibrated ResNet-50: BN folded into the convs (Fusion.scala conv + BN), every
    bottleneck becomes an int8 residual block whose last conv sums the shortcut in its epilogue, and
    every block but the last hands its output to the next block as int8 (MKL-DNN int8 scale
    propagation through conv + sum, DL/nn/mkldnn/Fusion.scala:120-165)."""
    from bigdl.nn.quantized import layers as Q
    from bigdl.nn.quantized.quantizer import Int8ResidualBlock
    from bigdl.nn import SpatialBatchNormalization
    m, _g = _resnet50_calibrated()
    q = m.quantize()
    assert not any(isinstance(b, SpatialBatchNormalization) for b in q.flattened_modules())
    blocks = [b for b in q.flattened_modules() if isinstance(b, Int8ResidualBlock)]
    assert len(blocks) == 16
    assert [b._out_qscale is not None for b in blocks] == [True] * 15 + [False]
    assert all(b._out_u8 for b in blocks[:15])
    # the block output scale is the next block's calibrated input scale (unsigned code: clip / 255)
    for a, b in zip(blocks, blocks[1:]):
        assert a._out_qscale == pytest.approx(b.head().static_scale * 127 / 255)
    # inside every branch conv1 → conv2 → conv3 are chained int8 with the ReLU fused
    for b in blocks:
        convs = [c for c in b.branch.modules if isinstance(c, Q.SpatialConvolution)]
        assert [c._out_qscale is not None for c in convs] == [True, True, False]
        assert convs[0]._relu_fused and convs[1]._relu_fused
    # the stem conv (+ folded BN, ReLU, max pooling) writes the first block's int8 input
    stem = [c for c in q.flattened_modules() if isinstance(c, Q.SpatialConvolution)][0]
    assert stem._out_qscale is not None and stem._relu_fused
    # the folded float model and the quantised one agree (CPU: dynamic int8 reference path)
    x = torch.randn(2, 3, 64, 64)
    with torch.no_grad():
        ref = m.forward(x).float()
        out = q.forward(x).float()
    cos = float(torch.nn.functional.cosine_similarity(out.reshape(1, -1), ref.reshape(1, -1)))
    assert cos > 0.99, cos


@pytest.mark.gpu
def test_int8_residual_epilogue_matches_reference():
    """conv2d_i8_forward_static(residual=…): ReLU(conv(x) + res) with the sum in the int8 kernel's
    epilogue equals the unfused conv (bf16 output) + the dequantised residual, for an int8 (unsigned
    code) and a bf16 residual, with bf16 and int8 outputs."""
    from bigdl.nn.quantized import layers as Q
    from bigdl.ops import native_ops as NO
    import bigdl.nn as nn
    torch.manual_seed(1)
    conv = nn.SpatialConvolution(128, 256, 1, 1).cuda()
    x = torch.randn(4, 128, 14, 14, device="cuda")
    conv.forward(x)
    conv.calcScales(x)
    q = Q.SpatialConvolution.from_float(conv).cuda()
    xb = x.bfloat16().contiguous(memory_format=torch.channels_last)
    plain = q._native_static(xb, (0, 0, 0, 0))  # bf16, no ReLU
    assert plain is not NotImplemented
    r = torch.relu(torch.randn(4, 256, 14, 14, device="cuda")).contiguous(memory_format=torch.channels_last)
    r8 = NO.quant_static(r, float(r.max()) / 255.0, u8=True)
    for res in (r8, r.bfloat16()):
        rf = Q.dequant(res).float() if res.dtype == torch.int8 else res.float()
        ref = torch.relu(plain.float() + rf)
        y = q.forward_residual(xb, res)
        torch.cuda.synchronize()
        assert y is not NotImplemented and y.dtype == torch.bfloat16
        torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2 * float(ref.abs().max()))
        sc = float(ref.max()) / 255.0
        yq = q.forward_residual(xb, res, out_scale=sc, out_u8=True)
        torch.cuda.synchronize()
        torch.testing.assert_close(Q.dequant(yq).float(), ref, rtol=0, atol=1.5 * sc + 2e-2 * float(ref.abs().max()))


@pytest.mark.gpu
def test_resnet50_int8_logits_track_fp32():
    """Calibrated int8 ResNet-50 (residual blocks, int8 block outputs) on the GPU vs the float model:
    logit cosine ≥ 0.99 (centred log-probabilities)."""
    from bigdl.utils.engine import Engine
    from bigdl.utils import config
    config.set_property("bigdl.compute.dtype", "bf16")
    Engine.init(device="cuda:0")
    m, g = _resnet50_calibrated(size=64, seed=4)
    q = m.quantize().cuda()
    q.evaluate()
    x = torch.randn(8, 3, 64, 64, generator=g)
    with torch.no_grad():
        ref = m.forward(x).double()
        out = q.forward(x.cuda().bfloat16().contiguous(memory_format=torch.channels_last)).double().cpu()
    ref, out = ref - ref.mean(1, keepdim=True), out - out.mean(1, keepdim=True)
    cos = float(torch.nn.functional.cosine_similarity(out.reshape(1, -1), ref.reshape(1, -1)))
    print("resnet50 int8 vs fp32 logit cosine", cos)
    assert cos >= 0.99, cos


def _inception_calibrated(size=224, seed=5):
    from bigdl.models.inception import Inception_v1_NoAuxClassifier
    from bigdl.utils.random import RNG
    RNG.setSeed(seed)
    torch.manual_seed(seed)
    m = Inception_v1_NoAuxClassifier.graph(10, has_dropout=False)
    m.evaluate()
    g = torch.Generator().manual_seed(seed)
    xc = torch.randn(2, 3, size, size, generator=g)
    with torch.no_grad():
        m.forward(xc)
    m.calcScales(xc)
    return m, g


def test_inception_int8_graph_links_and_unified_join_scales():
    """quantize() on a calibrated Inception-v1 graph: inside every branch the 1×1 reduce conv writes the
    3×3 / 5×5 conv's int8 input (ReLU fused), and every inception JoinTable whose consumers are int8
    convs gets its four producers at ONE common scale (the reference's input-scale unification ahead of
    a JoinTable, DL/nn/mkldnn/Fusion.scala:240-290) — the concat then runs on int8 codes."""
    from bigdl.nn.quantized import layers as Q
    from bigdl.nn.layers.table_ops import JoinTable
    m, _g = _inception_calibrated()
    q = m.quantize()
    joins = [n for n in q.forward_order if isinstance(n.element, JoinTable)]
    linked = [n for n in joins if n.element._i8_join]
    # 9 inception blocks; the last one feeds the average pooling (not a conv): stays float
    assert len(joins) == 9 and len(linked) == 8, (len(joins), len(linked))
    for n in linked:
        prods = []
        for p in n.prev_nodes:
            e = p.element if isinstance(p.element, Q.SpatialConvolution) else p.prev_nodes[0].element
            prods.append(e)
        assert len({c._out_qscale for c in prods}) == 1 and all(c._relu_fused for c in prods)
    # every 1×1 reduce conv feeding a 3×3 / 5×5 conv of its branch is linked
    reduces = [n.element for n in q.forward_order if isinstance(n.element, Q.SpatialConvolution)
               and n.element.get_name().startswith("inception_")
               and n.element.get_name().endswith(("3x3_reduce", "5x5_reduce"))]
    assert len(reduces) == 18
    # (the int8 kernel tiles channel counts % 16: the two 24-channel 5×5 reduces stay bf16-out)
    assert all(c._out_qscale is not None and c._relu_fused for c in reduces if c.nOutputPlane % 16 == 0)
    assert sum(c.nOutputPlane % 16 == 0 for c in reduces) == 16


@pytest.mark.gpu
def test_inception_int8_logits_track_fp32():
    """Calibrated int8 Inception-v1 on the GPU (int8 branch chains, int8 concats at unified scales) vs
    the float model: logit cosine ≥ 0.99 and the linked JoinTables really produce int8."""
    from bigdl.utils.engine import Engine
    from bigdl.utils import config
    from bigdl.nn.layers.table_ops import JoinTable
    config.set_property("bigdl.compute.dtype", "bf16")
    Engine.init(device="cuda:0")
    m, g = _inception_calibrated(seed=6)
    q = m.quantize().cuda()
    q.evaluate()
    x = torch.randn(8, 3, 224, 224, generator=g)
    with torch.no_grad():
        ref = m.forward(x).double()
        out = q.forward(x.cuda().bfloat16().contiguous(memory_format=torch.channels_last)).double().cpu()
    joins = [n.element for n in q.forward_order if isinstance(n.element, JoinTable) and n.element._i8_join]
    assert joins and all(j.output.dtype == torch.int8 for j in joins), [j.output.dtype for j in joins]
    ref, out = ref - ref.mean(1, keepdim=True), out - out.mean(1, keepdim=True)
    cos = float(torch.nn.functional.cosine_similarity(out.reshape(1, -1), ref.reshape(1, -1)))
    print("inception int8 vs fp32 logit cosine", cos)
    assert cos >= 0.99, cos
