"""GPU numerics: LRN forward/backward kernels (K18), conv epilogue ReLU + strided output slice,
zero-copy Inception concat — each vs the fp32 PyTorch reference of the same op."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = "cuda"


def _N():
    from bigdl.ops import native, native_status
    assert native_status()["loaded"]
    return native


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("C,size", [(64, 5), (192, 5), (24, 3), (16, 9), (8, 5)])
def test_lrn_forward_backward(C, size):
    N = _N()
    torch.manual_seed(0)
    x = _cl(torch.randn(3, C, 7, 5, device=dev) * 3).to(torch.bfloat16)
    x = _cl(x)
    gy = _cl(torch.randn(3, C, 7, 5, device=dev)).to(torch.bfloat16)
    gy = _cl(gy)
    alpha, beta, k = 1e-2, 0.75, 1.0
    y = N.lrn_forward(x, size, alpha, beta, k)
    assert y is not NotImplemented
    xr = x.float().requires_grad_(True)
    yr = F.local_response_norm(xr, size, alpha, beta, k)
    torch.testing.assert_close(y.float(), yr.detach(), rtol=2e-2, atol=2e-2)
    gx = N.lrn_backward(gy, x, size, alpha, beta, k)
    assert gx is not NotImplemented
    (gr,) = torch.autograd.grad(yr, xr, gy.float())
    torch.testing.assert_close(gx.float(), gr, rtol=3e-2, atol=3e-2)


def test_conv_relu_epilogue_and_slice_output():
    N = _N()
    torch.manual_seed(1)
    x = _cl(torch.randn(2, 64, 9, 9, device=dev)).to(torch.bfloat16)
    x = _cl(x)
    w = torch.randn(48, 64, 3, 3, device=dev) * 0.05
    b = torch.randn(48, device=dev)
    ref = torch.relu(F.conv2d(x.float(), w.to(torch.bfloat16).float(), b, 1, 1))
    y = N.conv2d_forward(x, w.to(torch.bfloat16), b, (1, 1), (1, 1), relu=True)
    assert y is not NotImplemented
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)
    big = torch.full((2, 80, 9, 9), 7.0, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    out = big[:, 16:64]
    y2 = N.conv2d_forward(x, w.to(torch.bfloat16), b, (1, 1), (1, 1), relu=True, out=out)
    assert y2 is not NotImplemented and y2.data_ptr() == out.data_ptr()
    torch.testing.assert_close(big[:, 16:64].float(), ref, rtol=2e-2, atol=2e-2)
    assert bool((big[:, :16] == 7).all()) and bool((big[:, 64:] == 7).all())  # neighbours untouched


def test_inception_zero_copy_concat_and_lrn_model():
    from bigdl.utils import config
    config.set_property("bigdl.compute.dtype", "bf16")
    from bigdl.models.inception import Inception_v1_NoAuxClassifier
    from bigdl.nn.fusion import fuse
    from bigdl.utils.random import RNG
    RNG.setSeed(3)
    ref_model = Inception_v1_NoAuxClassifier.graph(1000, has_dropout=False)
    ref_model.evaluate()
    x = torch.randn(2, 3, 224, 224)
    with torch.no_grad():
        ref = ref_model.forward(x).float().clone()
    m = ref_model.cuda()
    m.evaluate()
    fuse(m)
    xd = _cl(x.to(dev).to(torch.bfloat16))
    with torch.no_grad():
        y1 = m.forward(xd).float().cpu()   # plans record shapes
        y2 = m.forward(xd).float().cpu()   # zero-copy concats armed
    assert any(p.shapes for _, p in m._plans), "no concat plan recorded"
    torch.testing.assert_close(y1, y2, rtol=0, atol=0)
    # bf16 end-to-end vs the fp32 CPU model: log-probabilities agree to bf16 accuracy
    assert (y2 - ref).abs().max().item() < 0.15


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("n", [1 << 20, 1000003])
def test_dropout_regenerated_mask(dtype, n):
    N = _N()
    p = 0.3
    x = (torch.rand(n, device=dev) + 1.0).to(dtype)  # never exactly zero
    r = N.dropout_forward(x, p)
    assert r is not NotImplemented
    y, mask = r
    kept = y != 0
    frac = kept.float().mean().item()
    assert abs(frac - (1 - p)) < 5e-3, frac
    torch.testing.assert_close(y[kept].float(), (x[kept].float() / (1 - p)).to(dtype).float(), rtol=1e-2, atol=1e-2)
    gy = torch.randn(n, device=dev).to(dtype)
    gx = N.dropout_backward(gy, mask, p)
    assert torch.equal(gx != 0, kept & (gy != 0))
    # a new call draws a new seed
    y2, _ = N.dropout_forward(x, p)
    assert not torch.equal(y2 != 0, kept)


def test_dropout_layer_channels_last_backward():
    from bigdl.nn import Dropout
    d = Dropout(0.5)
    x = (torch.randn(4, 16, 8, 8, device=dev) + 3).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = d.forward(x)
    g = d.backward(x, torch.ones_like(y).contiguous())  # gradient arrives in the other layout
    assert torch.equal((g != 0), (y != 0))


def test_ir_resnet_inference_native():
    """IR lowering on the device: BN-folded convs with ReLU / residual-sum epilogues (bf16) vs the
    fp32 eval model on the CPU."""
    from bigdl.utils import config
    config.set_property("bigdl.compute.dtype", "bf16")
    from bigdl.models.resnet import ResNet, DatasetType, model_init
    from bigdl.utils.intermediate import ConversionUtils
    torch.manual_seed(0)
    m = model_init(ResNet(10, depth=20, dataset=DatasetType.CIFAR10))
    m.training()
    m.forward(torch.randn(8, 3, 32, 32))
    m.evaluate()
    x = torch.randn(16, 3, 32, 32)
    ref = m.forward(x).float().clone()
    ir = ConversionUtils.convert(m)
    ir.to(dev)
    with torch.no_grad():
        y = ir.forward(_cl(x.to(dev).to(torch.bfloat16))).float().cpu()
    assert (y - ref).abs().max().item() < 0.1
    assert (y.argmax(1) == ref.argmax(1)).float().mean().item() >= 0.9


def test_native_loader_to_device():
    """C++ batch loader → pinned slots → async H2D on a side stream (bf16, NHWC memory)."""
    import numpy as np
    from bigdl.runtime import NativeBatchLoader
    x = np.random.RandomState(0).randint(0, 256, size=(40, 16, 16, 3)).astype(np.uint8)
    y = np.arange(40, dtype=np.float32) + 1
    ld = NativeBatchLoader(x, y, 8, crop=(16, 16), pad=2, flip=True, train=True, dtype=torch.bfloat16,
                           layout="NHWC", mean=[125.0] * 3, std=[60.0] * 3, threads=4, prefetch=3, device=dev)
    seen = []
    for _ in range(10):
        b = ld.next_batch()
        xb = b.getInput()
        assert xb.is_cuda and xb.dtype == torch.bfloat16 and xb.shape == (8, 3, 16, 16)
        assert xb.is_contiguous(memory_format=torch.channels_last)
        seen.append(b.getTarget().cpu())
    torch.cuda.synchronize()
    assert sorted(torch.cat(seen[:5]).tolist()) == list(range(1, 41))
    ld.close()


@pytest.mark.parametrize("shadow", [False, True])
@pytest.mark.parametrize("nesterov", [False, True])
def test_sgd_per_element_decay_with_and_without_shadow(shadow, nesterov):
    """Fused SGD with per-element weight decays (folded L2 regularizers), with and without the bf16
    shadow output — the sharded fp32-wire DistriOptimizer update passes no shadow."""
    from bigdl.ops import reference as R
    N = _N()
    torch.manual_seed(0)
    n = 4096 + 64
    w = torch.randn(n, device=dev)
    g = torch.randn(n, device=dev)
    buf = torch.randn(n, device=dev)
    wds = torch.rand(n, device=dev)
    sh = torch.empty(n, dtype=torch.bfloat16, device=dev) if shadow else None
    w_ref, buf_ref = w.clone(), buf.clone()
    R.sgd_step(w_ref, g.clone(), buf_ref, 0.1, 0.9, 0.0, 1e-3, nesterov, False, 0.5, None, None, wds.clone())
    assert N.sgd_step(w, g, buf, 0.1, 0.9, 0.0, 1e-3, nesterov, False, 0.5, sh, None, wds) is not NotImplemented
    torch.testing.assert_close(w, w_ref, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(buf, buf_ref, rtol=1e-5, atol=1e-6)
    if shadow:
        torch.testing.assert_close(sh, w.to(torch.bfloat16), rtol=0, atol=0)


def test_hip_graph_train_step_vgg_like():
    """A LocalOptimizer step with conv/BN/ReLU/dropout/linear captured into a HIP graph: replays
    train (loss falls), draw fresh dropout masks each replay, and keep the host counters."""
    from bigdl.utils import config
    config.set_property("bigdl.compute.dtype", "bf16")
    from bigdl.nn import (Sequential, SpatialConvolution, SpatialBatchNormalization, ReLU, Dropout, View, Linear,
                          LogSoftMax, ClassNLLCriterion, SpatialMaxPooling)
    from bigdl.optim import SGD
    from bigdl.optim.optimizer import LocalOptimizer
    from bigdl.optim.graph_step import GraphedTrainStep
    from bigdl.dataset import MiniBatch
    torch.manual_seed(0)
    m = (Sequential().add(SpatialConvolution(3, 16, 3, 3, 1, 1, 1, 1)).add(SpatialBatchNormalization(16)).add(ReLU())
         .add(Dropout(0.3)).add(SpatialMaxPooling(2, 2, 2, 2)).add(View(16 * 8 * 8)).add(Linear(1024, 10))
         .add(LogSoftMax()))
    x = _cl(torch.randn(32, 3, 16, 16, device=dev).to(torch.bfloat16))
    y = (torch.randint(0, 10, (32,), device=dev) + 1).float()
    b = MiniBatch(x, y)
    opt = LocalOptimizer(m, [b], ClassNLLCriterion(), SGD(learningrate=0.05, momentum=0.9, dampening=0.0), batch_size=32)
    opt.prepare()
    g = GraphedTrainStep(opt, b)
    n0 = opt.state.get("neval", 0)
    drop = m.modules[3]
    losses, masks = [], []
    for _ in range(30):
        losses.append(float(g.step(b)))
        masks.append((drop.output != 0).clone())
    assert opt.state["neval"] == n0 + 30
    assert losses[-1] < losses[0]
    assert not torch.equal(masks[0], masks[1])


@pytest.mark.gpu
@pytest.mark.parametrize("K,C,R,S,stride", [(64, 32, 3, 3, 1), (72, 40, 7, 7, 2), (128, 64, 1, 1, 2), (48, 24, 3, 3, 2), (200, 136, 1, 1, 1)])
def test_dgrad_weight_transform_kernel(K, C, R, S, stride):
    """weight_xform.hip: every parity sub-filter W'[c][i][j][k] = W[k][c][rs[-1-i]][ss[-1-j]] in one
    launch, against the plain index gather."""
    from bigdl.ops import native_ops as NO
    w = torch.randn(K, R, S, C, device="cuda").to(torch.bfloat16).permute(0, 3, 1, 2)  # KRSC storage
    pad = R // 2
    classes = []
    for a in range(stride):
        rs = list(range((a + pad) % stride, R, stride))
        for b in range(stride):
            ss = list(range((b + pad) % stride, S, stride))
            classes.append((a, b, rs, ss))
    got = NO._subfilters(w, classes)
    for (a, b, rs, ss), g in zip(classes, got):
        if not rs or not ss:
            assert g is None
            continue
        ref = w[:, :, rs[::-1]][:, :, :, ss[::-1]].permute(1, 2, 3, 0)
        torch.testing.assert_close(g, ref, rtol=0, atol=0)


@pytest.mark.gpu
def test_hip_graph_step_fresh_batches_matches_eager():
    """A graphed step replayed on DIFFERENT batches (C = 3 stem → channel-padded input) must follow
    the eager trajectory exactly: the padded copy is produced inside the graph, never taken from a
    process-global cache (no Dropout, so both runs are deterministic)."""
    import copy
    from bigdl.utils import config
    config.set_property("bigdl.compute.dtype", "bf16")
    from bigdl.nn import (Sequential, SpatialConvolution, SpatialBatchNormalization, ReLU, View, Linear,
                          LogSoftMax, ClassNLLCriterion, SpatialMaxPooling)
    from bigdl.optim import SGD
    from bigdl.optim.optimizer import LocalOptimizer
    from bigdl.optim.graph_step import GraphedTrainStep
    from bigdl.dataset import MiniBatch
    torch.manual_seed(0)
    m = (Sequential().add(SpatialConvolution(3, 16, 3, 3, 1, 1, 1, 1)).add(SpatialBatchNormalization(16)).add(ReLU())
         .add(SpatialMaxPooling(2, 2, 2, 2)).add(View(16 * 8 * 8)).add(Linear(1024, 10)).add(LogSoftMax()))
    m2 = copy.deepcopy(m)
    bs = [MiniBatch(_cl(torch.randn(32, 3, 16, 16, device=dev).to(torch.bfloat16)),
                    (torch.randint(0, 10, (32,), device=dev) + 1).float()) for _ in range(4)]
    mk = lambda mm: LocalOptimizer(mm, [bs[0]], ClassNLLCriterion(), SGD(learningrate=0.05), batch_size=32)  # noqa
    eager, graphed = mk(m), mk(m2)
    eager.prepare()
    graphed.prepare()
    g = GraphedTrainStep(graphed, bs[0], warmup=3)  # warmup updates are undone after capture
    le = [float(eager.train_step(bs[i % 4])) for i in range(8)]
    lg = [float(g.step(bs[i % 4])) for i in range(8)]
    torch.testing.assert_close(torch.tensor(lg), torch.tensor(le), rtol=2e-2, atol=2e-2)
    assert len(set(round(v, 3) for v in lg[:4])) == 4, lg  # each replay saw its own batch
