"""No silent fallbacks: one training step (or inference batch) of each BASELINE.json config's model on
the GPU must run every dispatched op on a HIP kernel — ``ops.fallback_counts()`` stays empty.

LeNet-5 (MNIST shape), VggForCifar10, ResNet-50 (ImageNet topology, small batch), the PTB 2-layer
LSTM LM and Inception-v1 inference; small batches so the test stays a few seconds."""
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"


@pytest.fixture(autouse=True)
def _setup():
    from bigdl.utils import config
    from bigdl.utils.engine import Engine
    config.set_property("bigdl.compute.dtype", "bf16")
    Engine.init(device="cuda:0")
    from bigdl import ops
    assert ops.native_status()["loaded"]
    ops.reset_fallbacks()
    yield
    config.set_property("bigdl.compute.dtype", "auto")


def _train_steps(model, x, y, crit, method, n=2):
    from bigdl.dataset import MiniBatch
    from bigdl.optim.optimizer import LocalOptimizer
    opt = LocalOptimizer(model, [MiniBatch(x, y)], crit, method, batch_size=x.shape[0])
    opt.prepare()
    losses = [float(opt.train_step(MiniBatch(x, y))) for _ in range(n)]
    torch.cuda.synchronize()
    assert all(l == l for l in losses), losses
    return losses


def _assert_clean():
    from bigdl import ops
    fb = ops.fallback_counts()
    assert fb == {}, "device ops fell back to torch: " + "; ".join(f"{k}: {v}" for k, v in fb.items())


def _img(b, c, h, w):
    from bigdl.utils.engine import Engine
    return torch.randn(b, c, h, w, device=dev).to(Engine.compute_dtype()).contiguous(memory_format=torch.channels_last)


def test_lenet_step_native():
    from bigdl.models.lenet import LeNet5
    from bigdl.nn import ClassNLLCriterion
    from bigdl.optim import SGD
    x = _img(16, 1, 28, 28)
    y = (torch.randint(0, 10, (16,)) + 1).float().to(dev)
    _train_steps(LeNet5(10), x, y, ClassNLLCriterion(), SGD(learningrate=0.05))
    _assert_clean()


def test_vgg_cifar_step_native():
    from bigdl.models.vgg import VggForCifar10
    from bigdl.nn import ClassNLLCriterion
    from bigdl.optim import SGD
    x = _img(16, 3, 32, 32)
    y = (torch.randint(0, 10, (16,)) + 1).float().to(dev)
    _train_steps(VggForCifar10(10), x, y, ClassNLLCriterion(), SGD(learningrate=0.01, momentum=0.9, dampening=0.0))
    _assert_clean()


def test_resnet50_step_native():
    from bigdl.models.resnet import ResNet, DatasetType, model_init
    from bigdl.nn import CrossEntropyCriterion
    from bigdl.optim import SGD
    x = _img(4, 3, 224, 224)
    y = (torch.randint(0, 1000, (4,)) + 1).float().to(dev)
    model = model_init(ResNet(1000, depth=50, dataset=DatasetType.ImageNet))
    _train_steps(model, x, y, CrossEntropyCriterion(),
                 SGD(learningrate=0.1, momentum=0.9, dampening=0.0, nesterov=True, weightdecay=1e-4))
    _assert_clean()


def test_ptb_lstm_step_native():
    from bigdl.models.rnn import PTBModel
    from bigdl.nn import CrossEntropyCriterion, TimeDistributedCriterion
    from bigdl.optim import Adagrad
    V, B, T = 10000, 20, 20
    x = (torch.randint(0, V, (B, T)) + 1).float().to(dev)
    y = (torch.randint(0, V, (B, T)) + 1).float().to(dev)
    crit = TimeDistributedCriterion(CrossEntropyCriterion(), size_average=False)
    _train_steps(PTBModel.lstm(V, 200, V, 2), x, y, crit, Adagrad(learningrate=0.01, learningrate_decay=0.001))
    _assert_clean()


def test_inception_v1_inference_native():
    from bigdl.models.inception import Inception_v1_NoAuxClassifier
    from bigdl.nn.fusion import fuse
    model = Inception_v1_NoAuxClassifier.graph(1000, has_dropout=True)
    model.cuda()
    model.evaluate()
    fuse(model)
    with torch.no_grad():
        out = model.forward(_img(4, 3, 224, 224))
    torch.cuda.synchronize()
    assert out.shape == (4, 1000)
    _assert_clean()


def test_grouped_conv_model_step_native():
    """An AlexNet-style grouped-convolution stack (nGroup = 2) trains through the native kernels."""
    import bigdl.nn as nn
    from bigdl.nn import ClassNLLCriterion
    from bigdl.optim import SGD
    m = nn.Sequential()
    m.add(nn.SpatialConvolution(3, 32, 3, 3, 1, 1, 1, 1)).add(nn.ReLU())
    m.add(nn.SpatialConvolution(32, 64, 3, 3, 1, 1, 1, 1, n_group=2)).add(nn.ReLU())
    m.add(nn.SpatialConvolution(64, 64, 3, 3, 2, 2, 1, 1, n_group=4)).add(nn.ReLU())
    m.add(nn.SpatialAveragePooling(8, 8, 8, 8)).add(nn.View(64)).add(nn.Linear(64, 10)).add(nn.LogSoftMax())
    x = _img(8, 3, 16, 16)
    y = (torch.randint(0, 10, (8,)) + 1).float().to(dev)
    _train_steps(m, x, y, ClassNLLCriterion(), SGD(learningrate=0.05))
    _assert_clean()


def test_separable_conv_native_matches_torch():
    """SpatialSeparableConvolution (depthwise + pointwise) through the native depthwise stencil and
    MFMA conv kernels as autograd ops: forward and gradients vs the torch fp32 composition."""
    import bigdl.nn as nn
    from bigdl import ops
    ops.reset_fallbacks()
    torch.manual_seed(0)
    m = nn.SpatialSeparableConvolution(32, 64, 1, 3, 3, 1, 1, 1, 1).to(device=dev)
    x = torch.randn(4, 32, 12, 12, device=dev)
    xb = x.bfloat16().contiguous(memory_format=torch.channels_last)
    y = m.forward(xb)
    gy = torch.randn_like(y.float())
    gi = m.backward(xb, gy.bfloat16().contiguous(memory_format=torch.channels_last))
    dw, pw, b = (m.depthWeight.detach().float().clone().requires_grad_(True),
                 m.pointWeight.detach().float().clone().requires_grad_(True),
                 m.bias.detach().float().clone().requires_grad_(True))
    xr = xb.float().requires_grad_(True)
    ref = torch.nn.functional.conv2d(torch.nn.functional.conv2d(xr, dw, None, 1, 1, 1, 32), pw, b)
    ref.backward(gy)
    torch.testing.assert_close(y.float(), ref.detach(), rtol=3e-2, atol=5e-2)
    torch.testing.assert_close(gi.float(), xr.grad, rtol=3e-2, atol=5e-2)
    _assert_clean()


def test_temporal_conv_native_matches_torch():
    """TemporalConvolution (1-D conv over frames) as the 2-D native conv with a 1×kW filter on the
    same NHWC memory: forward and input/weight gradients vs torch conv1d."""
    import bigdl.nn as nn
    from bigdl import ops
    ops.reset_fallbacks()
    torch.manual_seed(0)
    m = nn.TemporalConvolution(64, 32, 3, 1).to(device=dev)
    x = torch.randn(4, 20, 64, device=dev).bfloat16()
    y = m.forward(x)
    gy = torch.randn(y.shape, device=dev)
    m.zeroGradParameters()
    gi = m.backward(x, gy.bfloat16())
    xr = x.float().requires_grad_(True)
    w = m.weight.detach().float().view(32, 3, 64).permute(0, 2, 1).contiguous().bfloat16().float().requires_grad_(True)
    b = m.bias.detach().float().requires_grad_(True)
    ref = torch.nn.functional.conv1d(xr.transpose(1, 2), w, b, 1).transpose(1, 2)
    ref.backward(gy.bfloat16().float())
    torch.testing.assert_close(y.float(), ref.detach(), rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(gi.float(), xr.grad, rtol=2e-2, atol=3e-2)
    gw = m.gradWeight.float().view(32, 3, 64).permute(0, 2, 1)
    torch.testing.assert_close(gw, w.grad, rtol=3e-2, atol=3e-2 * float(w.grad.abs().max()))
    _assert_clean()


# ------------------------------------------------------------------------------------------- fp32 (bf16x3)
class _NoTorchConv:
    """Makes the torch conv entry points raise while active: an fp32 training step must run every
    convolution (forward, data and weight gradients) on the bf16x3 HIP kernels, never MIOpen."""

    def __enter__(self):
        import torch.nn.functional as F
        self.saved = [(F, "conv2d", F.conv2d), (torch, "conv2d", torch.conv2d),
                      (torch.nn.grad, "conv2d_input", torch.nn.grad.conv2d_input),
                      (torch.nn.grad, "conv2d_weight", torch.nn.grad.conv2d_weight)]

        def boom(*a, **k):
            raise AssertionError("torch / MIOpen convolution called on the fp32 path")
        for mod, name, _ in self.saved:
            setattr(mod, name, boom)
        return self

    def __exit__(self, *exc):
        for mod, name, fn in self.saved:
            setattr(mod, name, fn)


def _fp32():
    from bigdl.utils import config
    from bigdl.utils.engine import Engine
    config.set_property("bigdl.compute.dtype", "fp32")
    Engine.set_compute_dtype("fp32")


def test_resnet50_fp32_step_native():
    from bigdl.models.resnet import ResNet, DatasetType, model_init
    from bigdl.nn import CrossEntropyCriterion
    from bigdl.optim import SGD
    _fp32()
    try:
        x = torch.randn(4, 3, 224, 224, device=dev)
        y = (torch.randint(0, 1000, (4,)) + 1).float().to(dev)
        model = model_init(ResNet(1000, depth=50, dataset=DatasetType.ImageNet))
        with _NoTorchConv():
            _train_steps(model, x, y, CrossEntropyCriterion(),
                         SGD(learningrate=0.1, momentum=0.9, dampening=0.0, nesterov=True, weightdecay=1e-4))
        _assert_clean()
    finally:
        from bigdl.utils.engine import Engine
        Engine.set_compute_dtype("bf16")


def test_vgg_cifar_fp32_step_native():
    from bigdl.models.vgg import VggForCifar10
    from bigdl.nn import ClassNLLCriterion
    from bigdl.optim import SGD
    _fp32()
    try:
        x = torch.randn(16, 3, 32, 32, device=dev)
        y = (torch.randint(0, 10, (16,)) + 1).float().to(dev)
        with _NoTorchConv():
            _train_steps(VggForCifar10(10), x, y, ClassNLLCriterion(),
                         SGD(learningrate=0.01, momentum=0.9, dampening=0.0))
        _assert_clean()
    finally:
        from bigdl.utils.engine import Engine
        Engine.set_compute_dtype("bf16")


def test_lenet_fp32_step_native():
    """Config 1 at the reference's precision on the GPU: odd channel counts (6 / 12 maps, a 1-channel
    input) take the split-operand bf16x3 kernels; Tanh, max pooling, Linear, LogSoftMax / NLL native."""
    from bigdl.models.lenet import LeNet5
    from bigdl.nn import ClassNLLCriterion
    from bigdl.optim import SGD
    _fp32()
    try:
        x = torch.randn(16, 1, 28, 28, device=dev)
        y = (torch.randint(0, 10, (16,)) + 1).float().to(dev)
        with _NoTorchConv():
            _train_steps(LeNet5(10), x, y, ClassNLLCriterion(), SGD(learningrate=0.05))
        _assert_clean()
    finally:
        from bigdl.utils.engine import Engine
        Engine.set_compute_dtype("bf16")


def test_ptb_lstm_fp32_step_native():
    """Config 4 at the reference's precision: fp32 embedding, the bf16x3 LSTM step kernels, fp32
    TimeDistributed Linear + cross entropy, the fused Adagrad."""
    from bigdl.models.rnn import PTBModel
    from bigdl.nn import CrossEntropyCriterion, TimeDistributedCriterion
    from bigdl.optim import Adagrad
    _fp32()
    try:
        V, B, T = 10000, 20, 20
        x = (torch.randint(0, V, (B, T)) + 1).float().to(dev)
        y = (torch.randint(0, V, (B, T)) + 1).float().to(dev)
        crit = TimeDistributedCriterion(CrossEntropyCriterion(), size_average=False)
        _train_steps(PTBModel.lstm(V, 200, V, 2), x, y, crit, Adagrad(learningrate=0.01, learningrate_decay=0.001))
        _assert_clean()
    finally:
        from bigdl.utils.engine import Engine
        Engine.set_compute_dtype("bf16")


def test_inception_v1_fp32_inference_native():
    """Config 5 at the reference's precision: the s2d stem, bf16x3 convs, native fp32 LRN
    (SpatialCrossMapLRN.scala:96-200), pooling, concat and the classifier — no torch compute."""
    from bigdl.models.inception import Inception_v1_NoAuxClassifier
    from bigdl.nn.fusion import fuse
    _fp32()
    try:
        model = Inception_v1_NoAuxClassifier.graph(1000, has_dropout=True)
        model.cuda()
        model.evaluate()
        fuse(model)
        x = torch.randn(4, 3, 224, 224, device=dev)
        with _NoTorchConv(), torch.no_grad():
            out = model.forward(x)
        torch.cuda.synchronize()
        assert out.shape == (4, 1000) and out.dtype == torch.float32
        assert bool(torch.isfinite(out).all())
        _assert_clean()
    finally:
        from bigdl.utils.engine import Engine
        Engine.set_compute_dtype("bf16")


def test_lrn_fp32_kernel_matches_fp64():
    """fp32 LRN forward / backward (csrc/lrn.hip, float instantiation) against torch fp64."""
    import bigdl.nn as nn
    from bigdl.ops import native_ops as NO
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 64, 7, 9, generator=g)
    xr = x.double().requires_grad_(True)
    ref = torch.nn.functional.local_response_norm(xr, 5, 1e-4 * 5 / 5, 0.75, 1.0)
    gy = torch.randn(ref.shape, generator=g)
    ref.backward(gy.double())
    xd = x.to(dev).contiguous(memory_format=torch.channels_last)
    y = NO.lrn_forward(xd, 5, 1e-4, 0.75, 1.0)
    gi = NO.lrn_backward(gy.to(dev).contiguous(memory_format=torch.channels_last), xd, 5, 1e-4, 0.75, 1.0)
    torch.cuda.synchronize()
    assert y is not NotImplemented and gi is not NotImplemented
    torch.testing.assert_close(y.double().cpu(), ref.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(gi.double().cpu(), xr.grad, rtol=1e-5, atol=1e-6)
