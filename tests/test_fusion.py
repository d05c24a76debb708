"""Fusion (conv-bias→BN fold, BN+ReLU, residual BN+add+ReLU) must not change the math."""
import copy

import pytest
import torch

from bigdl.models.resnet import ResNet, DatasetType, model_init
from bigdl.nn import CrossEntropyCriterion, Sequential, SpatialConvolution, SpatialBatchNormalization, ReLU
from bigdl.nn.fusion import fuse, unfuse


def _run(model, x, t):
    model.zeroGradParameters()
    y = model.forward(x)
    crit = CrossEntropyCriterion()
    loss = crit.forward(y, t)
    gi = model.backward(x, crit.backward(y, t))
    return y.clone(), gi.clone(), [g.clone() for g in model.parameters()[1]], \
        [b.clone() for b in model.getExtraParameter()]


@pytest.mark.parametrize("n_in,n,stride,proj", [(16, 4, 1, False), (8, 4, 2, True), (8, 4, 1, True)])
def test_fused_bottleneck_matches_unfused(n_in, n, stride, proj):
    """ImageNet ResNet bottleneck (ResNet.scala:199-222) with identity / projection shortcut."""
    from bigdl.models.resnet import Convolution, Sbn
    from bigdl.nn import ConcatTable, Identity
    torch.manual_seed(0)
    s = Sequential().add(Convolution(n_in, n, 1, 1)).add(Sbn(n)).add(ReLU(True))
    s.add(Convolution(n, n, 3, 3, stride, stride, 1, 1)).add(Sbn(n)).add(ReLU(True))
    s.add(Convolution(n, n * 4, 1, 1)).add(Sbn(n * 4))
    sc = Sequential().add(Convolution(n_in, n * 4, 1, 1, stride, stride)).add(Sbn(n * 4)) if proj else Identity()
    a = Sequential().add(ConcatTable().add(s).add(sc)).add(CAddTable(True)).add(ReLU(True))
    for m in a.flattened_modules():
        if isinstance(m, SpatialConvolution) and m.bias is not None:
            m.bias.uniform_(-0.1, 0.1)
        if isinstance(m, SpatialBatchNormalization):
            m.weight.uniform_(0.5, 1.5)
            m.bias.uniform_(-0.2, 0.2)
    b = copy.deepcopy(a)
    fuse(b)
    x = torch.randn(4, n_in, 6, 6)
    ya, yb = a.forward(x), b.forward(x)
    gy = torch.randn_like(ya)
    ga, gb = a.backward(x, gy), b.backward(x, gy)
    torch.testing.assert_close(yb, ya, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(gb, ga, rtol=1e-5, atol=1e-5)
    for u, v in zip(b.parameters()[1], a.parameters()[1]):
        torch.testing.assert_close(u, v, rtol=1e-4, atol=1e-4)


from bigdl.nn import CAddTable  # noqa: E402


@pytest.mark.parametrize("dataset,depth,shape", [(DatasetType.CIFAR10, 20, (2, 3, 32, 32))])
def test_fused_resnet_matches_unfused(dataset, depth, shape):
    torch.manual_seed(0)
    a = model_init(ResNet(10, depth=depth, dataset=dataset))
    if dataset == DatasetType.ImageNet:
        # make the 7x7 global pool valid for the small input; avg-pool the stem so ~1e-7 rounding
        # differences (folded vs added conv bias) cannot flip a max-pool argmax
        from bigdl.nn import SpatialAveragePooling
        a.modules[-3] = SpatialAveragePooling(2, 2, 1, 1)
        a.modules[3] = SpatialAveragePooling(3, 3, 2, 2, 1, 1)
    # non-zero biases and BN stats so every fused path is exercised
    for m in a.flattened_modules():
        if isinstance(m, SpatialConvolution) and m.bias is not None:
            m.bias.uniform_(-0.1, 0.1)
        if isinstance(m, SpatialBatchNormalization):
            m.weight.uniform_(0.5, 1.5)
            m.bias.uniform_(-0.2, 0.2)
    b = copy.deepcopy(a)
    fuse(b)
    assert any(getattr(m, "_residual", None) for m in b.flattened_modules())
    x = torch.randn(*shape)
    t = torch.randint(1, 11, (shape[0],)).float()
    ya, ga, pa, ea = _run(a, x, t)
    yb, gb, pb, eb = _run(b, x, t)
    torch.testing.assert_close(yb, ya, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(gb, ga, rtol=1e-3, atol=1e-5)
    for u, v in zip(pb, pa):
        torch.testing.assert_close(u, v, rtol=1e-3, atol=2e-5)
    for u, v in zip(eb, ea):  # running stats (running mean includes the folded conv bias)
        torch.testing.assert_close(u, v, rtol=1e-4, atol=1e-5)
    # eval mode too
    a.evaluate()
    b.evaluate()
    torch.testing.assert_close(b.forward(x), a.forward(x), rtol=1e-4, atol=1e-4)


def test_unfuse_restores_flags():
    m = Sequential().add(SpatialConvolution(3, 8, 3, 3)).add(SpatialBatchNormalization(8)).add(ReLU())
    fuse(m)
    assert m.modules[2]._passthrough and m.modules[1]._fused_relu
    unfuse(m)
    assert not m.modules[2]._passthrough and not m.modules[1]._fused_relu


def test_shortcut_bn_deferred_flag_on_projection_blocks():
    """fuse() marks the BN of a conv → BN projection shortcut for the deferred apply (the fused tail
    applies it); identity shortcuts have no such BN; unfuse() clears the flag."""
    from bigdl.models.resnet import ResNet, DatasetType
    from bigdl.nn.fusion import fuse, unfuse
    from bigdl.nn.layers.normalization import BatchNormalization
    m = ResNet(10, depth=50, dataset=DatasetType.ImageNet)
    fuse(m)
    flagged = [b for b in m.flattened_modules() if isinstance(b, BatchNormalization) and b._defer_ok]
    assert len(flagged) == 4  # one projection shortcut per stage
    unfuse(m)
    assert not any(getattr(b, "_defer_ok", False) for b in m.flattened_modules() if isinstance(b, BatchNormalization))


def test_bnout_dense_is_the_affine_map():
    """A deferred BN output materialises as x·scale + shift per channel (NCHW logical, channels-last)."""
    from bigdl.ops.reference import BNOut
    torch.manual_seed(0)
    x = torch.randn(2, 8, 5, 6).contiguous(memory_format=torch.channels_last)
    coef = torch.randn(16)
    y = BNOut(x, coef).dense()
    ref = x * coef[:8].view(1, 8, 1, 1) + coef[8:].view(1, 8, 1, 1)
    assert y.shape == x.shape and y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y, ref)
    assert BNOut(x, coef).dim() == 4 and BNOut(x, coef).shape == tuple(x.shape)
