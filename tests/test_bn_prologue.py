"""Deferred BatchNorm input gradients (ops.reference.BNGrad): a BN whose producer is a 1×1 stride-1
conv hands it A·g + B·x + Cc unapplied, and the conv's backward-data (conv_igemm.hip AT prologue)
and weight-gradient (conv_wgrad.hip AT prologue) kernels apply it while loading their operands.
The values entering the MFMAs are the same bf16 roundings the separate apply pass wrote, so a
ResNet-50 stage run with the prologue must reproduce the materialised path — and launch fewer
BN apply kernels."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _partials_stats():
    """Bit-exact comparisons: per-tile statistics partials (atomic accumulation order varies)."""
    from bigdl.utils import config
    prev = config.get_property("bigdl.bn.atomicStats")
    config.set_property("bigdl.bn.atomicStats", False)
    yield
    config.set_property("bigdl.bn.atomicStats", prev)


def _run(model, x, gy, prologue):
    from bigdl.utils import config
    config.set_property("bigdl.fusion.bnprologue", prologue)
    try:
        model.zeroGradParameters()
        with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
            y = model.forward(x).float().cpu()
            gi = model.backward(x, gy)
            torch.cuda.synchronize()
    finally:
        config.set_property("bigdl.fusion.bnprologue", 0)
    names = [e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA]
    return y, gi.float().cpu(), [g.float().cpu().clone() for g in model.parameters()[1]], names


def test_resnet_stage_prologue_matches_materialised():
    from bigdl.models.resnet import ResNet, DatasetType, model_init
    from bigdl.nn.fusion import fuse
    from bigdl.utils import config
    from bigdl.utils.engine import Engine
    from bigdl.utils.random import RNG
    config.set_property("bigdl.compute.dtype", "bf16")
    Engine.init(device="cuda:0")
    RNG.setSeed(5)
    m = model_init(ResNet(10, depth=50, dataset=DatasetType.ImageNet, image_size=64))
    m.cuda()
    m.training()
    fuse(m)
    m.getParameters()
    m.flat_parameters().enable_shadow(torch.bfloat16)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(8, 3, 64, 64, generator=g).cuda().bfloat16().contiguous(memory_format=torch.channels_last)
    y0 = m.forward(x)
    gy = torch.randn(y0.shape, generator=g).cuda().to(y0.dtype)
    # the conv-epilogue BN statistics are shifted by the running mean, which every training forward
    # moves: restore it so both runs round identically
    extra = [e.clone() for e in m.getExtraParameter()]

    def reset():
        for e, v in zip(m.getExtraParameter(), extra):
            e.copy_(v)
        for mod in m.flattened_modules():  # the statistics-shift ring restarts from the running mean
            mod.__dict__.pop("_kbuf", None)
    reset()
    ya, ga, pa, na = _run(m, x, gy, 0)
    reset()
    yb, gb, pb, nb = _run(m, x, gy, 2)
    torch.testing.assert_close(yb, ya, rtol=0, atol=0)
    torch.testing.assert_close(gb, ga, rtol=1e-3, atol=1e-3)
    worst = max(float((u - v).norm() / v.norm().clamp_min(1e-12)) for u, v in zip(pb, pa))
    assert worst < 1e-3, worst
    import re
    # the BN-backward prologue instantiations: k_conv_fwd<…, AT = true> and k_conv_wgrad<…, AT = true, …>
    at = [n for n in nb if re.search(r"k_conv_fwd<\d+, \d+, \d+, \d+, \w+, true>", n)
          or re.search(r"k_conv_wgrad<\d+, \d+, \d+, \w+, \w+, true", n) or "Lb0ELb1E" in n]
    assert any("k_conv_fwd" in n for n in at) and any("k_conv_wgrad" in n for n in at), sorted(set(nb))
    apply_a = sum("k_bn_bwd_apply" in n for n in na)
    apply_b = sum("k_bn_bwd_apply" in n for n in nb)
    assert apply_b < apply_a, (apply_a, apply_b)
