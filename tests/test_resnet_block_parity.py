"""Per-bottleneck-block parity of the fused native bf16 ResNet-50 path against an fp32 host oracle,
on REAL mid-network activations (reference method: the fused DNN topology compared block by block
with the plain one, spark/dl/src/test/scala/.../nn/mkldnn/TopologySpec.scala:946-1057).

A ResNet-50 forward in fp32 on the host produces each block's input.  Every test takes a PAIR of
consecutive blocks — so the block-tail fusion across the boundary (the next block's first conv
applies the tail ReLU mask, sums the shortcut gradient and produces the tail BN's backward
reductions in its dgrad epilogue) is inside the unit under test — including every stage
transition (stride-2 3×3, strided 1×1 projection shortcut whose input gradient reaches the next
dgrad as a strided residual).  Forward output, input gradient and every parameter gradient must
agree with the fp32 oracle: cosine median > 0.95, minimum > 0.9 (bf16 activation storage is the
remaining difference).  BN γ are drawn in [0.5, 1.5] so no branch is switched off (with the
builder's zero-γ block tails the branch weights get exactly zero gradient)."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"
_CACHE = {}


def _cos(a, b):
    a, b = a.double().reshape(-1), b.double().reshape(-1)
    return float((a @ b) / (a.norm() * b.norm()).clamp_min(1e-30))


def _net():
    if "net" in _CACHE:
        return _CACHE["net"]
    from bigdl.utils import config
    from bigdl.utils.engine import Engine
    config.set_property("bigdl.compute.dtype", "bf16")
    Engine.init(device="cuda:0")
    from bigdl.models.resnet import ResNet, DatasetType, model_init
    from bigdl.nn import SpatialBatchNormalization, SpatialConvolution
    from bigdl.utils.random import RNG
    RNG.setSeed(11)
    torch.manual_seed(11)
    m = model_init(ResNet(100, depth=50, dataset=DatasetType.ImageNet, image_size=128))
    g = torch.Generator().manual_seed(5)
    with torch.no_grad():
        for mod in m.flattened_modules():
            if isinstance(mod, SpatialBatchNormalization):
                mod.weight.copy_(torch.rand(mod.weight.shape, generator=g) + 0.5)
                mod.bias.copy_(torch.rand(mod.bias.shape, generator=g) * 0.4 - 0.2)
            if isinstance(mod, SpatialConvolution) and mod.bias is not None:
                mod.bias.copy_(torch.rand(mod.bias.shape, generator=g) * 0.2 - 0.1)
        for w in m.parameters()[0]:
            w.copy_(w.to(torch.bfloat16).float())
    m.training()
    x = torch.randn(8, 3, 128, 128, generator=g)
    h = x
    blocks = []
    for mod in m.modules:
        if type(mod).__name__ == "Sequential" and mod.modules and type(mod.modules[0]).__name__ == "Sequential":
            for blk in mod.modules:  # a stage: Sequential of bottleneck blocks
                blocks.append((blk, h.detach().clone()))
                h = blk.forward(h)
        else:
            h = mod.forward(h)
            if type(mod).__name__ == "SpatialAveragePooling":
                break
    _CACHE["net"] = blocks
    return blocks


# (stage-local block index pairs as indices into the flat block list of ResNet-50: 3/4/6/3)
PAIRS = {"stage1_identity": (0, 1), "stage1_to_2": (2, 3), "stage2_identity": (4, 5), "stage2_to_3": (6, 7),
         "stage3_identity": (8, 9), "stage3_to_4": (12, 13), "stage4_identity": (14, 15)}


@pytest.mark.parametrize("name", list(PAIRS))
def test_block_pair_fused_bf16_matches_fp32(name):
    from bigdl.nn import Sequential
    from bigdl.nn.fusion import fuse
    from bigdl.utils.engine import Engine
    blocks = _net()
    i, j = PAIRS[name]
    (ba, xa), (bb, _) = blocks[i], blocks[j]
    ref = Sequential().add(copy.deepcopy(ba)).add(copy.deepcopy(bb))
    gpu = copy.deepcopy(ref)
    ref.training()
    ref.zeroGradParameters()
    yr = ref.forward(xa)
    g = torch.Generator().manual_seed(17)
    gy = torch.randn(yr.shape, generator=g)
    gxr = ref.backward(xa, gy)
    gpu.cuda()
    gpu.training()
    fuse(gpu)
    gpu.getParameters()
    gpu.flat_parameters().enable_shadow(Engine.compute_dtype())
    gpu.zeroGradParameters()
    xg = xa.to(dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    yg = gpu.forward(xg)
    gxg = gpu.backward(xg, gy.to(dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last))
    torch.cuda.synchronize()
    assert _cos(yg.float().cpu(), yr) > 0.99
    assert _cos(gxg.float().cpu(), gxr) > 0.95, _cos(gxg.float().cpu(), gxr)
    names = [f"{type(m).__name__}.{n}" for (m, n, _g) in ref._param_entries()]
    cos = [(nm, _cos(a.float().cpu(), b)) for nm, a, b in zip(names, gpu.parameters()[1], ref.parameters()[1])
           if not (nm.endswith(".bias") and "Convolution" in nm) and float(b.norm()) > 1e-8]
    cs = sorted(c for _, c in cos)
    assert cs[len(cs) // 2] > 0.95 and cs[0] > 0.9, sorted(cos, key=lambda t: t[1])[:5]


@pytest.mark.parametrize("mode", ["atomic", "replicas"])
@pytest.mark.parametrize("name", ["stage1_identity", "stage2_to_3", "stage4_identity"])
def test_atomic_bn_statistics_match_partials_path(name, mode):
    """bigdl.bn.atomicStats: the conv epilogues ADD the BN statistics (forward Σ, Σ²; backward Σg',
    Σg'·(x−μ)) into [2C] buffers and every BN is one finalize+apply launch.  Two training passes must
    match the per-tile-partials path (fold + finalize kernels) to summation-order rounding, and every
    buffer must be back to zero afterwards (the last arriving block re-zeroes it).  ``replicas``:
    bigdl.bn.statReplicas — the tiles add into 64 replicas and the finalize clears them.""" 
    from bigdl.nn import Sequential, SpatialBatchNormalization
    from bigdl.nn.fusion import fuse
    from bigdl.utils import config
    from bigdl.utils.engine import Engine
    blocks = _net()
    i, j = PAIRS[name]
    (ba, xa), (bb, _) = blocks[i], blocks[j]
    base = Sequential().add(copy.deepcopy(ba)).add(copy.deepcopy(bb))
    g = torch.Generator().manual_seed(23)
    out = {}
    prev = config.get_property("bigdl.bn.atomicStats")
    prev_rep = config.get_property("bigdl.bn.statReplicas")
    for atomic in (False, True):
        config.set_property("bigdl.bn.atomicStats", atomic and mode == "atomic")
        config.set_property("bigdl.bn.statReplicas", 64 if (atomic and mode == "replicas") else 0)
        try:
            m = copy.deepcopy(base).cuda()
            m.training()
            fuse(m)
            m.getParameters()
            m.flat_parameters().enable_shadow(Engine.compute_dtype())
            xg = xa.to(dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            ys = []
            for step in range(2):
                m.zeroGradParameters()
                y = m.forward(xg)
                gy = torch.randn(y.shape, generator=torch.Generator().manual_seed(100 + step)).to(dev)
                gx = m.backward(xg, gy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last))
                ys.append((y.float().cpu(), gx.float().cpu()))
            torch.cuda.synchronize()
            bns = [mod for mod in m.flattened_modules() if isinstance(mod, SpatialBatchNormalization)]
            if atomic:
                keys = ("_sums_fwd", "_sums_bwd") if mode == "atomic" else ("_rep_fwd", "_rep_bwd")
                # replica sets alternate per step (bigdl.bn.foldFinalize): the set the NEXT producer adds
                # into (the current one after the consumer's flip) must be zero
                bufs = []
                for mod in bns:
                    for k in keys:
                        v = mod.__dict__.get(k)
                        if isinstance(v, list):
                            v = v[mod.__dict__["_repi_" + k[len("_rep_"):]]]
                        bufs.append(v)
                assert sum(b is not None for b in bufs) >= len(bns), "the atomic path was not taken"
                assert all(b is None or float(b.abs().max()) == 0.0 for b in bufs), "sums not re-zeroed"
            # conv biases feeding a training BN have an exactly-zero gradient (the BN removes the
            # mean): what both paths produce there is rounding noise, so they are not compared
            names = [f"{type(mm).__name__}.{n}" for (mm, n, _g) in m._param_entries()]
            out[atomic] = ([(nm, p.float().cpu().clone()) for nm, p in zip(names, m.parameters()[1])
                            if not (nm.endswith(".bias") and "Convolution" in nm)], ys,
                           [torch.cat([b.runningMean, b.runningVar]).cpu() for b in bns])
        finally:
            config.set_property("bigdl.bn.atomicStats", prev)
            config.set_property("bigdl.bn.statReplicas", prev_rep)
    (ga, ya, ra), (gb, yb, rb) = out[False], out[True]
    for (y0, gx0), (y1, gx1) in zip(ya, yb):
        assert _cos(y1, y0) > 0.999 and _cos(gx1, gx0) > 0.995
    for a, b in zip(ra, rb):
        torch.testing.assert_close(b, a, rtol=2e-3, atol=2e-3)
    cs = sorted((_cos(b[1], a[1]), a[0]) for a, b in zip(ga, gb) if float(a[1].norm()) > 1e-8)
    assert cs[0][0] > 0.99, cs[:3]
