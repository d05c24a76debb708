"""Two-phase execution (nn/compiled.py; reference nn/mkldnn/DnnGraph.scala compile(phase)):
the shape / layout / workspace plan on the host, and the HIP-graph executor on a GPU."""
import pytest
import torch


def _cnn():
    import bigdl.nn as nn
    m = nn.Sequential()
    m.add(nn.SpatialConvolution(3, 8, 3, 3, 1, 1, 1, 1)).add(nn.SpatialBatchNormalization(8)).add(nn.ReLU())
    m.add(nn.SpatialMaxPooling(2, 2, 2, 2)).add(nn.SpatialConvolution(8, 16, 3, 3, 1, 1, 1, 1)).add(nn.ReLU())
    m.add(nn.View(16 * 8 * 8)).add(nn.Linear(16 * 8 * 8, 10)).add(nn.LogSoftMax())
    return m


def test_plan_shapes_and_workspace():
    from bigdl.nn.compiled import plan
    m = _cnn()
    x = torch.randn(4, 3, 16, 16)
    p = plan(m, x, "inference")
    kinds = [r.kind for r in p.layers]
    assert kinds[0] == "SpatialConvolution" and kinds[-1] == "LogSoftMax"
    assert p.layers[0].out_shapes[0] == (4, 8, 16, 16)
    assert p.layers[-1].out_shapes[0] == (4, 10)
    # inference frees buffers after their last use: peak and arena below the sum of all outputs
    assert 0 < p.peak_bytes <= p.arena_bytes <= p.total_bytes
    assert p.peak_bytes < p.total_bytes
    # no two buffers that are live at the same time overlap in the arena
    for a in p.buffers:
        for b in p.buffers:
            if a is b or a.last < b.first or b.last < a.first:
                continue
            assert a.offset + a.nbytes <= b.offset or b.offset + b.nbytes <= a.offset
    tr = plan(m, x, "training")
    assert tr.peak_bytes >= p.peak_bytes and tr.peak_bytes == tr.total_bytes
    assert m.isTraining()  # planning restores the mode
    assert "LogSoftMax" in p.summary()


def test_compiled_eager_on_host_matches_model():
    from bigdl.nn.compiled import compile
    m = _cnn()
    x = torch.randn(2, 3, 16, 16)
    c = compile(m, x)
    assert not c.captured
    m.evaluate()
    torch.testing.assert_close(c(x), m.forward(x))


@pytest.mark.gpu
def test_compiled_hip_graph_inference():
    from bigdl.nn.compiled import compile
    from bigdl.utils.engine import Engine
    from bigdl.models.resnet import ResNet
    Engine.init(device="cuda:0")
    torch.manual_seed(0)
    m = ResNet(10, depth=20).to(device="cuda")
    x = torch.randn(8, 3, 32, 32, device="cuda")
    c = compile(m, x)
    assert c.captured
    for seed in (1, 2):
        xi = torch.randn(8, 3, 32, 32, device="cuda", generator=torch.Generator("cuda").manual_seed(seed))
        m.evaluate()
        with torch.no_grad():
            ref = m.forward(xi).float().clone()
        got = c(xi).float()
        torch.testing.assert_close(got, ref, rtol=2e-2, atol=2e-2)
    p = c.plan
    assert any(r.out_layout == "NHWC" for r in p.layers)  # the conv path's device layout
    assert p.reorders  # NCHW input → NHWC conv output at least once
    # the graph's pool was reserved as one slab sized from the plan's first-fit arena
    assert c.arena_reserved >= p.arena_bytes > 0


@pytest.mark.gpu
def test_compile_autotune_pins_tiles_and_keeps_outputs():
    """Kernel selection: every recorded conv geometry is timed under the tile candidates; pinned
    choices are valid launcher tiles and the tuned, captured forward still matches eager."""
    from bigdl.nn.compiled import compile, autotune
    from bigdl.ops import native_ops as NO
    from bigdl.utils.engine import Engine
    from bigdl.models.resnet import ResNet
    Engine.init(device="cuda:0")
    torch.manual_seed(0)
    lib = NO._lib()
    assert lib.bigdl_conv_tile_ok(96, 0, 0) != 0 and lib.bigdl_conv_tile_ok(0, 32, 256) != 0
    assert lib.bigdl_conv_tile_ok(0, 0, 0) == 0
    m = ResNet(10, depth=20).to(device="cuda")
    x = torch.randn(64, 3, 32, 32, device="cuda")
    NO.conv_tile_table().clear()
    chosen = autotune(m, x, iters=2, min_gain=-1.0)  # pin the fastest candidate for every geometry
    assert chosen and all(t in __import__("bigdl.nn.compiled", fromlist=["x"]).TILE_CANDIDATES for t in chosen.values())
    assert set(chosen) <= set(NO.conv_tile_table())
    m.evaluate()
    with torch.no_grad():
        ref = m.forward(x).float().clone()
    NO.conv_tile_table().clear()
    with torch.no_grad():
        ref0 = m.forward(x).float().clone()
    torch.testing.assert_close(ref, ref0, rtol=2e-2, atol=2e-2)
    c = compile(m, x)
    assert c.captured
    torch.testing.assert_close(c(x).float(), ref0, rtol=2e-2, atol=2e-2)
    NO.conv_tile_table().clear()


@pytest.mark.gpu
def test_training_compile_phase_pins_fwd_dgrad_wgrad_and_keeps_training():
    """Training compile phase: the first iteration records forward, backward-data and weight-gradient
    launches; pinning the fastest candidate for EVERY geometry (min_gain < 0: every candidate family,
    including the 32x32x16 conv tiles and the wgrad split / depth choices, ends up in use) must leave
    training numerically where the heuristic kernels put it."""
    import copy
    from bigdl.nn.compiled import autotune_training_step, TILE_CANDIDATES, WGRAD_CANDIDATES, WGRAD_EXTRA
    from bigdl.ops import native_ops as NO
    from bigdl.utils.engine import Engine
    from bigdl.utils import config
    from bigdl.models.resnet import ResNet, model_init
    from bigdl.nn import CrossEntropyCriterion
    from bigdl.optim import SGD
    from bigdl.optim.optimizer import LocalOptimizer
    from bigdl.dataset import MiniBatch
    config.set_property("bigdl.compute.dtype", "bf16")
    Engine.init(device="cuda:0")
    torch.manual_seed(0)
    base = model_init(ResNet(10, depth=20))
    g = torch.Generator().manual_seed(4)
    x = torch.randn(64, 3, 32, 32, generator=g).cuda()
    y = (torch.randint(0, 10, (64,), generator=g) + 1).float().cuda()

    def run(tune):
        NO.conv_tile_table().clear()
        m = copy.deepcopy(base)
        opt = LocalOptimizer(m, [MiniBatch(x, y)], CrossEntropyCriterion(), SGD(learningrate=0.05, momentum=0.9))
        opt.prepare()
        opt._kernels_selected = True  # drive the phase by hand below
        chosen = {}
        if tune:
            _, chosen = autotune_training_step(lambda: opt._train_step_run(MiniBatch(x, y)), iters=1, min_gain=-1.0)
        else:
            opt._train_step_run(MiniBatch(x, y))
        for _ in range(2):
            loss = opt._train_step_run(MiniBatch(x, y))
        torch.cuda.synchronize()
        w = torch.cat([p.reshape(-1).float() for p in m.parameters()[0]])
        return float(loss), w, chosen

    l0, w0, _ = run(False)
    l1, w1, chosen = run(True)
    kinds = {"wg" if k[0] == "wg" else "conv" for k in chosen}
    assert kinds == {"wg", "conv"}, chosen
    assert all(v in (WGRAD_CANDIDATES + WGRAD_EXTRA if k[0] == "wg" else TILE_CANDIDATES) for k, v in chosen.items())
    rel = float((w1 - w0).norm() / w0.norm())
    assert rel < 2e-2 and abs(l1 - l0) < 0.05 * max(1.0, abs(l0)), (rel, l0, l1)
    NO.conv_tile_table().clear()


@pytest.mark.gpu
def test_compiled_inference_lowers_through_ir_and_predictors_use_it():
    """compile(model, x) in the inference phase lowers through the IR first (BN folded into the convs,
    conv+sum+ReLU epilogues), captures the lowered forward, and matches the eager UNFUSED model within
    bf16 tolerance; LocalPredictor uses the same lowered + captured form by default on a GPU
    (reference: LocalPredictor.scala:66, Predictor.scala:131,165 → ConversionUtils.convert)."""
    import bigdl.nn as nn
    from bigdl.nn.compiled import compile
    from bigdl.nn.fusion import unfuse
    from bigdl.optim.predictor import LocalPredictor
    from bigdl.utils.engine import Engine
    from bigdl.models.resnet import ResNet, DatasetType, model_init
    from bigdl.utils.intermediate import IRGraph
    Engine.init(device="cuda:0")
    torch.manual_seed(0)
    m = model_init(ResNet(1000, depth=50, dataset=DatasetType.ImageNet))
    m.training()
    with torch.no_grad():  # real running statistics, so the folded BN is not the identity
        m.forward(torch.randn(2, 3, 224, 224))
    m.to(device="cuda")
    m.evaluate()
    x = torch.randn(4, 3, 224, 224, device="cuda")
    unfuse(m)
    with torch.no_grad():
        ref = m.forward(x).float().clone()
    c = compile(m, x)
    assert c.lowered and isinstance(c.model, IRGraph) and c.captured
    kinds = {type(mm).__name__ for mm in c.model._need().flattened_modules()}
    assert "FusedConvSum" in kinds and "SpatialBatchNormalization" not in kinds
    got = c(x).float()
    rel = float((got - ref).norm() / ref.norm())
    assert rel < 2e-2, rel
    pred = LocalPredictor(m, batch_size=4)
    out = pred.predict(x.cpu())
    assert pred._graphs and all(g.captured for g in pred._graphs.values())
    rel2 = float((torch.stack([o.float() for o in out]).cuda() - ref).norm() / ref.norm())
    assert rel2 < 2e-2, rel2
