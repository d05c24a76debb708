#!/usr/bin/env python
"""Benchmarks for the secondary BASELINE.json configs (the headline ResNet-50 one is ``bench.py``).

    python tools/bench_configs.py --config lenet      # 1: LeNet-5 MNIST-shape, LocalOptimizer on CPU
    python tools/bench_configs.py --config vgg        # 2: VggForCifar10 CIFAR-shape, 1 GPU bf16
    python tools/bench_configs.py --config ptb        # 4: PTB 2-layer LSTM LM (N GPUs via torch.distributed.run)
    python tools/bench_configs.py --config inception  # 5: Inception-v1 from Caffe files, batch inference
    python tools/bench_configs.py --config transformer  # Transformer LM 6x512 (native LayerNorm A/B)
    python tools/bench_configs.py --config int8       # VGG16 inference: int8 vs fp32 (bf16x3) vs bf16
    python tools/bench_configs.py --config all

Every config builds the model exactly as the reference's example/model builder does, uses synthetic
inputs of the reference shape and random-init weights (no datasets or checkpoints are available),
times K full steps (forward + criterion + backward + optimizer, or one inference forward) between
device synchronisations after W warmup steps, and prints one JSON line per config.

Config 5 round-trips the model through the loaders: the random-init Inception-v1 is written as a
Caffe prototxt + caffemodel (``CaffePersister``), loaded back with ``CaffeLoader``, saved as a
``.bigdl`` protobuf and re-loaded from it — the timed model is the one that came out of the loaders.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(_HERE, "..", "bigdl-1_amd"))


def _sync(dev):
    import torch
    if dev.type == "cuda":
        torch.cuda.synchronize()


_CPROFILE = {"n": 0}


def _time_steps(fn, dev, steps, warmup):
    for _ in range(warmup):
        fn()
    _sync(dev)
    t0 = time.perf_counter()
    r = None
    for _ in range(steps):
        r = fn()
    _sync(dev)
    el = time.perf_counter() - t0
    if _CPROFILE["n"]:  # host-side hot spots of the step (stderr), after the timed run
        import cProfile
        import io
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(_CPROFILE["n"]):
            fn()
        _sync(dev)
        pr.disable()
        out = io.StringIO()
        pstats.Stats(pr, stream=out).sort_stats("tottime").print_stats(35)
        print(out.getvalue()[:9000], file=sys.stderr, flush=True)
    return el, r


def bench_lenet(args):
    """Config 1: LeNet-5 (``DL/models/lenet/LeNet5.scala:25``), MNIST shape 1×28×28, 10 classes,
    ClassNLLCriterion, SGD lr 0.05 (``lenet/Train.scala``), LocalOptimizer on the CPU."""
    import torch
    from bigdl.utils.engine import Engine
    Engine.init(device="cpu")
    from bigdl.models.lenet import LeNet5
    from bigdl.nn import ClassNLLCriterion
    from bigdl.optim import SGD
    from bigdl.optim.optimizer import LocalOptimizer
    from bigdl.dataset import MiniBatch
    B = args.batch or 128
    g = torch.Generator().manual_seed(1)
    x = torch.randn(B, 1, 28, 28, generator=g)
    y = (torch.randint(0, 10, (B,), generator=g) + 1).float()
    batch = MiniBatch(x, y)
    opt = LocalOptimizer(LeNet5(10), [batch], ClassNLLCriterion(), SGD(learningrate=0.05), batch_size=B)
    opt.prepare()
    dev = torch.device("cpu")
    el, loss = _time_steps(lambda: opt.train_step(batch), dev, args.steps, args.warmup)
    return {"metric": "records/sec LeNet-5 MNIST-shape LocalOptimizer (CPU)", "value": round(B * args.steps / el, 1),
            "unit": "records/sec", "n_gpus": 0, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True, "dtype": "fp32",
            "data": "synthetic", "config": {"model": "LeNet-5", "global_batch": B, "device": "cpu",
                                            "threads": torch.get_num_threads()},
            "final_loss": float(loss)}


def bench_vgg(args):
    """Config 2: VggForCifar10 (``DL/models/vgg/VggForCifar10.scala:23-75``), 3×32×32, 10 classes,
    ClassNLLCriterion, SGD(lr 0.01, wd 5e-4, momentum 0.9) as ``vgg/Train.scala``; bf16 compute."""
    import torch
    from bigdl.utils import config
    config.set_property("bigdl.compute.dtype", args.dtype)
    from bigdl.utils.engine import Engine
    Engine.init()
    dev = Engine.device()
    from bigdl.models.vgg import VggForCifar10
    from bigdl.nn import ClassNLLCriterion
    from bigdl.optim import SGD
    from bigdl.optim.optimizer import LocalOptimizer
    from bigdl.dataset import MiniBatch
    B = args.batch or 128
    g = torch.Generator().manual_seed(2)
    x = torch.randn(B, 3, 32, 32, generator=g).to(dev).to(Engine.compute_dtype()).contiguous(
        memory_format=torch.channels_last)
    y = (torch.randint(0, 10, (B,), generator=g) + 1).float().to(dev)
    batch = MiniBatch(x, y)
    sgd = SGD(learningrate=0.01, weightdecay=5e-4, momentum=0.9, dampening=0.0)
    opt = LocalOptimizer(VggForCifar10(10), [batch], ClassNLLCriterion(), sgd, batch_size=B)
    opt.prepare()
    tiles = None
    if getattr(args, "tune", False) and dev.type == "cuda":
        # compile-phase kernel selection on this model's conv geometries (nn/compiled.py autotune)
        from bigdl.nn.compiled import autotune
        tiles = len(autotune(opt.model, batch.getInput()))
    step = opt.train_step
    if args.graph:
        from bigdl.optim.graph_step import graphed_train_step
        step = lambda b: graphed_train_step(opt, b)  # noqa: E731
    el, loss = _time_steps(lambda: step(batch), dev, args.steps, args.warmup)
    return {"metric": "images/sec VggForCifar10 CIFAR-shape 1 GPU", "value": round(B * args.steps / el, 1),
            "unit": "images/sec", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True, "dtype": args.dtype,
            "data": "synthetic", "config": {"model": "VggForCifar10", "global_batch": B,
                                            "hip_graph": bool(args.graph and getattr(opt, "_graphed", None)),
                                            "tuned_tiles": tiles},
            "final_loss": float(loss)}


def bench_ptb(args):
    """Config 4: PTB LSTM language model (``DL/example/languagemodel/PTBModel.scala``, defaults
    ``languagemodel/Utils.scala:44-53``: vocab 10000, hidden 200, 2 layers, 20 steps, batch 20),
    TimeDistributedCriterion(CrossEntropy, sizeAverage=false), Adagrad(lr 0.01, decay 0.001).
    N>1 ranks run the DistriOptimizer; ``value`` is whole-job tokens/sec."""
    import torch
    from bigdl.utils import config
    config.set_property("bigdl.compute.dtype", args.dtype)
    from bigdl.utils.engine import Engine
    world = int(os.environ.get("WORLD_SIZE", "1"))
    distri = world > 1 or args.force_distri
    if args.force_distri and "RANK" not in os.environ:
        # one rank outside torchrun: env:// rendezvous with itself (the DistriOptimizer path at world 1)
        import socket
        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        os.environ.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=str(sk.getsockname()[1]))
        sk.close()
    Engine.init(dist=distri)
    dev = Engine.device()
    rank = Engine.rank()
    from bigdl.models.rnn import PTBModel
    from bigdl.nn import CrossEntropyCriterion, TimeDistributedCriterion
    from bigdl.optim import Adagrad
    from bigdl.optim.optimizer import LocalOptimizer
    from bigdl.dataset import MiniBatch
    from bigdl.parallel import comm
    B = args.batch or 20
    T = args.seq_len
    V, H = 10000, args.hidden
    g = torch.Generator().manual_seed(3 + rank)
    x = (torch.randint(0, V, (B, T), generator=g) + 1).float().to(dev)
    y = (torch.randint(0, V, (B, T), generator=g) + 1).float().to(dev)
    batch = MiniBatch(x, y)
    model = PTBModel.lstm(V, H, V, 2)
    crit = TimeDistributedCriterion(CrossEntropyCriterion(), size_average=False)
    ada = Adagrad(learningrate=0.01, learningrate_decay=0.001)
    if distri:
        from bigdl.parallel import DistriOptimizer
        opt = DistriOptimizer(model, [batch], crit, ada, batch_size=B)
    else:
        opt = LocalOptimizer(model, [batch], crit, ada, batch_size=B)
    opt.prepare()
    step = opt.train_step
    if args.graph and world == 1:
        from bigdl.optim.graph_step import graphed_train_step
        step = lambda b: graphed_train_step(opt, b)  # noqa: E731
    for _ in range(args.warmup):
        step(batch)
    if hasattr(opt, "_wait_all_gathers"):
        opt._wait_all_gathers()
    comm.barrier()
    _sync(dev)
    t0 = time.perf_counter()
    loss = None
    for _ in range(args.steps):
        loss = step(batch)
    if hasattr(opt, "_wait_all_gathers"):
        opt._wait_all_gathers()
    _sync(dev)
    comm.barrier()
    el = comm.allreduce_max(time.perf_counter() - t0)
    if _CPROFILE["n"] and rank == 0:  # host-side hot spots of the step (stderr), after the timed run
        import cProfile
        import io
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(_CPROFILE["n"]):
            step(batch)
        _sync(dev)
        pr.disable()
        out = io.StringIO()
        pstats.Stats(pr, stream=out).sort_stats("tottime").print_stats(40)
        pstats.Stats(pr, stream=out).sort_stats("cumulative").print_stats(45)
        print(out.getvalue()[:24000], file=sys.stderr, flush=True)
    res = {"metric": "tokens/sec PTB 2-layer LSTM LM", "value": round(B * T * world * args.steps / el, 1),
           "unit": "tokens/sec", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True, "dtype": args.dtype,
           "data": "synthetic", "scaling": "weak",
           "config": {"model": "PTBModel.lstm", "vocab": V, "hidden": H, "layers": 2, "seq_len": T,
                      "per_gpu_batch": B, "global_batch": B * world, "parallelism": f"dp{world}",
                      "hip_graph": bool(getattr(opt, "_graphed", None)),
                      "driver": type(opt).__name__,
                      "update_mode": ("sharded" if getattr(opt, "sharded", False) else "replicated") if distri
                      else "local"},
           "final_loss": float(loss)}
    return res if rank == 0 else None


def bench_inception(args):
    """Config 5: Inception-v1 (bvlc_googlenet topology, ``DL/models/inception/Inception_v1.scala``)
    written to / loaded from Caffe prototxt+caffemodel and .bigdl, then batch inference, bf16."""
    import torch
    from bigdl.utils import config
    config.set_property("bigdl.compute.dtype", args.dtype)
    from bigdl.utils.engine import Engine
    Engine.init()
    dev = Engine.device()
    from bigdl.models.inception import Inception_v1_NoAuxClassifier
    from bigdl.serialization.caffe_persister import save_caffe
    from bigdl.serialization.caffe_loader import load_caffe_model
    from bigdl.nn.module import Module
    from bigdl.utils.random import RNG
    RNG.setSeed(5)
    src = Inception_v1_NoAuxClassifier.graph(1000, has_dropout=True)
    with tempfile.TemporaryDirectory() as td:
        proto, cm, bd = (os.path.join(td, n) for n in ("googlenet.prototxt", "googlenet.caffemodel", "g.bigdl"))
        t0 = time.perf_counter()
        save_caffe(src.evaluate(), proto, cm, use_v2=True, overwrite=True)
        loaded = load_caffe_model(proto, cm)
        loaded.saveModule(bd, over_write=True)
        model = Module.loadModule(bd)
        load_s = time.perf_counter() - t0
    B = args.batch or 256
    g = torch.Generator().manual_seed(5)
    xc = torch.randn(4, 3, 224, 224, generator=g)
    # loader correctness gate (fp32 CPU): the round-tripped model matches the source model
    src.evaluate()
    model.evaluate()
    with torch.no_grad():
        ref = src.forward(xc).float()
        got = model.forward(xc).float()
    # Caffe has no LogSoftMax layer: the persister writes a Softmax and the loader maps it back to
    # SoftMax (``Converter.scala``), so compare probabilities.
    if torch.allclose(got.sum(1), torch.ones(got.shape[0]), atol=1e-3):
        ref = ref.exp()
    err = float((ref - got).abs().max())
    assert err < 1e-4, f"Caffe/.bigdl round trip changed the output: max|diff|={err}"
    model.cuda() if dev.type == "cuda" else None
    model.evaluate()
    from bigdl.nn.fusion import fuse
    fuse(model)  # what LocalPredictor does: conv+ReLU epilogues, zero-copy concats
    dt = Engine.compute_dtype() if dev.type == "cuda" else torch.float32
    x = torch.randn(B, 3, 224, 224, generator=g).to(dev).to(dt).contiguous(memory_format=torch.channels_last)

    def step():
        with torch.no_grad():
            return model.forward(x)
    tiles = None
    if getattr(args, "compiled", False) and dev.type == "cuda":
        # the LocalPredictor path: plan + conv kernel selection + HIP-graph forward (nn/compiled.py)
        from bigdl.nn.compiled import compile as compile_module
        cm = compile_module(model, x)
        tiles = len(cm.tiles)

        def step():  # noqa: F811
            return cm(x)
    el, out = _time_steps(step, dev, args.steps, args.warmup)
    return {"metric": "images/sec Inception-v1 (Caffe-loaded) batch inference 1 GPU",
            "value": round(B * args.steps / el, 1), "unit": "images/sec", "n_gpus": 1, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
            "dtype": args.dtype if dev.type == "cuda" else "fp32", "data": "synthetic",
            "config": {"model": "Inception-v1 (NoAux, Caffe round-trip)", "global_batch": B,
                       "executor": "compiled (autotuned tiles %s, HIP graph)" % tiles if tiles is not None else "eager",
                       "load_roundtrip_s": round(load_s, 2), "roundtrip_max_abs_diff": err}}


def bench_resnet_infer(args):
    """ResNet-50 batch inference through the IR lowering (``ConversionUtils.convert``: BN folded
    into the convs, ReLU in the conv epilogues), bf16, random-init weights with non-trivial BN
    running statistics; checked against the unfolded eval model before timing."""
    import torch
    from bigdl.utils import config
    config.set_property("bigdl.compute.dtype", args.dtype)
    from bigdl.utils.engine import Engine
    Engine.init()
    dev = Engine.device()
    from bigdl.models.resnet import ResNet, DatasetType, model_init
    from bigdl.utils.intermediate import ConversionUtils
    from bigdl.utils.random import RNG
    RNG.setSeed(7)
    model = model_init(ResNet(1000, depth=50, dataset=DatasetType.ImageNet))
    model.training()
    with torch.no_grad():  # a few training forwards on CPU give the BNs real running statistics
        model.forward(torch.randn(2, 3, 224, 224))
    model.evaluate()
    xc = torch.randn(2, 3, 224, 224)
    with torch.no_grad():
        ref = model.forward(xc).float().clone()
    ir = ConversionUtils.convert(model)
    with torch.no_grad():
        err = float((ir.forward(xc).float() - ref).abs().max())
    assert err < 1e-3, f"IR lowering changed the output: {err}"
    if dev.type == "cuda":
        ir.to(dev)
    B = args.batch or 256
    dt = Engine.compute_dtype() if dev.type == "cuda" else torch.float32
    x = torch.randn(B, 3, 224, 224).to(dev).to(dt).contiguous(memory_format=torch.channels_last)

    def step():
        with torch.no_grad():
            return ir.forward(x)
    el, _ = _time_steps(step, dev, args.steps, args.warmup)
    return {"metric": "images/sec ResNet-50 batch inference (IR: BN folded) 1 GPU",
            "value": round(B * args.steps / el, 1), "unit": "images/sec", "n_gpus": 1, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
            "dtype": args.dtype if dev.type == "cuda" else "fp32", "data": "synthetic",
            "config": {"model": "ResNet-50 (IRGraph inference lowering)", "global_batch": B,
                       "fold_max_abs_diff": err}}


def bench_transformer(args):
    """Transformer language model (``DL/nn/Transformer.scala``, type LanguageModel with the shared
    embedding/softmax projection): pre-norm blocks (native LayerNorm kernels), fused attention,
    TimeDistributedCriterion(CrossEntropy), Adam; bf16 compute, 1 GPU.  ``--no-native-ln`` runs the
    composed torch LayerNorm for an A/B of the kernel."""
    import torch
    from bigdl.utils import config
    config.set_property("bigdl.compute.dtype", args.dtype)
    from bigdl.utils.engine import Engine
    Engine.init()
    dev = Engine.device()
    if args.no_native_ln:
        from bigdl.ops import native
        native._PY_OPS.pop("layer_norm", None)
    from bigdl.nn import Transformer, CrossEntropyCriterion, TimeDistributedCriterion
    from bigdl.optim import Adam
    from bigdl.optim.optimizer import LocalOptimizer
    from bigdl.dataset import MiniBatch
    B = args.batch or 32
    L, V, H = args.seq_len if args.seq_len != 20 else 128, 8000, 512
    g = torch.Generator().manual_seed(5)
    x = (torch.randint(1, V, (B, L), generator=g)).float().to(dev)
    y = (torch.randint(0, V, (B, L), generator=g) + 1).float().to(dev)
    batch = MiniBatch(x, y)
    model = Transformer(V, H, 8, 2048, 6, 1.0, 1.0, 1.0, with_share_weights_linear=True,
                        transformer_type="LanguageModel")
    crit = TimeDistributedCriterion(CrossEntropyCriterion(), size_average=True)
    opt = LocalOptimizer(model, [batch], crit, Adam(learningrate=1e-4), batch_size=B)
    opt.prepare()
    step = opt.train_step
    if args.graph:
        from bigdl.optim.graph_step import graphed_train_step
        step = lambda b: graphed_train_step(opt, b)  # noqa: E731
    el, loss = _time_steps(lambda: step(batch), dev, args.steps, args.warmup)
    return {"metric": "tokens/sec Transformer LM 6x512 1 GPU", "value": round(B * L * args.steps / el, 1),
            "unit": "tokens/sec", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True, "dtype": args.dtype,
            "data": "synthetic", "config": {"model": "Transformer-LM", "layers": 6, "hidden": H, "heads": 8,
                                            "filter": 2048, "vocab": V, "seq_len": L, "global_batch": B,
                                            "native_layernorm": not args.no_native_ln,
                                            "hip_graph": bool(args.graph and getattr(opt, "_graphed", None))},
            "final_loss": float(loss)}


def _lsuv(model, x):
    """Data-dependent init of a random-init plain Sequential (CPU, fp32, a small batch): layer by
    layer, every conv output channel is shifted and scaled to zero mean and unit standard deviation
    over the batch and pixels (bias ← (bias − μ)/σ, weight row ← row/σ); a Linear is scaled to unit
    output standard deviation as a whole.  A random-init VGG16 on
    random images otherwise ends in logits that are one image-independent vector (every image the
    same top-1), so an int8-vs-fp32 comparison of them measures nothing; centred, the logits carry
    image-dependent signal as a trained network's do."""
    import torch
    from bigdl.nn import Linear, SpatialConvolution
    with torch.no_grad():
        h = x
        for m in model.modules:
            y = m.forward(h)
            if isinstance(m, (Linear, SpatialConvolution)) and getattr(m, "bias", None) is not None:
                yc = y.float().transpose(0, 1).reshape(y.shape[1], -1)  # [channels][batch·pixels]
                mu, sd = yc.mean(1), yc.std(1).clamp_min(1e-6)
                if isinstance(m, Linear):
                    # a few images give each FC output only a few samples: per-feature centring would
                    # blow the weights up (cancelling W·x against a huge bias); scale globally
                    mu, sd = torch.zeros_like(mu), torch.full_like(sd, float(yc.std()))
                wt = m.weight  # [K][...] or the grouped [g][K/g][...] (g = 1 here)
                lead = 2 if wt.dim() == 5 else 1
                wt.div_(sd.view(*wt.shape[:lead], *([1] * (wt.dim() - lead))))
                m.bias.sub_(mu).div_(sd)
                y = m.forward(h)
            h = y.clone() if isinstance(y, torch.Tensor) else y


def bench_int8(args):
    """int8 inference vs the reference's published claim (VGG16 int8 2.04× over fp32,
    ``docs/docs/whitepaper.md:192-196``): VGG16 (``DL/models/vgg/Vgg_16``), 224², batch 128,
    random-init weights, synthetic images; the same model timed in fp32 compute (bf16x3 on the
    matrix cores — the reference's precision), bf16, and quantized (``Module.quantize``: int8
    implicit-GEMM convs with per-image activation scales, int8 GEMM FCs).  Also reports the cosine
    of the int8 logits against fp32 on the timed batch (weights LSUV-rescaled, :func:`_lsuv`, so the
    logits are image-dependent) and the top-1 agreement.""" 
    import torch
    from bigdl.utils import config
    from bigdl.utils.engine import Engine
    from bigdl.models.vgg import Vgg_16
    from bigdl.utils.random import RNG
    B = args.batch or (128 if args.int8_model == "vgg16" else 256)
    res = {}
    RNG.setSeed(11)
    torch.manual_seed(11)
    g = torch.Generator().manual_seed(3)
    x32 = torch.randn(B, 3, 224, 224, generator=g)
    if args.int8_model == "vgg16":
        base = Vgg_16(1000, has_dropout=False)
        base.evaluate()
        _lsuv(base, x32[:8])
    elif args.int8_model == "resnet50":
        # residual blocks: BN folded into the convs, conv + sum epilogues, int8 block outputs
        from bigdl.models.resnet import ResNet, DatasetType, model_init
        base = model_init(ResNet(1000, depth=50, dataset=DatasetType.ImageNet))
        from bigdl.nn import SpatialBatchNormalization
        with torch.no_grad():  # trained-like BN affine parameters (model_init zeroes the block-tail γ)
            for bn in base.flattened_modules():
                if isinstance(bn, SpatialBatchNormalization):
                    bn.weight.uniform_(0.2, 1.0, generator=g)
                    bn.bias.normal_(0.0, 0.1, generator=g)
        base.training()
        with torch.no_grad():  # a few training forwards give the BNs real running statistics
            for i in range(2):
                base.forward(torch.randn(8, 3, 224, 224, generator=g))
        base.evaluate()
    else:
        from bigdl.models.inception import Inception_v1_NoAuxClassifier
        base = Inception_v1_NoAuxClassifier.graph(1000, has_dropout=False)
        base.evaluate()
    outs = {}
    modes = ("fp32", "bf16", "int8") + (("bf16_compiled", "int8_graph") if args.int8_model != "vgg16" else ())
    for mode in modes:
        config.set_property("bigdl.compute.dtype", "fp32" if mode == "fp32" else "bf16")
        Engine.init()
        dev = Engine.device()
        if mode.startswith("int8") and args.calib > 0:
            # calibration (MklInt8Convertible.calcScales): a forward of CALIB images that are not the
            # timed batch records every layer's max|input|; quantize() then runs static int8 chains
            cal = base.cloneModule().to(dev)
            cal.evaluate()
            gc = torch.Generator().manual_seed(5)
            xc = torch.randn(args.calib, 3, 224, 224, generator=gc).to(dev).to(torch.bfloat16).contiguous(
                memory_format=torch.channels_last)
            with torch.no_grad():
                cal.forward(xc)
            cal.calcScales(xc)
            # the FC head: with calibrated scales the quantised Linears take the chain's int8
            # activation as is and hand int8 to each other (split-K int8 GEMM, requantising
            # epilogue): VGG16 4.32 → 4.26 ms at the same logit cosine (profiles/r6_int8.txt);
            # --int8-fc 0 keeps it in bf16 (round 5's choice, profiles/r5_int8_calibration_sweep.txt)
            old_fc = config.get_property("bigdl.int8.quantizeLinear")
            config.set_property("bigdl.int8.quantizeLinear", bool(args.int8_fc))
            try:
                m = cal.quantize()
            finally:
                config.set_property("bigdl.int8.quantizeLinear", old_fc)
            del cal
        elif mode.startswith("int8"):
            m = base.quantize()
        else:
            m = base.cloneModule()
        m.evaluate()
        m = m.to(dev)
        dt = torch.float32 if mode == "fp32" else torch.bfloat16
        x = x32.to(dev).to(dt).contiguous(memory_format=torch.channels_last)

        def step():
            with torch.no_grad():
                return m.forward(x)
        if mode == "bf16_compiled":
            # the compiled inference path the predictors use (IR lowering: BN folded, conv+sum+ReLU
            # epilogues; kernel selection; HIP graph) — the strongest bf16 baseline
            from bigdl.nn.compiled import compile as compile_module
            cm = compile_module(m, x)
            step = lambda: cm(x)  # noqa: E731
        elif mode == "int8_graph" and dev.type == "cuda":
            # the int8 forward captured in one HIP graph (no per-layer host dispatch)
            st = torch.cuda.Stream()
            st.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(st), torch.no_grad():
                for _ in range(2):
                    m.forward(x)
            torch.cuda.current_stream().wait_stream(st)
            gr = torch.cuda.CUDAGraph()
            with torch.no_grad(), torch.cuda.graph(gr):
                gout = m.forward(x)

            def step():  # noqa: F811
                gr.replay()
                return gout
        el, y = _time_steps(step, dev, args.steps, args.warmup)
        outs[mode] = y.float().cpu()
        res[mode] = {"value": round(B * args.steps / el, 1), "ms_per_step": round(el / args.steps * 1e3, 3)}
        del m
        if dev.type == "cuda":
            torch.cuda.empty_cache()
    def _cos(a, b):
        a, b = a.double().flatten(), b.double().flatten()
        return float(a @ b / (a.norm() * b.norm()))
    qi, qf = outs["int8"].reshape(B, -1).double(), outs["fp32"].reshape(B, -1).double()
    # the model ends in LogSoftMax (log p = logits − logsumexp, a per-image constant): compare the
    # row-centred log-probabilities (= centred logits); and, since a random-init VGG's logits are
    # dominated by one image-independent vector, also the image-dependent part (batch mean removed)
    ci, cf = qi - qi.mean(1, keepdim=True), qf - qf.mean(1, keepdim=True)
    cos = _cos(ci, cf)
    cos_img = _cos(ci - ci.mean(0, keepdim=True), cf - cf.mean(0, keepdim=True))
    top1 = float((qi.argmax(1) == qf.argmax(1)).float().mean())
    extra = {}
    if "int8_graph" in res:
        extra = {"bf16_compiled": res["bf16_compiled"], "int8_graph": res["int8_graph"],
                 "int8_graph_over_bf16_compiled": round(res["int8_graph"]["value"] / res["bf16_compiled"]["value"], 3),
                 "cosine_int8_graph_vs_fp32": round(_cos(outs["int8_graph"].reshape(B, -1) - outs["int8_graph"].reshape(
                     B, -1).mean(1, keepdim=True), cf), 5)}
    name = {"vgg16": "VGG16", "resnet50": "ResNet-50", "inception": "Inception-v1"}[args.int8_model]
    return {"metric": f"images/sec {name} 224x224 batch inference 1 GPU: int8 vs fp32 vs bf16",
            "value": res["int8"]["value"], "unit": "images/sec", "n_gpus": 1, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": res["int8"]["ms_per_step"], "higher_is_better": True,
            "dtype": "int8", "data": "synthetic", "config": {"model": name, "global_batch": B, "image_size": 224},
            "fp32": res["fp32"], "bf16": res["bf16"], **extra,
            "int8_over_fp32": round(res["int8"]["value"] / res["fp32"]["value"], 3),
            "int8_over_bf16": round(res["int8"]["value"] / res["bf16"]["value"], 3),
            "reference_int8_over_fp32": 2.04, "cosine_int8_vs_fp32": round(cos, 5), "calibration_images": args.calib,
            "cosine_image_dependent": round(cos_img, 5), "top1_agreement": top1,
            "calibration": str(config.get_property("bigdl.int8.calibration")),
            "unsigned_activations": bool(config.get_property("bigdl.int8.unsignedActivations")),
            "fc_dtype": "int8" if (args.int8_fc or args.calib <= 0) else "bf16",
            "logit_spread_fp32": round(float(cf.std()), 5)}


CONFIGS = {"lenet": bench_lenet, "vgg": bench_vgg, "ptb": bench_ptb, "inception": bench_inception,
           "resnet_infer": bench_resnet_infer, "transformer": bench_transformer, "int8": bench_int8}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="all", choices=list(CONFIGS) + ["all"])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=0, help="0 = the config's reference default")
    ap.add_argument("--seq-len", type=int, default=20)
    ap.add_argument("--hidden", type=int, default=200)
    ap.add_argument("--calib", type=int, default=32, help="int8: calibration images (0 = per-image dynamic scales)")
    ap.add_argument("--int8-fc", type=int, default=1, help="int8 (calibrated): quantize the Linear layers too")
    ap.add_argument("--tune", action="store_true", help="vgg: pin autotuned conv tiles before timing")
    ap.add_argument("--compiled", action="store_true", help="inception: run through nn.compiled (kernel selection + HIP graph)")
    ap.add_argument("--graph", action="store_true", help="capture the training step into a HIP graph (vgg, ptb, transformer)")
    ap.add_argument("--cprofile", type=int, default=0, help="cProfile this many extra steps (host hot spots, stderr)")
    ap.add_argument("--no-native-ln", action="store_true", help="transformer: composed torch LayerNorm")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"],
                    help="compute dtype of the GPU configs (fp32 = the reference's precision, bf16x3 kernels)")
    ap.add_argument("--force-distri", action="store_true", help="ptb: the DistriOptimizer even at world 1")
    ap.add_argument("--int8-model", default="vgg16", choices=["vgg16", "resnet50", "inception"],
                    help="int8: the network (resnet50: BN folded + int8 residual blocks; inception: concat)")
    args = ap.parse_args()
    _CPROFILE["n"] = args.cprofile
    names = list(CONFIGS) if args.config == "all" else [args.config]
    for n in names:
        r = CONFIGS[n](args)
        if r is not None:
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
