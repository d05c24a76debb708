"""Shared plumbing of the training CLIs: argument sets, engine start-up, optimizer assembly
(checkpoint / validation / summaries / end trigger / snapshot resume) — the pieces every reference
``Train.scala`` main repeats."""
from __future__ import annotations

import argparse
import os
import time
from typing import List, Optional, Sequence

import numpy as np
import torch

from ...utils.logger import get_logger

log = get_logger("bigdl.models.train")


def base_parser(desc: str, batch: int, epochs: int, lr: float) -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description=desc)
    ap.add_argument("-f", "--folder", default=None, help="dataset folder (format per model)")
    ap.add_argument("-b", "--batchSize", type=int, default=batch, help="GLOBAL batch size (split over ranks)")
    ap.add_argument("-e", "--nEpochs", "--maxEpoch", dest="nEpochs", type=int, default=epochs)
    ap.add_argument("--maxIteration", type=int, default=None, help="stop after this many iterations")
    ap.add_argument("-r", "--learningRate", type=float, default=lr)
    ap.add_argument("--learningRateDecay", type=float, default=0.0)
    ap.add_argument("--momentum", type=float, default=0.9)
    ap.add_argument("--weightDecay", type=float, default=1e-4)
    ap.add_argument("--dampening", type=float, default=0.0)
    ap.add_argument("--nesterov", type=lambda s: str(s).lower() in ("1", "true", "yes"), default=True)
    ap.add_argument("--model", dest="modelSnapshot", default=None, help="resume from a saved .bigdl model")
    ap.add_argument("--state", dest="stateSnapshot", default=None, help="resume from a saved optimMethod")
    ap.add_argument("--checkpoint", default=None, help="checkpoint directory (written every epoch)")
    ap.add_argument("--overwrite", action="store_true", help="overwrite the checkpoint files")
    ap.add_argument("--summary", default=None, help="TensorBoard log dir for Train/Validation summaries")
    ap.add_argument("--appName", default=None)
    ap.add_argument("--synthetic", type=int, default=0, help="N random training records (no dataset needed)")
    ap.add_argument("--dtype", default="auto", choices=["auto", "bf16", "fp32"], help="compute dtype")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--threads", type=int, default=4, help="native loader worker threads")
    ap.add_argument("--saveModel", default=None, help="write the trained model here (.bigdl)")
    return ap


def init_engine(args):
    from ...utils import config
    from ...utils.engine import Engine
    from ...utils.random import RNG
    config.set_property("bigdl.compute.dtype", args.dtype)
    Engine.init(dist=int(os.environ.get("WORLD_SIZE", "1")) > 1)
    RNG.setSeed(args.seed + Engine.rank())
    torch.manual_seed(args.seed)
    return Engine


def per_rank_batch(args) -> int:
    from ...utils.engine import Engine
    w = Engine.world_size()
    if args.batchSize % w:
        raise ValueError(f"batch size {args.batchSize} must be a multiple of the world size {w}")
    return args.batchSize // w


def synthetic_images(n: int, h: int, w: int, c: int, classes: int, seed: int):
    """uint8 NHWC images with learnable structure (class-dependent mean) and 1-based labels."""
    g = np.random.default_rng(seed)
    labels = g.integers(0, classes, n)
    # the class templates are shared by every split (train / validation draw from one distribution)
    base = np.random.default_rng(1234567).integers(0, 256, (classes, 1, 1, c))
    imgs = np.clip(base[labels] + g.normal(0, 40, (n, h, w, c)), 0, 255).astype(np.uint8)
    return imgs, (labels + 1).astype(np.float32)


def image_loader(images, labels, batch, crop, train, mean, std, args, pad=0, flip=None, layout=None):
    """The native C++ batch loader (pinned slots, async H2D, per-rank partition)."""
    from ...runtime.loader import NativeBatchLoader
    from ...utils.engine import Engine
    dev = Engine.device()
    on_gpu = dev.type == "cuda"
    return NativeBatchLoader(images, labels, batch, crop=crop, pad=pad, flip=train if flip is None else flip,
                             train=train, mean=mean, std=std,
                             dtype=torch.bfloat16 if (on_gpu and Engine.compute_dtype() == torch.bfloat16)
                             else torch.float32,
                             layout=layout or ("NHWC" if on_gpu else "NCHW"), shuffle=train, drop_last=train,
                             seed=args.seed, threads=args.threads, device=dev, rank=Engine.rank(),
                             world=Engine.world_size())


def load_model_or(args, build):
    from ...nn.module import Module
    if args.modelSnapshot:
        log.info(f"loading model snapshot {args.modelSnapshot}")
        return Module.load(args.modelSnapshot)
    return build()


def optim_or(args, build):
    if args.stateSnapshot:
        from ...optim.optim_method import OptimMethod
        log.info(f"loading optimMethod snapshot {args.stateSnapshot}")
        return OptimMethod.load(args.stateSnapshot)
    return build()


def assemble(model, train_set, criterion, optim, args, val_set=None, vmethods: Optional[Sequence] = None,
             batch: Optional[int] = None, app: str = "bigdl"):
    """Optimizer (Local or Distri by world size) with the reference's standard wiring."""
    from ...optim.optimizer import Optimizer
    from ...optim.trigger import Trigger, MaxIteration
    from ...visualization import TrainSummary, ValidationSummary
    opt = Optimizer.create(model, train_set, criterion, batch_size=batch or args.batchSize, optim_method=optim)
    end = Trigger.maxEpoch(args.nEpochs)
    if args.maxIteration:
        from ...optim.trigger import TriggerOr
        end = TriggerOr(end, MaxIteration(args.maxIteration))
    opt.setEndWhen(end)
    if args.checkpoint:
        opt.setCheckpoint(args.checkpoint, Trigger.everyEpoch(), args.overwrite)
    if val_set is not None and vmethods:
        opt.setValidation(Trigger.everyEpoch(), val_set, list(vmethods), batch or args.batchSize)
    if args.summary:
        name = args.appName or f"{app}-{time.strftime('%Y%m%d-%H%M%S')}"
        ts = TrainSummary(args.summary, name)
        ts.setSummaryTrigger("LearningRate", Trigger.severalIteration(1))
        opt.setTrainSummary(ts)
        if val_set is not None:
            opt.setValidationSummary(ValidationSummary(args.summary, name))
    return opt


def finish(opt, model, args) -> dict:
    from ...utils.engine import Engine
    if args.saveModel and Engine.rank() == 0:
        model.saveModel(args.saveModel, over_write=True)
    st = dict(opt.state)
    if Engine.is_distributed():
        import torch.distributed as tdist
        tdist.barrier()  # every rank is done with the group before it is torn down
        Engine.shutdown()
    return {k: st[k] for k in ("epoch", "neval", "Loss") if k in st}


def evaluate(model, data, methods: List, device=None):
    """Test.scala: run the validation methods over one pass of ``data`` (a loader or a data set)."""
    from ...optim.validation import allreduce_results
    model.evaluate()
    res = None
    with torch.no_grad():
        for b in data.data(train=False):
            if device is not None and device.type == "cuda":
                b = b.to(device)
            out = model.forward(b.getInput())
            rs = [m(out, b.getTarget()) for m in methods]
            res = rs if res is None else [a + r for a, r in zip(res, rs)]
    res = allreduce_results(res) if res is not None else []
    return list(zip(methods, res))
