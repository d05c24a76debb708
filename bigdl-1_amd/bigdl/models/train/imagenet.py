"""ImageNet training / evaluation (``DL/models/resnet/TrainImageNet.scala:52-140``,
``TestImageNet.scala``, ``inception/Train.scala``, ``vgg/TrainImageNet.scala``).

Data: ``--folder`` holds ``train/`` and ``val/`` Hadoop sequence files of BGR records (the
reference's ``ImageNetSeqFileGenerator`` format; ``bigdl.models.utils.seqfile_generator`` writes
them), decoded once into a uint8 array and streamed through the native C++ batch loader (random
crop + flip + normalise on worker threads, pinned slots, async host→device copy, each rank its own
partition).  ResNet: SGD with ``EpochDecayWithWarmUp`` (linear warm-up over ``--warmupEpoch``
epochs from ``--learningRate`` to ``--maxLr``, then ×0.1 at epochs 30/60/80), optional SyncBN
(``--syncBN``; the reference's ``setParallism``), Top-1/Top-5 validation and a checkpoint every
epoch, Train/Validation summaries.
"""
from __future__ import annotations

import math
import sys

from .common import (assemble, base_parser, evaluate, finish, image_loader, init_engine, load_model_or, log,
                     optim_or, per_rank_batch, synthetic_images)

MEAN = [0.485 * 255, 0.456 * 255, 0.406 * 255]
STD = [0.229 * 255, 0.224 * 255, 0.225 * 255]


def imagenet_decay(epoch: int) -> float:
    """TrainImageNet.imageNetDecay: the number of ×0.1 steps at epoch ``epoch``."""
    return 3 if epoch >= 80 else 2 if epoch >= 60 else 1 if epoch >= 30 else 0.0


def _parser():
    ap = base_parser("Train a model on ImageNet (sequence files)", batch=256, epochs=90, lr=0.1)
    ap.add_argument("--net", default="resnet", choices=["resnet", "inception", "vgg16"])
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--classes", type=int, default=1000)
    ap.add_argument("--shortcutType", default="B")
    ap.add_argument("--optnet", type=lambda s: str(s).lower() in ("1", "true"), default=False)
    ap.add_argument("--warmupEpoch", type=int, default=0)
    ap.add_argument("--maxLr", type=float, default=None)
    ap.add_argument("--syncBN", action="store_true", help="cross-rank BatchNorm statistics (setParallism)")
    ap.add_argument("--imageSize", type=int, default=224)
    ap.add_argument("--test", action="store_true", help="TestImageNet: evaluate --model on the val set")
    return ap


def _data(args, batch):
    size = args.imageSize
    if args.synthetic:
        src = max(size, 32 + size // 8)
        tr = synthetic_images(args.synthetic, src, src, 3, args.classes, args.seed)
        va = synthetic_images(max(batch, args.synthetic // 4), src, src, 3, args.classes, args.seed + 1)
    else:
        if not args.folder:
            raise SystemExit("--folder (ImageNet sequence files) or --synthetic N is required")
        from ...dataset.seqfile import SeqFileFolder
        tr = SeqFileFolder.to_arrays(args.folder + "/train", args.classes)
        va = SeqFileFolder.to_arrays(args.folder + "/val", args.classes)
    train = image_loader(tr[0], tr[1], batch, (size, size), True, MEAN, STD, args)
    val = image_loader(va[0], va[1], batch, (size, size), False, MEAN, STD, args)
    return train, val, int(tr[0].shape[0])


def _build(args):
    from ...models.resnet import ResNet, DatasetType, model_init
    if args.net == "resnet":
        return model_init(ResNet(args.classes, depth=args.depth, shortcut_type=args.shortcutType,
                                 dataset=DatasetType.ImageNet, optnet=args.optnet))
    if args.net == "inception":
        from ...models.inception import Inception_v1_NoAuxClassifier
        return Inception_v1_NoAuxClassifier(args.classes)
    from ...models.vgg import Vgg_16
    return Vgg_16(args.classes)


def set_sync_bn(model):
    """TrainImageNet.setParallism: every BatchNormalization syncs its statistics across ranks."""
    from ...nn.layers.normalization import BatchNormalization
    from ...utils.engine import Engine
    n = 0
    for m in model.flattened_modules():
        if isinstance(m, BatchNormalization):
            m.setParallism(Engine.world_size())
            n += 1
    return n


def main(argv=None):
    args = _parser().parse_args(argv)
    Engine = init_engine(args)
    from ...nn import CrossEntropyCriterion
    from ...optim import SGD
    from ...optim.optim_method import EpochDecayWithWarmUp
    from ...optim.validation import Top1Accuracy, Top5Accuracy
    batch = per_rank_batch(args)
    train, val, n_train = _data(args, batch)
    if args.test:
        model = load_model_or(args, lambda: _build(args))
        model.to(Engine.device())
        res = evaluate(model, val, [Top1Accuracy(), Top5Accuracy()], Engine.device())
        for m, r in res:
            log.info(f"{m.format()} is {r}")
        return {m.format(): r.result()[0] for m, r in res}
    model = load_model_or(args, lambda: _build(args))
    if args.syncBN and Engine.world_size() > 1:
        log.info(f"SyncBN on {set_sync_bn(model)} BatchNormalization layers")
    iters_per_epoch = max(1, math.ceil(n_train / args.batchSize))
    warm = iters_per_epoch * args.warmupEpoch
    max_lr = args.maxLr if args.maxLr is not None else args.learningRate
    delta = (max_lr - args.learningRate) / warm if warm > 0 else 0.0
    log.info(f"warmUpIteration: {warm}, startLr: {args.learningRate}, maxLr: {max_lr}, delta: {delta}, "
             f"nesterov: {args.nesterov}")

    def _sgd():
        return SGD(learningrate=args.learningRate, learningrate_decay=0.0, weightdecay=args.weightDecay,
                   momentum=args.momentum, dampening=args.dampening, nesterov=args.nesterov,
                   leaningrate_schedule=EpochDecayWithWarmUp(warm, delta, imagenet_decay))
    optim = optim_or(args, _sgd)
    if args.stateSnapshot:
        optim.learningRateSchedule = EpochDecayWithWarmUp(warm, delta, imagenet_decay)
    opt = assemble(model, train, CrossEntropyCriterion(), optim, args, val, [Top1Accuracy(), Top5Accuracy()],
                   batch, app=f"{args.net}-imagenet")
    opt.optimize()
    return finish(opt, model, args)


if __name__ == "__main__":
    main(sys.argv[1:])
