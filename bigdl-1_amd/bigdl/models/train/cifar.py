"""CIFAR-10 training (``DL/models/vgg/Train.scala``, ``DL/models/resnet/TrainCIFAR10.scala``).

Data: ``--folder`` with the CIFAR-10 binary batches (``data_batch_{1..5}.bin``, ``test_batch.bin``:
one label byte + 3072 CHW pixel bytes per record) or ``--synthetic N``.  Training augmentation as
the reference: 4-pixel zero-pad + random 32×32 crop + horizontal flip, per-channel normalisation;
VGG: SGD(lr, weightDecay 5e-4, momentum 0.9, EpochStep(25, 0.5)); ResNet: EpochSchedule as
TrainCIFAR10 (×0.1 at epochs 81 and 122).
"""
from __future__ import annotations

import os
import sys

import numpy as np

from .common import (assemble, base_parser, finish, image_loader, init_engine, load_model_or, optim_or,
                     per_rank_batch, synthetic_images)

MEAN = [125.3, 123.0, 113.9]
STD = [63.0, 62.1, 66.7]


def read_cifar_bin(paths):
    xs, ys = [], []
    for p in paths:
        raw = np.fromfile(p, dtype=np.uint8).reshape(-1, 3073)
        ys.append(raw[:, 0].astype(np.float32) + 1)
        xs.append(raw[:, 1:].reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1))
    return np.ascontiguousarray(np.concatenate(xs)), np.concatenate(ys)


def main(argv=None):
    ap = base_parser("Train VGG / ResNet on CIFAR-10", batch=128, epochs=90, lr=0.01)
    ap.add_argument("--net", default="vgg", choices=["vgg", "resnet"])
    ap.add_argument("--depth", type=int, default=20)
    args = ap.parse_args(argv)
    init_engine(args)
    from ...nn import ClassNLLCriterion, CrossEntropyCriterion
    from ...optim import SGD
    from ...optim.optim_method import EpochStep, EpochSchedule, Regime
    from ...optim.validation import Top1Accuracy
    batch = per_rank_batch(args)
    if args.synthetic:
        tr = synthetic_images(args.synthetic, 32, 32, 3, 10, args.seed)
        va = synthetic_images(max(batch, args.synthetic // 4), 32, 32, 3, 10, args.seed + 1)
    else:
        if not args.folder:
            raise SystemExit("--folder (CIFAR-10 binary batches) or --synthetic N is required")
        tr = read_cifar_bin([os.path.join(args.folder, f"data_batch_{i}.bin") for i in range(1, 6)])
        va = read_cifar_bin([os.path.join(args.folder, "test_batch.bin")])
    train = image_loader(tr[0], tr[1], batch, (32, 32), True, MEAN, STD, args, pad=4)
    val = image_loader(va[0], va[1], batch, (32, 32), False, MEAN, STD, args)
    if args.net == "vgg":
        from ...models.vgg import VggForCifar10
        model = load_model_or(args, lambda: VggForCifar10(10))
        crit = ClassNLLCriterion()
        optim = optim_or(args, lambda: SGD(learningrate=args.learningRate, learningrate_decay=0.0,
                                           weightdecay=5e-4, momentum=0.9, dampening=0.0, nesterov=False,
                                           leaningrate_schedule=EpochStep(25, 0.5)))
    else:
        from ...models.resnet import ResNet, DatasetType, model_init
        model = load_model_or(args, lambda: model_init(ResNet(10, depth=args.depth, dataset=DatasetType.CIFAR10)))
        crit = CrossEntropyCriterion()
        optim = optim_or(args, lambda: SGD(learningrate=args.learningRate, weightdecay=args.weightDecay,
                                           momentum=args.momentum, dampening=args.dampening,
                                           nesterov=args.nesterov,
                                           leaningrate_schedule=EpochSchedule([
                                               Regime(1, 80, {"learningRate": args.learningRate}),
                                               Regime(81, 121, {"learningRate": args.learningRate * 0.1}),
                                               Regime(122, 10 ** 9, {"learningRate": args.learningRate * 0.01})])))
    opt = assemble(model, train, crit, optim, args, val, [Top1Accuracy()], batch, app=f"{args.net}-cifar10")
    opt.optimize()
    return finish(opt, model, args)


if __name__ == "__main__":
    main(sys.argv[1:])
