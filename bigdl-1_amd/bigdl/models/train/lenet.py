"""LeNet-5 on MNIST (``DL/models/lenet/Train.scala``, ``Test.scala``).

Data: ``--folder`` with the MNIST idx files (``train-images-idx3-ubyte[.gz]`` …) or
``--synthetic N``.  SGD(lr 0.05, decay 0.0) with ClassNLLCriterion, Top-1 + Loss validation every
epoch, batch 128 (the reference defaults); ``--test`` evaluates ``--model`` on the test set.
"""
from __future__ import annotations

import sys

from .common import (assemble, base_parser, evaluate, finish, image_loader, init_engine, load_model_or, log,
                     optim_or, per_rank_batch, synthetic_images)

MEAN = [0.13066047740239506 * 255]
STD = [0.3081078 * 255]


def main(argv=None):
    ap = base_parser("Train LeNet-5 on MNIST", batch=128, epochs=15, lr=0.05)
    ap.add_argument("--test", action="store_true")
    args = ap.parse_args(argv)
    Engine = init_engine(args)
    from ...models.lenet import LeNet5
    from ...nn import ClassNLLCriterion
    from ...optim import SGD
    from ...optim.validation import Top1Accuracy, Loss
    batch = per_rank_batch(args)
    if args.synthetic:
        tr = synthetic_images(args.synthetic, 28, 28, 1, 10, args.seed)
        te = synthetic_images(max(batch, args.synthetic // 4), 28, 28, 1, 10, args.seed + 1)
    else:
        if not args.folder:
            raise SystemExit("--folder (MNIST idx files) or --synthetic N is required")
        from ...dataset.mnist import read_data_sets
        x, y = read_data_sets(args.folder, "train")
        tr = (x, y.astype("float32") + 1)
        x, y = read_data_sets(args.folder, "test")
        te = (x, y.astype("float32") + 1)
    # LeNet reshapes its input itself; the loader hands over NCHW 1×28×28 in the compute dtype
    train = image_loader(tr[0], tr[1], batch, None, True, MEAN, STD, args, flip=False, layout="NCHW")
    test = image_loader(te[0], te[1], batch, None, False, MEAN, STD, args, layout="NCHW")
    model = load_model_or(args, lambda: LeNet5(10))
    if args.test:
        model.to(Engine.device())
        res = evaluate(model, test, [Top1Accuracy()], Engine.device())
        for m, r in res:
            log.info(f"{m.format()} is {r}")
        return {m.format(): r.result()[0] for m, r in res}
    optim = optim_or(args, lambda: SGD(learningrate=args.learningRate, learningrate_decay=args.learningRateDecay))
    opt = assemble(model, train, ClassNLLCriterion(), optim, args, test, [Top1Accuracy(), Loss()], batch,
                   app="lenet5")
    opt.optimize()
    return finish(opt, model, args)


if __name__ == "__main__":
    main(sys.argv[1:])
