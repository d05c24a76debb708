"""LeNet-5 in local mode, no cluster (``DL/example/lenetLocal/{Train,Test,Predict,Utils}.scala``).

The reference's local pipeline, transformer for transformer:
``DataSet.array(load(images, labels)) -> BytesToGreyImg(28, 28) -> GreyImgNormalizer(mean, std)
-> GreyImgToBatch(batch)`` into a local ``Optimizer`` (ClassNLLCriterion, SGD(lr, decay),
Top1/Top5/Loss validation every epoch, optional checkpoint / snapshot resume); ``test`` evaluates a
saved model (Top-1), ``predict`` prints ``LocalPredictor.predictClass`` of every test record.

    python -m bigdl.example.lenetLocal train -f <mnist dir> -b 12 -e 5 [--checkpoint dir]
    python -m bigdl.example.lenetLocal test -f <mnist dir> --model <snapshot>
    python -m bigdl.example.lenetLocal predict -f <mnist dir> --model <snapshot>

The MNIST folder holds the four idx files (``train-images-idx3-ubyte`` …, optionally ``.gz``).
"""
from __future__ import annotations

import argparse
import logging
import os
import sys

import numpy as np

log = logging.getLogger("bigdl.example.lenetLocal")

TRAIN_MEAN, TRAIN_STD = 0.13066047740239506, 0.3081078
TEST_MEAN, TEST_STD = 0.13251460696903547, 0.31048024


def _idx(folder, name):
    p = os.path.join(folder, name)
    return p if os.path.exists(p) else p + ".gz"


def load(feature_file: str, label_file: str):
    """MNIST idx files → ``ByteRecord`` s (28·28 raw bytes, 1-based label), as ``Utils.load``."""
    from ..dataset.image import ByteRecord
    from ..dataset.mnist import extract_images, extract_labels
    with open(feature_file, "rb") as fi, open(label_file, "rb") as fl:
        x, y = extract_images(fi), extract_labels(fl)
    if len(x) != len(y):
        raise ValueError(f"{len(x)} images but {len(y)} labels")
    return [ByteRecord(x[i].tobytes(), float(y[i]) + 1.0) for i in range(len(x))]


def _pipeline(records, mean, std, batch):
    from ..dataset.core import DataSet
    from ..dataset.image import BytesToGreyImg, GreyImgNormalizer, GreyImgToBatch
    return DataSet.array(records) >> BytesToGreyImg(28, 28) >> GreyImgNormalizer(mean, std) >> GreyImgToBatch(batch)


def _parser():
    ap = argparse.ArgumentParser(description="BigDL LeNet local example")
    sub = ap.add_subparsers(dest="cmd", required=True)
    tr = sub.add_parser("train")
    tr.add_argument("-f", "--folder", default="./")
    tr.add_argument("--checkpoint", default=None)
    tr.add_argument("--model", dest="modelSnapshot", default=None)
    tr.add_argument("--state", dest="stateSnapshot", default=None)
    tr.add_argument("-b", "--batchSize", type=int, default=12)
    tr.add_argument("-r", "--learningRate", type=float, default=0.05)
    tr.add_argument("-d", "--learningRateDecay", type=float, default=0.0)
    tr.add_argument("-e", "--maxEpoch", type=int, default=5)
    tr.add_argument("-c", "--coreNumber", type=int, default=max(1, (os.cpu_count() or 2) // 2))
    tr.add_argument("--overWrite", action="store_true")
    for name in ("test", "predict"):
        p = sub.add_parser(name)
        p.add_argument("-f", "--folder", default="./")
        p.add_argument("--model", required=True)
        p.add_argument("-b", "--batchSize", type=int, default=128)
        p.add_argument("-c", "--coreNumber", type=int, default=max(1, (os.cpu_count() or 2) // 2))
    return ap


def _engine(core_number):
    from ..utils import config
    from ..utils.engine import Engine
    config.set_property("bigdl.localMode", True)
    config.set_property("bigdl.coreNumber", int(core_number))
    Engine.init()


def train(args):
    from ..models.lenet import LeNet5
    from ..nn import ClassNLLCriterion
    from ..nn.module import Module
    from ..optim import SGD, OptimMethod
    from ..optim.optimizer import Optimizer
    from ..optim.trigger import Trigger
    from ..optim.validation import Top1Accuracy, Top5Accuracy, Loss
    _engine(args.coreNumber)
    model = Module.load(args.modelSnapshot) if args.modelSnapshot else LeNet5(10)
    optim = OptimMethod.load(args.stateSnapshot) if args.stateSnapshot else \
        SGD(learningrate=args.learningRate, learningrate_decay=args.learningRateDecay)
    tr = load(_idx(args.folder, "train-images-idx3-ubyte"), _idx(args.folder, "train-labels-idx1-ubyte"))
    va = load(_idx(args.folder, "t10k-images-idx3-ubyte"), _idx(args.folder, "t10k-labels-idx1-ubyte"))
    opt = Optimizer(model, _pipeline(tr, TRAIN_MEAN, TRAIN_STD, args.batchSize), ClassNLLCriterion(),
                    batch_size=args.batchSize)
    if args.checkpoint:
        opt.setCheckpoint(args.checkpoint, Trigger.everyEpoch())
    if args.overWrite:
        opt.overWriteCheckpoint()
    opt.setValidation(Trigger.everyEpoch(), _pipeline(va, TEST_MEAN, TEST_STD, args.batchSize),
                      [Top1Accuracy(), Top5Accuracy(), Loss()])
    opt.setOptimMethod(optim)
    opt.setEndWhen(Trigger.maxEpoch(args.maxEpoch))
    return opt.optimize()


def _test_samples(folder):
    from ..dataset.core import DataSet
    from ..dataset.image import BytesToGreyImg, GreyImgNormalizer, GreyImgToSample
    recs = load(_idx(folder, "t10k-images-idx3-ubyte"), _idx(folder, "t10k-labels-idx1-ubyte"))
    return DataSet.array(recs) >> BytesToGreyImg(28, 28) >> GreyImgNormalizer(TRAIN_MEAN, TRAIN_STD) >> \
        GreyImgToSample()


def test(args):
    from ..dataset.core import SampleToMiniBatch
    from ..nn.module import Module
    from ..optim.validation import Top1Accuracy
    _engine(args.coreNumber)
    model = Module.load(args.model)
    data = _test_samples(args.folder) >> SampleToMiniBatch(args.batchSize)
    res = model.evaluate(data.toLocal(), [Top1Accuracy()])
    for r, m in res:
        print(f"{m} is {r}")
    return res


def predict(args):
    from ..nn.module import Module
    from ..optim.predictor import LocalPredictor
    _engine(args.coreNumber)
    samples = list(_test_samples(args.folder).data(train=False))
    model = Module.load(args.model)
    pred = LocalPredictor(model)
    classes = np.asarray(pred.predict_class(samples))
    for c in classes:
        print(int(c))
    return classes


def main(argv=None):
    args = _parser().parse_args(argv)
    return {"train": train, "test": test, "predict": predict}[args.cmd](args)


if __name__ == "__main__":
    main(sys.argv[1:])
