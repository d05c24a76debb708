"""PTB word-level language model (``DL/example/languagemodel/{PTBWordLM,Utils}.scala``;
``DL/models/rnn/Utils.scala`` SequencePreprocess).

Data: ``--dataFolder`` with ``ptb.train.txt`` / ``ptb.valid.txt`` / ``ptb.test.txt`` (whitespace
tokens; every line ends with ``<eos>``).  The dictionary keeps the ``vocab − 1`` most frequent
training words (the rest share the unknown index), and each file becomes a stream of 1-based word
ids (``fileToWordIdx``).  ``reader`` cuts a stream into overlapping ``numSteps + 1`` slices every
``numSteps`` words; ``TextToSentenceWithSteps`` splits each slice into (words, next words) and
``LabeledSentenceToSample(oneHot = false)`` keeps the ids as they are.  The model is
``PTBModel.lstm`` (or ``PTBModel.transformer`` with ``--withTransformerModel``), trained with
``TimeDistributedCriterion(CrossEntropyCriterion, sizeAverage = false, dimension = 1)`` and
Adagrad(lr, lrDecay); validation reports that loss every epoch; ``--test`` also scores the test
split (perplexity = exp(loss / numSteps)).

    python -m bigdl.example.languagemodel -f <ptb folder> -b 20 [--checkpoint DIR] [-e 4]
"""
from __future__ import annotations

import argparse
import logging
import math
import os
import sys
from typing import List, Tuple

log = logging.getLogger("bigdl.example.languagemodel")


def read_words(path: str) -> List[str]:
    """Tokens of a PTB file, ``<eos>`` after every line (``SequencePreprocess.readWords``)."""
    out: List[str] = []
    with open(path) as f:
        for line in f:
            out.extend(line.rstrip("\n").split(" "))
            out.append("<eos>")
    return out


def sequence_preprocess(folder: str, vocab_size: int) -> Tuple[List[float], List[float], List[float], object]:
    """(train ids, valid ids, test ids, Dictionary) — ``SequencePreprocess(dataFolder, vocabSize)``."""
    from ..dataset.text import Dictionary
    paths = [os.path.join(folder, f"ptb.{s}.txt") for s in ("train", "valid", "test")]
    for p in paths:
        if not os.path.exists(p):
            raise FileNotFoundError(f"data file {p} not exists!")
    dictionary = Dictionary(read_words(paths[0]), vocab_size - 1)
    streams = [[float(dictionary.get_index(w)) + 1.0 for w in read_words(p)] for p in paths]
    return streams[0], streams[1], streams[2], dictionary


def reader(raw: List[float], num_steps: int) -> List[List[float]]:
    """Slices of ``num_steps + 1`` ids starting every ``num_steps`` ids (``SequencePreprocess.reader``)."""
    out, off = [], 0
    while off <= len(raw) - 1 - num_steps:
        out.append(raw[off:off + num_steps + 1])
        off += num_steps
    return out


def to_dataset(ids: List[float], num_steps: int, batch: int):
    from ..dataset.core import DataSet, SampleToMiniBatch
    from ..dataset.text import LabeledSentenceToSample, TextToSentenceWithSteps
    return (DataSet.array(reader(ids, num_steps)) >> TextToSentenceWithSteps(num_steps)
            >> LabeledSentenceToSample(0, one_hot=False) >> SampleToMiniBatch(batch))


def _parser():
    ap = argparse.ArgumentParser(description="BigDL ptbModel Train Example", add_help=False)
    ap.add_argument("--help", action="help")
    ap.add_argument("-f", "--dataFolder", required=True, help="where you put the text data")
    ap.add_argument("--model", dest="modelSnapshot", help="model snapshot location")
    ap.add_argument("--state", dest="stateSnapshot", help="state snapshot location")
    ap.add_argument("--checkpoint", help="where to cache the model and state")
    ap.add_argument("-b", "--batchSize", type=int, required=True)
    ap.add_argument("-r", "--learningRate", type=float, default=0.01)
    ap.add_argument("--learningRateDecay", type=float, default=0.001)
    ap.add_argument("-h", "--hidden", dest="hiddenSize", type=int, default=200)
    ap.add_argument("--vocab", dest="vocabSize", type=int, default=10000)
    ap.add_argument("-e", "--nEpochs", type=int, default=4)
    ap.add_argument("--numLayers", type=int, default=2)
    ap.add_argument("--numSteps", type=int, default=20)
    ap.add_argument("--overWrite", dest="overWriteCheckpoint", action="store_true")
    ap.add_argument("--keepProb", type=float, default=2.0)
    ap.add_argument("--withTransformerModel", action="store_true")
    ap.add_argument("--test", action="store_true", help="also report the test-split loss / perplexity")
    return ap


def _criterion():
    from ..nn import CrossEntropyCriterion, TimeDistributedCriterion
    return TimeDistributedCriterion(CrossEntropyCriterion(), size_average=False, dimension=1)


def main(argv=None):
    a = _parser().parse_args(argv)
    from ..models.rnn import PTBModel
    from ..nn.module import Module
    from ..optim import Adagrad
    from ..optim.optim_method import OptimMethod
    from ..optim.optimizer import Optimizer
    from ..optim.trigger import Trigger
    from ..optim.validation import Loss
    from ..utils.engine import Engine
    Engine.init()
    train, valid, test, dictionary = sequence_preprocess(a.dataFolder, a.vocabSize)
    log.info(f"vocabulary {dictionary.get_vocab_size()}, train {len(train)} / valid {len(valid)} / "
             f"test {len(test)} words")
    train_set = to_dataset(train, a.numSteps, a.batchSize)
    valid_set = to_dataset(valid, a.numSteps, a.batchSize)
    if a.modelSnapshot:
        model = Module.loadModule(a.modelSnapshot)
    elif a.withTransformerModel:
        model = PTBModel.transformer(a.vocabSize, a.hiddenSize, a.vocabSize, a.numLayers, a.keepProb)
    else:
        model = PTBModel.lstm(a.vocabSize, a.hiddenSize, a.vocabSize, a.numLayers, a.keepProb)
    method = (OptimMethod.load(a.stateSnapshot) if a.stateSnapshot
              else Adagrad(learningrate=a.learningRate, learningrate_decay=a.learningRateDecay))
    opt = Optimizer(model, train_set, _criterion(), batch_size=a.batchSize)
    if a.checkpoint:
        opt.setCheckpoint(a.checkpoint, Trigger.everyEpoch())
    if a.overWriteCheckpoint:
        opt.overWriteCheckpoint()
    opt.setValidation(Trigger.everyEpoch(), valid_set, [Loss(_criterion())], a.batchSize)
    opt.setOptimMethod(method)
    opt.setEndWhen(Trigger.maxEpoch(a.nEpochs))
    trained = opt.optimize()
    if a.test:
        res = trained.evaluate(to_dataset(test, a.numSteps, a.batchSize), [Loss(_criterion())])
        loss = res[0][0].result()[0]
        log.info(f"test loss {loss:.4f}, perplexity {math.exp(loss / a.numSteps):.2f}")
        return trained, loss
    return trained


if __name__ == "__main__":
    main(sys.argv[1:])
