"""PTB language model (``DL/models/rnn/Train.scala``, ``DL/example/languagemodel/PTBWordLM.scala``).

Data: ``--folder`` with ``ptb.train.txt`` / ``ptb.valid.txt`` (whitespace tokens; the vocabulary is
built from the training text, ``--vocabSize`` most frequent words, the rest → <unk>) or
``--synthetic N`` (N random tokens).  The token stream is cut into ``batchSize`` parallel streams
of ``numSteps``-long windows (the reference's PTB reader), the model is PTBModel.lstm (embedding →
numLayers × LSTM → TimeDistributed Linear) trained with TimeDistributedCriterion(CrossEntropy,
sizeAverage=false) and Adagrad(lr 0.01, decay 0.001); validation reports Loss (perplexity =
exp(loss / numSteps)).
"""
from __future__ import annotations

import collections
import math
import os
import sys

import numpy as np
import torch

from .common import assemble, base_parser, finish, init_engine, load_model_or, log, optim_or, per_rank_batch


def _tokens(path):
    with open(path) as f:
        return f.read().replace("\n", " <eos> ").split()


def build_vocab(words, size):
    cnt = collections.Counter(words)
    vocab = ["<unk>"] + [w for w, _ in cnt.most_common(size - 1) if w != "<unk>"]
    return {w: i + 1 for i, w in enumerate(vocab[:size])}  # 1-based ids (LookupTable)


def windows(ids, batch, steps):
    """(inputs, targets) MiniBatches of [batch, steps] windows over ``batch`` parallel streams."""
    from ...dataset import MiniBatch
    n = (len(ids) - 1) // batch
    data = np.asarray(ids[:n * batch + 1], dtype=np.float32)
    x = data[:-1].reshape(batch, n)
    y = data[1:].reshape(batch, n)
    out = []
    for i in range(0, n - steps + 1, steps):
        out.append(MiniBatch(torch.from_numpy(x[:, i:i + steps].copy()), torch.from_numpy(y[:, i:i + steps].copy())))
    return out


def main(argv=None):
    ap = base_parser("Train the PTB LSTM language model", batch=20, epochs=13, lr=0.01)
    ap.add_argument("--vocabSize", type=int, default=10000)
    ap.add_argument("--hiddenSize", type=int, default=200)
    ap.add_argument("--numLayers", type=int, default=2)
    ap.add_argument("--numSteps", type=int, default=20)
    ap.add_argument("--keepProb", type=float, default=2.0)
    args = ap.parse_args(argv)
    Engine = init_engine(args)
    from ...models.rnn import PTBModel
    from ...nn import CrossEntropyCriterion, TimeDistributedCriterion
    from ...optim import Adagrad
    from ...optim.validation import Loss
    batch = per_rank_batch(args)
    if args.synthetic:
        g = np.random.default_rng(args.seed)
        tr_ids = list(g.integers(1, args.vocabSize + 1, args.synthetic))
        va_ids = list(g.integers(1, args.vocabSize + 1, max(args.synthetic // 4, batch * args.numSteps + 1)))
    else:
        if not args.folder:
            raise SystemExit("--folder (ptb.train.txt / ptb.valid.txt) or --synthetic N is required")
        tr_w = _tokens(os.path.join(args.folder, "ptb.train.txt"))
        vocab = build_vocab(tr_w, args.vocabSize)
        tr_ids = [vocab.get(w, 1) for w in tr_w]
        va_ids = [vocab.get(w, 1) for w in _tokens(os.path.join(args.folder, "ptb.valid.txt"))]
    # each rank takes its own contiguous slice of the token stream
    r, w = Engine.rank(), Engine.world_size()
    per = len(tr_ids) // w
    train = windows(tr_ids[r * per:(r + 1) * per], batch, args.numSteps)
    val = windows(va_ids, batch, args.numSteps)
    log.info(f"PTB: {len(train)} train windows × {batch}×{args.numSteps} per rank, {len(val)} valid windows")
    model = load_model_or(args, lambda: PTBModel.lstm(args.vocabSize, args.hiddenSize, args.vocabSize,
                                                      args.numLayers, args.keepProb))
    crit = TimeDistributedCriterion(CrossEntropyCriterion(), False)
    optim = optim_or(args, lambda: Adagrad(learningrate=args.learningRate, learningrate_decay=0.001))
    opt = assemble(model, train, crit, optim, args, val, [Loss(crit)], batch, app="ptb-lm")
    opt.optimize()
    out = finish(opt, model, args)
    if "Loss" in out:
        out["perplexity"] = math.exp(min(50.0, float(out["Loss"]) / args.numSteps))
    return out


if __name__ == "__main__":
    main(sys.argv[1:])
