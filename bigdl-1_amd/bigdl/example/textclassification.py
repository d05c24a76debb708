"""Text classification (``DL/example/textclassification/TextClassifier.scala``,
``example/utils/TextClassifier.scala:171-184``): tokens → pre-trained word vectors (GloVe) →
TemporalConvolution(embeddingDim, 256, 5) → ReLU → TemporalMaxPooling(seqLen − 4) → Squeeze →
Linear(256, 128) → Dropout(0.2) → ReLU → Linear(128, classes) → LogSoftMax, Adagrad(lr 0.01,
decay 0.0002), ClassNLL.  Data: ``--folder`` with the 20 Newsgroups tree + ``glove.6B.<dim>d.txt``
(``bigdl.dataset.news20``), or ``--synthetic N`` documents.
"""
from __future__ import annotations

import argparse
import re
import sys

import numpy as np
import torch


def build_model(class_num: int, embedding_dim: int = 100, seq_len: int = 500):
    from ..nn import Dropout, Linear, LogSoftMax, ReLU, Sequential, Squeeze, TemporalConvolution, TemporalMaxPooling
    return (Sequential().add(TemporalConvolution(embedding_dim, 256, 5)).add(ReLU())
            .add(TemporalMaxPooling(seq_len - 5 + 1)).add(Squeeze(2))
            .add(Linear(256, 128)).add(Dropout(0.2)).add(ReLU()).add(Linear(128, class_num)).add(LogSoftMax()))


def tokenize(text: str):
    return [w for w in re.split(r"\W+", text.lower()) if w]


def vectorize(docs, word2vec: dict, dim: int, seq_len: int) -> torch.Tensor:
    """[N, seqLen, dim]: each document's first seqLen known words (zero-padded)."""
    out = np.zeros((len(docs), seq_len, dim), dtype=np.float32)
    for i, d in enumerate(docs):
        vs = [word2vec[w] for w in tokenize(d) if w in word2vec][:seq_len]
        if vs:
            out[i, :len(vs)] = np.stack(vs)
    return torch.from_numpy(out)


def synthetic_corpus(n: int, classes: int, seed: int = 1, vocab: int = 200, dim: int = 20):
    """Documents whose class is carried by class-specific keywords, plus a random word2vec."""
    g = np.random.default_rng(seed)
    words = [f"w{i}" for i in range(vocab)]
    w2v = {w: g.normal(0, 1, dim).astype(np.float32) for w in words}
    docs, labels = [], []
    for _ in range(n):
        c = int(g.integers(0, classes))
        body = list(g.choice(words[classes * 5:], 30)) + [words[c * 5 + int(k)] for k in g.integers(0, 5, 8)]
        g.shuffle(body)
        docs.append(" ".join(body))
        labels.append(c + 1)
    return docs, labels, w2v


def train(docs, labels, w2v, dim, seq_len, classes, batch, epochs, lr=0.01, max_iter=None):
    from ..dataset import MiniBatch
    from ..nn import ClassNLLCriterion
    from ..optim import Adagrad, MaxIteration, Top1Accuracy, Trigger
    from ..optim.optimizer import Optimizer
    x = vectorize(docs, w2v, dim, seq_len)
    y = torch.tensor(labels, dtype=torch.float32)
    ntr = int(0.8 * len(docs))
    tr = [MiniBatch(x[i:i + batch], y[i:i + batch]) for i in range(0, ntr - batch + 1, batch)]
    va = [MiniBatch(x[i:i + batch], y[i:i + batch]) for i in range(ntr, len(docs), batch)]
    model = build_model(classes, dim, seq_len)
    opt = Optimizer.create(model, tr, ClassNLLCriterion(), batch_size=batch,
                           optim_method=Adagrad(learningrate=lr, learningrate_decay=0.0002))
    opt.setEndWhen(MaxIteration(max_iter) if max_iter else Trigger.maxEpoch(epochs))
    opt.setValidation(Trigger.everyEpoch(), va, [Top1Accuracy()], batch)
    opt.optimize()
    res = opt.validate()
    return model, (res[0][1].result()[0] if res else None)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("-f", "--folder", default=None)
    ap.add_argument("--embeddingDim", type=int, default=100)
    ap.add_argument("--maxSequenceLength", type=int, default=500)
    ap.add_argument("-b", "--batchSize", type=int, default=128)
    ap.add_argument("-e", "--maxEpoch", type=int, default=20)
    ap.add_argument("--learningRate", type=float, default=0.01)
    ap.add_argument("--synthetic", type=int, default=0)
    a = ap.parse_args(argv)
    from ..utils.engine import Engine
    Engine.init()
    if a.synthetic:
        docs, labels, w2v = synthetic_corpus(a.synthetic, 4)
        dim, classes = 20, 4
    else:
        from ..dataset import news20
        texts = news20.get_news20(a.folder)
        docs, labels = [t for t, _ in texts], [l for _, l in texts]
        w2v = news20.get_glove_w2v(a.folder, a.embeddingDim)
        dim, classes = a.embeddingDim, max(labels)
    _, acc = train(docs, labels, w2v, dim, a.maxSequenceLength, classes, a.batchSize, a.maxEpoch, a.learningRate)
    print(f"Top1Accuracy {acc}")
    return acc


if __name__ == "__main__":
    main(sys.argv[1:])
