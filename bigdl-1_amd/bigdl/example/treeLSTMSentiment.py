"""Tree-LSTM sentiment on the Stanford Sentiment Treebank
(``DL/example/treeLSTMSentiment/{Train,TreeSentiment,Utils}.scala``).

Data layout under ``--baseDir`` (the reference's ``fetch_and_preprocess.py`` output):
``glove/glove.840B.300d.txt`` (word vectors), ``sst/vocab-cased.txt`` and per split
``sst/{train,dev}/{parents,labels,sents}.txt`` (one sentence per line: the constituency-tree parent
pointers, the per-node labels in [-2, 2] and the tokens).

Each tree becomes the ``TensorTree`` matrix of ``readTree`` (root = node 1, leaves numbered in
order), labels are shifted to 1..5 (``remapLabel``) and rotated so the root's label comes first,
tokens map to vocabulary ids (out-of-vocabulary → 2, ids from 3).  The model is
``TreeLSTMSentiment(word2vec, hidden, 5, p)`` trained with ``TimeDistributedCriterion(ClassNLL)``
(label padding −1), Adagrad(lr, weight decay = regRate), batches padded with token 1 / tree rows
−1, and ``TreeNNAccuracy`` (root prediction) on the dev split every epoch.

    python -m bigdl.example.treeLSTMSentiment -b <baseDir> [-i 128] [-h 250] [-l 0.05] [-r 1e-4]
        [-p 0.5] [-e 5]
"""
from __future__ import annotations

import argparse
import logging
import os
import sys
from typing import Dict, List, Sequence, Tuple

import torch

log = logging.getLogger("bigdl.example.treeLSTMSentiment")

PADDING_VALUE, OOV_CHAR, INDEX_FROM, LABEL_PADDING = 1, 2, 3, -1.0


def read_tree(parents: Sequence[int]) -> torch.Tensor:
    """Parent-pointer array (1-based parents, 0 = root's parent … as SST's parents.txt) → the
    [size, maxChildren + 1] TensorTree content with node 1 the root (``Utils.readTree``)."""
    from ..nn.layers.tree_lstm import TensorTree
    size = len(parents)
    counts: Dict[int, int] = {}
    for p in parents:
        counts[p] = counts.get(p, 0) + 1
    max_children = max(counts.values()) if counts else 0
    trees = TensorTree(torch.zeros(size, max_children + 1))
    for i in range(size):
        if trees.noChild(i + 1) and parents[i] != -1:
            idx, prev = i + 1, 0
            while True:
                parent = parents[idx - 1] if idx != 0 else -1
                if parent == size:
                    parent = 0
                if prev != 0 and parent != -1:
                    trees.addChild(idx + 1, prev + 1)
                if parent == -1:
                    trees.markAsRoot(1)
                    if prev != 0:
                        trees.addChild(1, prev + 1)
                    break
                elif trees.hasChild(parent + 1):
                    trees.addChild(parent + 1, idx + 1)
                    break
                else:
                    prev, idx = idx, parent
    leaf = 1
    for i in range(2, size + 1):
        if trees.noChild(i):
            trees.markAsLeaf(i, leaf)
            leaf += 1
    return trees.content


def remap_label(label: float) -> float:
    return label + 3


def rotate(arr: List, offset: int) -> List:
    """Right-rotate ``arr`` by ``offset`` (``Utils.rotate``)."""
    if not arr or offset < 0:
        raise ValueError("Illegal argument!")
    k = offset % len(arr) if offset > len(arr) else offset
    return arr[len(arr) - k:] + arr[:len(arr) - k]


def pre_process_data(vocab: Dict[str, int], oov_char: int, tree_path: str, label_path: str, sentence_path: str):
    with open(tree_path) as f:
        trees = [read_tree([int(t) for t in line.split()]) for line in f if line.strip()]
    with open(label_path) as f:
        labels = [rotate([remap_label(float(t)) for t in line.split()], 1) for line in f if line.strip()]
    with open(sentence_path) as f:
        sentences = [[vocab.get(w, oov_char) for w in line.split()] for line in f if line.strip()]
    return trees, labels, sentences


def to_samples(trees, labels, sentences):
    from ..dataset.core import Sample
    out = []
    for sent, lab, tree in zip(sentences, labels, trees):
        out.append(Sample([torch.tensor(sent, dtype=torch.float32).view(len(sent), 1), tree],
                          torch.tensor(lab, dtype=torch.float32)))
    return out


def load_embedding_and_vocabulary(w2v_path: str, vocab_path: str, index_from: int) -> Tuple[torch.Tensor, Dict]:
    """GloVe text vectors + vocabulary file → (word2vec [len(vocab) + indexFrom − 1, dim], word → id);
    ids below ``index_from`` and words without a vector get U(−0.05, 0.05) rows."""
    from ..utils.random import RNG
    w2v: Dict[str, List[float]] = {}
    dim = 0
    with open(w2v_path, encoding="utf-8") as f:
        for line in f:
            vals = line.rstrip("\n").split(" ")
            if len(vals) < 2:
                continue
            w2v[vals[0]] = [float(v) for v in vals[1:]]
            dim = len(vals) - 1
    with open(vocab_path, encoding="utf-8") as f:
        words = [ln.rstrip("\n") for ln in f if ln.rstrip("\n")]
    table = torch.empty(len(words) + index_from - 1, dim)
    for i in range(index_from - 1):
        table[i].copy_(torch.tensor([RNG.uniform(-0.05, 0.05) for _ in range(dim)]))
    vocab = {}
    for k, w in enumerate(words):
        i = index_from - 1 + k
        if w in w2v:
            table[i].copy_(torch.tensor(w2v[w]))
        else:
            table[i].copy_(torch.tensor([RNG.uniform(-0.05, 0.05) for _ in range(dim)]))
        vocab[w] = i + 1
    return table, vocab


def _parser():
    ap = argparse.ArgumentParser(description="TreeLSTM Sentiment", add_help=False)
    ap.add_argument("--help", action="help")
    ap.add_argument("-b", "--baseDir", default="/tmp/.bigdl/dataset/")
    ap.add_argument("-i", "--batchSize", type=int, default=128)
    ap.add_argument("-h", "--hiddenSize", type=int, default=250)
    ap.add_argument("-l", "--learingRate", "--learningRate", dest="learningRate", type=float, default=0.05)
    ap.add_argument("-r", "--regRate", type=float, default=1e-4)
    ap.add_argument("-p", "--p", type=float, default=0.5)
    ap.add_argument("-e", "--epoch", type=int, default=5)
    ap.add_argument("--glove", default="glove/glove.840B.300d.txt", help="GloVe file under baseDir")
    return ap


def _batched(samples, batch):
    from ..dataset.core import DataSet, PaddingParam, SampleToMiniBatch
    fp = PaddingParam([torch.tensor([float(PADDING_VALUE)]), torch.tensor([-1.0, -1.0, -1.0])])
    lp = PaddingParam([torch.tensor([LABEL_PADDING])])
    return DataSet.array(samples) >> SampleToMiniBatch(batch, fp, lp)


def train(a):
    from ..models.treelstm import TreeLSTMSentiment
    from ..nn import ClassNLLCriterion, TimeDistributedCriterion
    from ..optim import Adagrad
    from ..optim.optimizer import Optimizer
    from ..optim.trigger import Trigger
    from ..optim.validation import TreeNNAccuracy
    from ..utils.engine import Engine
    Engine.init()
    d = a.baseDir
    log.info("Start loading embeddings")
    w2v, vocab = load_embedding_and_vocabulary(os.path.join(d, a.glove), os.path.join(d, "sst/vocab-cased.txt"),
                                               INDEX_FROM)
    log.info("Finish loading embeddings")
    split = lambda s: pre_process_data(vocab, OOV_CHAR, *(os.path.join(d, "sst", s, f)  # noqa: E731
                                                          for f in ("parents.txt", "labels.txt", "sents.txt")))
    tr, de = split("train"), split("dev")
    log.info(f"train trees {len(tr[0])}, dev trees {len(de[0])}")
    model = TreeLSTMSentiment(w2v, a.hiddenSize, 5, a.p)
    opt = Optimizer(model, _batched(to_samples(*tr), a.batchSize), TimeDistributedCriterion(ClassNLLCriterion()),
                    batch_size=a.batchSize)
    opt.setOptimMethod(Adagrad(learningrate=a.learningRate, weightdecay=a.regRate))
    opt.setValidation(Trigger.everyEpoch(), _batched(to_samples(*de), a.batchSize), [TreeNNAccuracy()], a.batchSize)
    opt.setEndWhen(Trigger.maxEpoch(a.epoch))
    return opt.optimize()


def main(argv=None):
    return train(_parser().parse_args(argv))


if __name__ == "__main__":
    main(sys.argv[1:])
