"""Tree-LSTM sentiment model (``DL/example/treeLSTMSentiment/TreeSentiment.scala``):
``MapTable(Squeeze(3))`` → ``ParallelTable(LookupTable(word2vec, scaleW=2), Identity)`` →
``BinaryTreeLSTM(embed, hidden)`` → ``TimeDistributed(Dropout(p))`` →
``TimeDistributed(Linear(hidden, classNum))`` → ``TimeDistributed(LogSoftMax)``.
Trained with ``TimeDistributedMaskCriterion(ClassNLLCriterion(paddingValue=pad), pad)`` and
evaluated with ``TreeNNAccuracy`` (root node = node 1)."""
from __future__ import annotations

import torch

from ..nn import (BinaryTreeLSTM, Dropout, Identity, Linear, LogSoftMax, LookupTable, MapTable, ParallelTable,
                  Sequential, Squeeze, TimeDistributed)


def TreeLSTMSentiment(word2vec: torch.Tensor, hidden_size: int, class_num: int, p: float = 0.5):
    vocab, dim = word2vec.shape
    emb = LookupTable(vocab, dim)
    emb.weight.data.copy_(word2vec)
    emb.setScaleW(2)
    tree = (Sequential()
            .add(BinaryTreeLSTM(dim, hidden_size, with_graph=True))
            .add(TimeDistributed(Dropout(p)))
            .add(TimeDistributed(Linear(hidden_size, class_num)))
            .add(TimeDistributed(LogSoftMax())))
    return (Sequential()
            .add(MapTable(Squeeze(3)))
            .add(ParallelTable().add(emb).add(Identity()))
            .add(tree))
