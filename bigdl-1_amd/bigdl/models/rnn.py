"""Recurrent model zoo.

* ``PTBModel.lstm`` — ``DL/example/languagemodel/PTBModel.scala``: LookupTable(vocab, H) →
  [Dropout(keepProb) when keepProb < 1 — the reference passes keepProb as the *drop*
  probability, kept as-is] → numLayers × Recurrent(LSTM(H, H)) → TimeDistributed(Linear(H, vocab)).
  Trained with TimeDistributedCriterion(CrossEntropyCriterion, sizeAverage=false) and Adagrad
  (lr 0.01, decay 0.001), batch 20, 20 steps (``languagemodel/Utils.scala:44-53``).
* ``PTBModel.transformer`` — Transformer LM variant of the same example.
* ``SimpleRNN`` — ``DL/models/rnn/SimpleRNN.scala``: Recurrent(RnnCell(tanh)) →
  TimeDistributed(Linear).
"""
from __future__ import annotations

from ..nn import (Dropout, Graph, Input, Linear, LookupTable, LSTM, Recurrent, RnnCell, Sequential, Tanh,
                  TimeDistributed)


class PTBModel:
    @staticmethod
    def lstm(input_size=10000, hidden_size=200, output_size=10000, num_layers=2, keep_prob=2.0):
        inp = Input()
        x = LookupTable(input_size, hidden_size)(inp)
        if keep_prob < 1:
            x = Dropout(keep_prob)(x)
        in_size = hidden_size
        for _ in range(num_layers):
            x = Recurrent().add(LSTM(in_size, hidden_size))(x)
        out = TimeDistributed(Linear(hidden_size, output_size))(x)
        return Graph(inp, out)

    @staticmethod
    def transformer(input_size=10000, hidden_size=256, output_size=10000, num_layers=2, keep_prob=2.0):
        from ..nn.layers.attention import Transformer
        inp = Input()
        t = Transformer(vocab_size=input_size, hidden_size=hidden_size, num_heads=4, filter_size=hidden_size * 4,
                        num_hidden_layers=num_layers, embedding_dropout=1 - keep_prob, attention_dropout=0.1,
                        ffn_dropout=0.1)(inp)
        out = TimeDistributed(Linear(hidden_size, output_size))(t)
        return Graph(inp, out)


def SimpleRNN(input_size, hidden_size, output_size):
    return (Sequential()
            .add(Recurrent().add(RnnCell(input_size, hidden_size, Tanh())))
            .add(TimeDistributed(Linear(hidden_size, output_size))))
