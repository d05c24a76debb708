"""PTB word language model (``DL/example/languagemodel/PTBWordLM.scala``): the same program as the
model-zoo trainer :mod:`bigdl.models.train.rnn` (PTBModel.lstm, Adagrad, TimeDistributedCriterion)."""
import sys

from ..models.train.rnn import main

if __name__ == "__main__":
    main(sys.argv[1:])
