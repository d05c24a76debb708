"""Text pipeline (``DL/dataset/text/*.scala``): Dictionary, SentenceSplitter, SentenceTokenizer,
SentenceBiPadding, TextToLabeledSentence, TextToSentenceWithSteps, LabeledSentenceToSample."""
from __future__ import annotations

import os
import random
import re
from collections import Counter
from typing import Iterable, Iterator, List, Optional, Sequence

import numpy as np
import torch

from .core import Sample, Transformer


class SentenceToken:
    start = "SENTENCESTART"
    end = "SENTENCEEND"


class Dictionary:
    """Word ↔ index map of the ``vocab_size`` most frequent words (ties keep the reference's
    ascending-frequency sort, most frequent last); unknown words map to ``vocab_size``."""

    def __init__(self, sentences=None, vocab_size: int = 10000, directory: Optional[str] = None):
        self._word2index, self._index2word = {}, {}
        self._vocabulary: List[str] = []
        self._discard: List[str] = []
        if directory is not None:
            self._load(directory)
        elif sentences is not None:
            words = []
            for s in sentences:
                if isinstance(s, str):
                    words.append(s)
                else:
                    words.extend(s)
            freq = sorted(Counter(words).items(), key=lambda kv: kv[1])
            self._update(freq, vocab_size)

    def _update(self, freq, vocab_size):
        n = min(vocab_size, len(freq))
        self._vocabulary = [w for w, _ in freq[len(freq) - n:]]
        self._word2index = {w: i for i, w in enumerate(self._vocabulary)}
        self._index2word = {i: w for w, i in self._word2index.items()}
        self._discard = [w for w, _ in freq[:len(freq) - n]]

    def _load(self, directory):
        with open(os.path.join(directory, "dictionary.txt")) as f:
            for line in f:
                line = line.rstrip("\n")
                if not line:
                    continue
                w, i = line.split("->", 1)
                self._word2index[w.rstrip(" ")] = int(i.lstrip(" "))
        self._index2word = {i: w for w, i in self._word2index.items()}
        self._vocabulary = list(self._word2index.keys())
        with open(os.path.join(directory, "discard.txt")) as f:
            self._discard = [l.rstrip("\n") for l in f if l.rstrip("\n")]

    def get_vocab_size(self) -> int:
        return len(self._vocabulary)

    getVocabSize = get_vocab_size

    def get_discard_size(self) -> int:
        return len(self._discard)

    getDiscardSize = get_discard_size

    def word2index(self):
        return dict(self._word2index)

    def index2word(self):
        return dict(self._index2word)

    def vocabulary(self):
        return list(self._vocabulary)

    def discard_vocab(self):
        return list(self._discard)

    discardVocab = discard_vocab

    def get_index(self, word: str) -> int:
        return self._word2index.get(word, len(self._vocabulary))

    getIndex = get_index

    def get_word(self, index) -> str:
        index = int(index)
        if index in self._index2word:
            return self._index2word[index]
        if self._discard:
            return random.choice(self._discard)
        return self.get_word(random.randrange(len(self._vocabulary)))

    getWord = get_word

    def save(self, folder: str):
        os.makedirs(folder, exist_ok=True)
        with open(os.path.join(folder, "dictionary.txt"), "w") as f:
            for w, i in self._word2index.items():
                f.write(f"{w} -> {i}\n")
        with open(os.path.join(folder, "discard.txt"), "w") as f:
            for w in self._discard:
                f.write(w + "\n")


_SENT_RE = re.compile(r"(?<=[.!?])\s+")
_TOKEN_RE = re.compile(r"[A-Za-z0-9]+(?:['’][A-Za-z]+)?|[^\sA-Za-z0-9]")


class SentenceSplitter(Transformer):
    """Paragraph → sentences (rule-based stand-in for the OpenNLP sentence model)."""

    def __init__(self, sent_file: Optional[str] = None):
        self.sent_file = sent_file

    def apply(self, it: Iterator[str]) -> Iterator[List[str]]:
        for text in it:
            yield [s.strip() for s in _SENT_RE.split(text.strip()) if s.strip()]


class SentenceTokenizer(Transformer):
    """Sentence → tokens (rule-based stand-in for the OpenNLP tokenizer)."""

    def __init__(self, token_file: Optional[str] = None):
        self.token_file = token_file

    def apply(self, it: Iterator[str]) -> Iterator[List[str]]:
        for s in it:
            yield _TOKEN_RE.findall(s)


class SentenceBiPadding(Transformer):
    def __init__(self, start: Optional[str] = None, end: Optional[str] = None):
        self.start = start or SentenceToken.start
        self.end = end or SentenceToken.end

    def apply(self, it):
        for s in it:
            yield f"{self.start} {s} {self.end}"


class LabeledSentence:
    def __init__(self, data: Sequence[float], label: Sequence[float]):
        self._data = np.asarray(data, dtype=np.float32)
        self._label = np.asarray(label, dtype=np.float32)

    def data(self):
        return self._data

    def label(self):
        return self._label

    def dataLength(self):
        return len(self._data)

    def labelLength(self):
        return len(self._label)

    def getData(self, i):
        return self._data[i]

    def getLabel(self, i):
        return self._label[i]


class TextToLabeledSentence(Transformer):
    """Token array → LabeledSentence(data = idx[:-1], label = idx[1:]) (next-word targets)."""

    def __init__(self, dictionary: Dictionary):
        self.dictionary = dictionary

    def apply(self, it):
        for sent in it:
            idx = [float(self.dictionary.get_index(w)) for w in sent]
            yield LabeledSentence(idx[:-1], idx[1:])


class TextToSentenceWithSteps(Transformer):
    """A flat index stream → LabeledSentences of ``num_steps`` (PTB-style language modelling)."""

    def __init__(self, num_steps: int):
        self.n = num_steps

    def apply(self, it):
        for arr in it:
            a = np.asarray(arr, dtype=np.float32)
            for i in range(0, len(a) - self.n - 1 + 1, self.n):
                yield LabeledSentence(a[i:i + self.n], a[i + 1:i + 1 + self.n])


class LabeledSentenceToSample(Transformer):
    """LabeledSentence → Sample (``dataset/text/LabeledSentenceToSample.scala``).

    ``one_hot`` (default): feature ``[len, vocab]`` one-hot of the 0-based word indices, rows past
    the sentence set at the END token (the last label); labels +1 (1-based class ids), padded with
    the START token (the first data index) + 1.  ``one_hot=False``: feature and label are the raw
    index arrays copied as they are (the PTB reader already made them 1-based), truncated or
    zero-padded to the fixed lengths."""

    def __init__(self, vocab_length: int, fix_data_length: Optional[int] = None,
                 fix_label_length: Optional[int] = None, one_hot: bool = True):
        self.V, self.fd, self.fl, self.one_hot = vocab_length, fix_data_length, fix_label_length, one_hot

    def apply(self, it):
        for s in it:
            dl = self.fd or s.dataLength()
            ll = self.fl or s.labelLength()
            if self.one_hot:
                start_tok = int(s.getData(0))
                end_tok = 0 if ll == 1 else int(s.getLabel(s.labelLength() - 1))
                feat = torch.zeros(dl, self.V)
                n = min(s.dataLength(), dl)
                feat[torch.arange(n), torch.as_tensor(s.data()[:n], dtype=torch.long)] = 1.0
                if n < dl:
                    feat[n:, end_tok] = 1.0
                lab = torch.full((ll,), float(start_tok + 1))
                m = min(s.labelLength(), ll)
                lab[:m] = torch.as_tensor(s.label()[:m]) + 1
            else:
                feat = torch.zeros(dl)
                n = min(s.dataLength(), dl)
                feat[:n] = torch.as_tensor(s.data()[:n])
                lab = torch.zeros(ll)
                m = min(s.labelLength(), ll)
                lab[:m] = torch.as_tensor(s.label()[:m])
            yield Sample(feat, lab)
