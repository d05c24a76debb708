"""``bigdl.dataset.sentence`` (``PY/dataset/sentence.py``): sentence split / tokenize / bi-padding."""
from __future__ import annotations

import re

SENTENCE_START = "SENTENCESTART"
SENTENCE_END = "SENTENCEEND"


def read_localfile(fileName):
    with open(fileName) as f:
        return [line.strip() for line in f]


def sentences_split(line):
    """Split a paragraph into sentences (on . ! ? followed by whitespace)."""
    return [s for s in re.split(r"(?<=[.!?])\s+", line.strip()) if s]


def sentences_bipadding(sent):
    return f"{SENTENCE_START} {sent} {SENTENCE_END}"


def sentence_tokenizer(sentences):
    return re.findall(r"\w+|[^\w\s]", sentences)
