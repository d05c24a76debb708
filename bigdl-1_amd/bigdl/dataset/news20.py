"""``bigdl.dataset.news20`` (``PY/dataset/news20.py``): 20 Newsgroups texts and GloVe vectors from
local directories (``20news-18828/<category>/<id>``, ``glove.6B/glove.6B.<dim>d.txt``)."""
from __future__ import annotations

import os

from . import base

NEWS20_URL = "http://qwone.com/~jason/20Newsgroups/20news-18828.tar.gz"
GLOVE_URL = "http://nlp.stanford.edu/data/glove.6B.zip"
CLASS_NUM = 20


def _find(dest_dir, name, url):
    p = os.path.join(dest_dir, name)
    if os.path.isdir(p):
        return p
    import tarfile
    import zipfile
    for arc in (p + ".tar.gz", p + ".zip", os.path.join(dest_dir, os.path.basename(url))):
        if os.path.exists(arc):
            if arc.endswith(".zip"):
                with zipfile.ZipFile(arc) as z:
                    z.extractall(p if name.startswith("glove") else dest_dir)
            else:
                with tarfile.open(arc) as t:
                    t.extractall(dest_dir)
            if os.path.isdir(p):
                return p
    return base.maybe_download(name, dest_dir, url)


def download_news20(dest_dir):
    return _find(dest_dir, "20news-18828", NEWS20_URL)


def download_glove_w2v(dest_dir):
    return _find(dest_dir, "glove.6B", GLOVE_URL)


def get_news20(source_dir="./data/news20/"):
    """[(text, 1-based label)] over the sorted category directories (numeric file names only)."""
    news_dir = download_news20(source_dir)
    texts, label = [], 0
    for name in sorted(os.listdir(news_dir)):
        path = os.path.join(news_dir, name)
        label += 1
        if os.path.isdir(path):
            for fname in sorted(os.listdir(path)):
                if fname.isdigit():
                    with open(os.path.join(path, fname), encoding="latin-1") as f:
                        texts.append((f.read(), label))
    return texts


def get_glove_w2v(source_dir="./data/news20/", dim=100):
    w2v_dir = download_glove_w2v(source_dir)
    out = {}
    with open(os.path.join(w2v_dir, f"glove.6B.{dim}d.txt"), encoding="latin-1") as f:
        for line in f:
            items = line.rstrip("\n").split(" ")
            out[items[0]] = [float(i) for i in items[1:]]
    return out
