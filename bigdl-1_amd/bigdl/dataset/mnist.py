"""``bigdl.dataset.mnist`` (``PY/dataset/mnist.py``): idx-format MNIST readers.

``read_data_sets(dir, "train"|"test")`` → (images uint8 [N, 28, 28, 1], labels uint8 0-9);
``load_data(dir)`` → normalised float features and 1-based labels.
"""
from __future__ import annotations

import gzip

import numpy as np

from . import base
from .transformer import normalizer

SOURCE_URL = "http://yann.lecun.com/exdb/mnist/"
TRAIN_MEAN = 0.13066047740239506 * 255
TRAIN_STD = 0.3081078 * 255
TEST_MEAN = 0.13251460696903547 * 255
TEST_STD = 0.31048024 * 255


def extract_images(f) -> np.ndarray:
    """4-D uint8 [index, y, x, depth] from an (optionally gzipped) idx3 stream."""
    data = f.read()
    if data[:2] == b"\x1f\x8b":
        data = gzip.decompress(data)
    magic, n, r, c = np.frombuffer(data[:16], dtype=">u4")
    if magic != 2051:
        raise ValueError(f"Invalid magic number {magic} in MNIST image file")
    return np.frombuffer(data[16:16 + n * r * c], dtype=np.uint8).reshape(n, r, c, 1)


def extract_labels(f) -> np.ndarray:
    data = f.read()
    if data[:2] == b"\x1f\x8b":
        data = gzip.decompress(data)
    magic, n = np.frombuffer(data[:8], dtype=">u4")
    if magic != 2049:
        raise ValueError(f"Invalid magic number {magic} in MNIST label file")
    return np.frombuffer(data[8:8 + n], dtype=np.uint8)


def read_data_sets(train_dir, data_type="train"):
    pre = "train" if data_type == "train" else "t10k"
    img = base.maybe_download(f"{pre}-images-idx3-ubyte.gz", train_dir, SOURCE_URL)
    lab = base.maybe_download(f"{pre}-labels-idx1-ubyte.gz", train_dir, SOURCE_URL)
    with open(img, "rb") as fi, open(lab, "rb") as fl:
        return extract_images(fi), extract_labels(fl)


def load_data(location="/tmp/mnist"):
    (x_tr, y_tr) = read_data_sets(location, "train")
    (x_te, y_te) = read_data_sets(location, "test")
    return (normalizer(x_tr, TRAIN_MEAN, TRAIN_STD), y_tr + 1), (normalizer(x_te, TRAIN_MEAN, TRAIN_STD), y_te + 1)
