"""Dataset file readers used by the examples (``pyspark/bigdl/dataset/{mnist,news20,movielens}.py``,
``DL/models/lenet/Utils.scala``, ``DL/models/vgg/Utils.scala``).  There is no network access, so
every reader parses files that are already on disk."""
from __future__ import annotations

import gzip
import os
import struct
from typing import List, Tuple

import numpy as np

TRAIN_MEAN, TRAIN_STD = 0.13066047740239506, 0.3081078
TEST_MEAN, TEST_STD = 0.13251460696903547, 0.31048024


def _open(path):
    return gzip.open(path, "rb") if path.endswith(".gz") else open(path, "rb")


def read_idx_images(path: str) -> np.ndarray:
    with _open(path) as f:
        magic, n, r, c = struct.unpack(">IIII", f.read(16))
        if magic != 2051:
            raise ValueError(f"{path}: bad MNIST image magic {magic}")
        return np.frombuffer(f.read(n * r * c), dtype=np.uint8).reshape(n, r, c)


def read_idx_labels(path: str) -> np.ndarray:
    with _open(path) as f:
        magic, n = struct.unpack(">II", f.read(8))
        if magic != 2049:
            raise ValueError(f"{path}: bad MNIST label magic {magic}")
        return np.frombuffer(f.read(n), dtype=np.uint8)


def load_mnist(folder: str, kind: str = "train") -> Tuple[np.ndarray, np.ndarray]:
    """(images [N, 28, 28] uint8, labels [N] 1-based float) from the standard idx files."""
    pre = "train" if kind == "train" else "t10k"
    cands = [f"{pre}-images-idx3-ubyte", f"{pre}-images.idx3-ubyte"]
    img = next((os.path.join(folder, c + s) for c in cands for s in ("", ".gz")
                if os.path.exists(os.path.join(folder, c + s))), None)
    lab = next((os.path.join(folder, f"{pre}-labels-idx1-ubyte" + s) for s in ("", ".gz")
                if os.path.exists(os.path.join(folder, f"{pre}-labels-idx1-ubyte" + s))), None)
    if img is None or lab is None:
        raise FileNotFoundError(f"MNIST idx files not found in {folder}")
    return read_idx_images(img), read_idx_labels(lab).astype(np.float32) + 1


def load_cifar10_bin(folder: str, train: bool = True) -> Tuple[np.ndarray, np.ndarray]:
    """CIFAR-10 binary batches → (images [N, 32, 32, 3] uint8 BGR, labels 1-based)."""
    files = [f"data_batch_{i}.bin" for i in range(1, 6)] if train else ["test_batch.bin"]
    xs, ys = [], []
    for fn in files:
        raw = np.fromfile(os.path.join(folder, fn), dtype=np.uint8).reshape(-1, 3073)
        ys.append(raw[:, 0].astype(np.float32) + 1)
        rgb = raw[:, 1:].reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1)
        xs.append(rgb[..., ::-1].copy())
    return np.concatenate(xs), np.concatenate(ys)


def load_news20(folder: str) -> List[Tuple[str, int]]:
    """20 Newsgroups directory tree → [(text, 1-based label)]."""
    out = []
    cats = sorted(d for d in os.listdir(folder) if os.path.isdir(os.path.join(folder, d)))
    for li, c in enumerate(cats):
        for fn in sorted(os.listdir(os.path.join(folder, c))):
            with open(os.path.join(folder, c, fn), encoding="latin-1") as f:
                out.append((f.read(), li + 1))
    return out


def load_glove(path: str, dim: int = 100) -> dict:
    w2v = {}
    with open(path, encoding="utf-8") as f:
        for line in f:
            parts = line.rstrip().split(" ")
            if len(parts) == dim + 1:
                w2v[parts[0]] = np.asarray(parts[1:], dtype=np.float32)
    return w2v


def load_movielens(path: str) -> np.ndarray:
    """``ratings.dat`` (``user::item::rating::ts``) → int array [N, 3]."""
    rows = []
    with open(path) as f:
        for line in f:
            p = line.strip().split("::")
            if len(p) >= 3:
                rows.append((int(p[0]), int(p[1]), int(p[2])))
    return np.asarray(rows, dtype=np.int64)
