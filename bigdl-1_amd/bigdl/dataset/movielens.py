"""``bigdl.dataset.movielens`` (``PY/dataset/movielens.py``): MovieLens-1M ``ratings.dat``."""
from __future__ import annotations

import os
import zipfile

import numpy as np

from . import base

SOURCE_URL = "http://files.grouplens.org/datasets/movielens/"


def read_data_sets(data_dir):
    """int array [N, 4] = (user, item, rating, timestamp) rows of ``ml-1m/ratings.dat``."""
    extracted = os.path.join(data_dir, "ml-1m")
    ratings = os.path.join(extracted, "ratings.dat")
    if not os.path.exists(ratings):
        local = base.maybe_download("ml-1m.zip", data_dir, SOURCE_URL + "ml-1m.zip")
        with zipfile.ZipFile(local) as z:
            z.extractall(data_dir)
    with open(ratings) as f:
        rows = [line.strip().split("::") for line in f if line.strip()]
    return np.array(rows).astype(int)


def get_id_pairs(data_dir):
    return read_data_sets(data_dir)[:, 0:2]


def get_id_ratings(data_dir):
    return read_data_sets(data_dir)[:, 0:3]
