"""``bigdl.dataset.transformer`` (``PY/dataset/transformer.py``)."""
from __future__ import annotations


def normalizer(data, mean, std):
    """Normalise features: (data - mean) / std (ndarray in, float ndarray out)."""
    return (data - mean) / std
