"""Seedable random generator (``RNG``).

Reference: ``DL/utils/RandomGenerator.scala:23-272`` — a Torch-compatible Mersenne Twister with
``setSeed``, ``uniform``, ``normal``, ``bernoulli``.  Host-side we use numpy's MT19937 (the same
generator family) for data shuffling and parameter init; device-side randomness (dropout masks)
uses torch's Philox generator seeded from this one, so ``RNG.setSeed`` makes a whole run
reproducible.
"""
from __future__ import annotations

import threading

import numpy as np
import torch


class RandomGenerator:
    def __init__(self, seed: int = 1):
        self._lock = threading.Lock()
        self.setSeed(seed)

    def setSeed(self, seed: int):
        with self._lock:
            self._seed = int(seed)
            self._np = np.random.RandomState(self._seed & 0xFFFFFFFF)
            self._torch = torch.Generator()
            self._torch.manual_seed(self._seed)
            torch.manual_seed(self._seed)
        return self

    set_seed = setSeed

    def getSeed(self) -> int:
        return self._seed

    def uniform(self, a: float = 0.0, b: float = 1.0) -> float:
        with self._lock:
            return float(self._np.uniform(a, b))

    def normal(self, mean: float = 0.0, stdv: float = 1.0) -> float:
        with self._lock:
            return float(self._np.normal(mean, stdv))

    def bernoulli(self, p: float) -> bool:
        return self.uniform() < p

    def random(self) -> int:
        with self._lock:
            return int(self._np.randint(0, 2**31 - 1))

    def shuffle(self, arr):
        with self._lock:
            self._np.shuffle(arr)
        return arr

    def permutation(self, n: int) -> np.ndarray:
        with self._lock:
            return self._np.permutation(n)

    @property
    def torch_generator(self) -> torch.Generator:
        return self._torch

    def uniform_tensor(self, shape, a=0.0, b=1.0, dtype=torch.float32):
        with self._lock:
            t = torch.empty(shape, dtype=torch.float32)
            t.uniform_(a, b, generator=self._torch)
        return t.to(dtype)

    def normal_tensor(self, shape, mean=0.0, std=1.0, dtype=torch.float32):
        with self._lock:
            t = torch.empty(shape, dtype=torch.float32)
            t.normal_(mean, std, generator=self._torch)
        return t.to(dtype)


RNG = RandomGenerator(1)
