"""``DL/utils/Util.scala`` helpers: ``kthLargest`` (straggler threshold), ``shift``, weight/bias
extraction and restoration for model cloning / broadcast."""
from __future__ import annotations

import random
from typing import List, Sequence, Tuple

import torch


def kthLargest(arr: List[int], l: int, r: int, k: int) -> int:
    """k-th largest of ``arr[l..r]`` (inclusive, 1-based k) by randomised quickselect; reorders
    ``arr`` in place like the reference."""
    if k <= 0 or k > r - l + 1:
        raise ValueError(f"k={k} outside [1, {r - l + 1}]")
    while True:
        piv = random.randint(l, r)
        arr[piv], arr[r] = arr[r], arr[piv]
        x, i = arr[r], l
        for j in range(l, r):
            if arr[j] >= x:
                arr[i], arr[j] = arr[j], arr[i]
                i += 1
        arr[i], arr[r] = arr[r], arr[i]
        pos = i - l + 1
        if pos == k:
            return arr[i]
        if pos > k:
            r = i - 1
        else:
            k -= pos
            l = i + 1


def shift(data: list, frm: int, to: int) -> list:
    """Move element ``frm`` to index ``to`` (shifting the ones between)."""
    v = data.pop(frm)
    data.insert(to, v)
    return data


def getAndClearWeightBias(parameters: Tuple[Sequence[torch.Tensor], Sequence[torch.Tensor]]):
    """Detach the weights (copies) so a model can be shipped without them; ``putWeightBias``
    restores them."""
    weights = [w.detach().clone() for w in parameters[0]]
    for w in parameters[0]:
        w.data = torch.empty(0, dtype=w.dtype, device=w.device)
    return weights


def putWeightBias(weights: Sequence[torch.Tensor], parameters):
    for dst, src in zip(parameters[0], weights):
        dst.data = src.clone()


class Util:
    kthLargest = staticmethod(kthLargest)
    shift = staticmethod(shift)
    getAndClearWeightBias = staticmethod(getAndClearWeightBias)
    putWeightBias = staticmethod(putWeightBias)
