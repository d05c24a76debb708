"""Lua-style heterogeneous container used as the multi-input/multi-output ``Activity``.

Reference behaviour: ``DL/utils/Table.scala:34`` (class ``Table``) and ``object T`` (``:323``).
Keys are usually 1-based integers; arbitrary hashable keys are also allowed.  ``length()``
counts the consecutive integer keys starting at 1, like Lua's ``#`` operator.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Any, Iterator


class Table:
    __slots__ = ("_state",)

    def __init__(self, *args, **kwargs):
        self._state: "OrderedDict[Any, Any]" = OrderedDict()
        for i, v in enumerate(args):
            self._state[i + 1] = v
        for k, v in kwargs.items():
            self._state[k] = v

    # --- Lua-ish access -------------------------------------------------
    def __getitem__(self, key):
        return self._state[key]

    def get(self, key, default=None):
        return self._state.get(key, default)

    def __setitem__(self, key, value):
        self._state[key] = value

    def update(self, key, value):
        self._state[key] = value
        return self

    def insert(self, *args):
        """``insert(value)`` appends; ``insert(index, value)`` shifts (1-based), as Table.scala."""
        if len(args) == 1:
            self._state[self.length() + 1] = args[0]
        else:
            index, value = args
            n = self.length()
            for i in range(n, index - 1, -1):
                self._state[i + 1] = self._state[i]
            self._state[index] = value
        return self

    def remove(self, index=None):
        n = self.length()
        if index is None:
            index = n
        if n == 0 or index not in self._state:
            return None
        v = self._state.pop(index)
        for i in range(index + 1, n + 1):
            self._state[i - 1] = self._state.pop(i)
        return v

    def contains(self, key) -> bool:
        return key in self._state

    __contains__ = contains

    def delete(self, key):
        self._state.pop(key, None)
        return self

    def clear(self):
        self._state.clear()
        return self

    def length(self) -> int:
        n = 0
        while (n + 1) in self._state:
            n += 1
        return n

    def __len__(self) -> int:
        return self.length()

    def keys(self):
        return list(self._state.keys())

    def values(self):
        return list(self._state.values())

    def items(self):
        return list(self._state.items())

    def __contains__(self, key) -> bool:
        return key in self._state

    def __iter__(self) -> Iterator:
        for i in range(1, self.length() + 1):
            yield self._state[i]

    def to_list(self) -> list:
        return [self._state[i] for i in range(1, self.length() + 1)]

    def flatten(self) -> "Table":
        out = Table()
        def rec(t):
            for v in t:
                if isinstance(v, Table):
                    rec(v)
                else:
                    out.insert(v)
        rec(self)
        return out

    def clone(self) -> "Table":
        t = Table()
        for k, v in self._state.items():
            if hasattr(v, "clone"):
                v = v.clone()
            t[k] = v
        return t

    def __eq__(self, other):
        if not isinstance(other, Table):
            return False
        if set(self._state.keys()) != set(other._state.keys()):
            return False
        import torch
        for k, v in self._state.items():
            o = other._state[k]
            if isinstance(v, torch.Tensor):
                if not (isinstance(o, torch.Tensor) and v.shape == o.shape and torch.equal(v.cpu(), o.cpu())):
                    return False
            elif v != o:
                return False
        return True

    def __repr__(self):
        body = ", ".join(f"{k}: {type(v).__name__ if hasattr(v, 'shape') else v!r}" for k, v in self._state.items())
        return "T(" + body + ")"


def T(*args, **kwargs) -> Table:
    """``T(a, b, c)`` → Table{1: a, 2: b, 3: c} (``object T``, Table.scala:323)."""
    return Table(*args, **kwargs)


def to_table(x) -> Table:
    if isinstance(x, Table):
        return x
    if isinstance(x, (list, tuple)):
        return Table(*x)
    return Table(x)
