"""Single/multi shape used by Keras-style shape inference (``DL/utils/Shape.scala``)."""
from __future__ import annotations


class Shape:
    @staticmethod
    def of(*args):
        if len(args) == 1 and isinstance(args[0], (list, tuple)) and args[0] and isinstance(args[0][0], Shape):
            return MultiShape(list(args[0]))
        if len(args) == 1 and isinstance(args[0], (list, tuple)):
            return SingleShape(list(args[0]))
        if args and all(isinstance(a, Shape) for a in args):
            return MultiShape(list(args))
        return SingleShape(list(args))


class SingleShape(Shape):
    def __init__(self, value):
        self.value = [int(v) if v is not None else -1 for v in value]

    def toSingle(self):
        return list(self.value)

    def toMulti(self):
        raise ValueError("SingleShape cannot be converted to MultiShape")

    def copyAndUpdate(self, dim, v):
        val = list(self.value)
        val[dim if dim >= 0 else len(val) + dim] = v
        return SingleShape(val)

    def __eq__(self, o):
        return isinstance(o, SingleShape) and o.value == self.value

    def __repr__(self):
        return f"SingleShape({self.value})"


class MultiShape(Shape):
    def __init__(self, value):
        self.value = list(value)

    def toSingle(self):
        raise ValueError("MultiShape cannot be converted to SingleShape")

    def toMulti(self):
        return list(self.value)

    def __eq__(self, o):
        return isinstance(o, MultiShape) and o.value == self.value

    def __repr__(self):
        return f"MultiShape({self.value})"
