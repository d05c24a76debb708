"""Row → Table transformer (``DL/dataset/datamining/RowTransformer.scala``).

A "row" is a mapping (dict / pandas Series / namedtuple via ``_asdict``) or a sequence with a
schema (field names).  ``RowTransformer(schema, transformers)`` produces a ``Table`` keyed by each
transformer's ``schema_key`` with the tensor it builds from its fields."""
from __future__ import annotations

from typing import Callable, Dict, Iterator, List, Optional, Sequence

import torch

from ..utils.table import Table
from .core import Transformer


class ColToTensor:
    def __init__(self, schema_key: str, field_names: Sequence[str], dtype=torch.float32):
        self.schema_key, self.field_names, self.dtype = schema_key, list(field_names), dtype

    def __call__(self, row: Dict) -> torch.Tensor:
        return torch.tensor([float(row[f]) for f in self.field_names], dtype=self.dtype)


class RowTransformer(Transformer):
    def __init__(self, schema: Optional[Sequence[str]], transformers: Sequence[ColToTensor]):
        self.schema = list(schema) if schema is not None else None
        self.transformers = list(transformers)

    def _as_dict(self, row):
        if isinstance(row, dict):
            return row
        if hasattr(row, "to_dict"):
            return row.to_dict()
        if hasattr(row, "_asdict"):
            return row._asdict()
        if self.schema is None:
            raise ValueError("a sequence row needs a schema")
        return dict(zip(self.schema, row))

    def apply(self, it: Iterator) -> Iterator[Table]:
        for row in it:
            d = self._as_dict(row)
            t = Table()
            for tr in self.transformers:
                t[tr.schema_key] = tr(d)
            yield t

    @staticmethod
    def atomic(field_names: Sequence[str], schema: Optional[Sequence[str]] = None) -> "RowTransformer":
        """One table entry per field (key = field name)."""
        return RowTransformer(schema, [ColToTensor(f, [f]) for f in field_names])

    @staticmethod
    def numeric(numeric_fields: Dict[str, Sequence[str]], schema: Optional[Sequence[str]] = None
                ) -> "RowTransformer":
        """One table entry per key, concatenating the listed numeric fields."""
        return RowTransformer(schema, [ColToTensor(k, v) for k, v in numeric_fields.items()])
