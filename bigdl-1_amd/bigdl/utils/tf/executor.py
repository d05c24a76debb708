"""Host-side executor for a TensorFlow graph's INPUT PIPELINE: queues, readers and the parsing /
decoding ops between them (the part of ``DL/utils/tf/Session.scala`` that turns a graph's queue
runners into a data set — ``getRDD`` / ``BigDLSessionImpl.constructLocalData``).

TF semantics reproduced:

* ``FIFOQueueV2`` / ``RandomShuffleQueueV2`` / ``PaddingFIFOQueueV2`` with ``QueueEnqueue(Many)V2``
  producers and ``QueueDequeue(Many|UpTo)V2`` consumers.  A dequeue from an empty queue runs the
  queue's enqueue ops (round robin) until an element arrives; a producer whose inputs are exhausted
  (an upstream queue is empty and can no longer be filled) is retired, and when every producer is
  retired the dequeue raises :class:`OutOfRange` — the end of the data set.  A producer whose
  inputs come only from constants (``string_input_producer``'s file-name list) runs once.
* ``TFRecordReaderV2`` + ``ReaderReadV2``: a reader takes the next file name from its file-name
  queue when its current file is exhausted and returns ``(key, record)``.
* ``Switch`` / ``Merge`` dead-branch propagation (``tf.cond`` inside ``decode_image``): an op with a
  dead data or control input is dead, except ``Merge``, which forwards its live input.
* String tensors are numpy ``object`` arrays of ``bytes``; numeric tensors are torch tensors, and
  every numeric op is the loader's own op module (``loader._OPS``).
"""
from __future__ import annotations

import collections
import random
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ..table import Table
from .loader import _OPS, _attr, _split_ref
from .proto import tensor_to_torch, torch_dtype


class OutOfRange(Exception):
    """The input pipeline has no more data (TF's OutOfRangeError)."""


class _Dead:
    def __repr__(self):
        return "<dead>"


DEAD = _Dead()
_QUEUE_OPS = {"FIFOQueueV2", "FIFOQueue", "RandomShuffleQueueV2", "RandomShuffleQueue", "PaddingFIFOQueueV2"}
_ENQUEUE_OPS = {"QueueEnqueueV2", "QueueEnqueue", "QueueEnqueueManyV2", "QueueEnqueueMany"}
_READERS = {"TFRecordReaderV2", "TFRecordReader"}
_NO_VALUE = {"NoOp", "Assert", "QueueCloseV2", "QueueClose", "ScalarSummary", "HistogramSummary", "MergeSummary"}


def _is_str(v):
    return isinstance(v, np.ndarray) and v.dtype == object


def _as_str_array(v):
    if _is_str(v):
        return v
    if isinstance(v, (bytes, str)):
        return np.array(v if isinstance(v, bytes) else v.encode(), dtype=object)
    if isinstance(v, (list, tuple)):
        a = np.empty(len(v), dtype=object)
        a[:] = [x if isinstance(x, bytes) else str(x).encode() for x in v]
        return a
    raise TypeError(f"not a string tensor: {type(v)}")


class _Queue:
    def __init__(self, node, rng):
        self.node = node
        self.items = collections.deque()
        self.shuffle = node.op.startswith("RandomShuffle")
        self.rng = rng
        self.producers: List = []
        self.retired = set()

    def pop(self):
        if self.shuffle and len(self.items) > 1:
            i = self.rng.randrange(len(self.items))
            self.items.rotate(-i)
            v = self.items.popleft()
            self.items.rotate(i)
            return v
        return self.items.popleft()


class _Reader:
    def __init__(self):
        self.it = None
        self.name = b""
        self.n = 0


class GraphExecutor:
    def __init__(self, nodes, byte_order: str = "little", seed: int = 0,
                 variables: Optional[Dict[str, torch.Tensor]] = None):
        self.nodes = {n.name: n for n in nodes}
        self.byte_order = byte_order
        #: live variable values (VariableV2 / VarHandleOp reads return these tensors)
        self.variables: Dict[str, torch.Tensor] = variables if variables is not None else {}
        #: records mode: a DequeueMany also returns the final partial batch (every record is used,
        #: like the reference's per-record RDD)
        self.partial_batches = False
        self.rng = random.Random(seed)
        self.queues: Dict[str, _Queue] = {}
        self.readers: Dict[str, _Reader] = {}
        self._mods: Dict[str, object] = {}
        for n in nodes:
            if n.op in _QUEUE_OPS:
                self.queues[n.name] = _Queue(n, self.rng)
        for n in nodes:
            if n.op in _ENQUEUE_OPS:
                q = _split_ref(n.input[0])[0]
                if q in self.queues:
                    self.queues[q].producers.append(n)

    # ------------------------------------------------------------------ public
    def run(self, refs: Sequence[str], feeds: Optional[Dict[str, object]] = None):
        """One step: the values of ``refs`` (raises OutOfRange at the end of the data).  ``feeds``
        maps a node name to its output value (a tuple for multi-output nodes), e.g. a dequeue."""
        memo: Dict[str, object] = dict(feeds or {})
        return [self._eval(r, memo) for r in refs]

    def initialize_variables(self):
        """Run the ``Assign(variable, initial_value)`` initializers of variables without a value."""
        for n in self.nodes.values():
            if n.op in ("Assign", "AssignVariableOp") and len(n.input) >= 2:
                var = _split_ref(n.input[0])[0]
                if var in self.variables or self.nodes[var].op not in ("VariableV2", "Variable", "VarHandleOp"):
                    continue
                v = self.run([n.input[1]])[0]
                self.variables[var] = torch.as_tensor(v).clone()
        return self.variables

    def records(self, endpoint: str, limit: Optional[int] = None) -> List[Table]:
        """Run the pipeline until exhaustion: every dequeued element of ``endpoint`` (a dequeue node),
        batches split into single records, as Tables of its components."""
        out: List[Table] = []
        self.partial_batches = True
        node = self.nodes[_split_ref(endpoint)[0]]
        n_comp = len(_attr(node, "component_types", []) or []) or 1
        while limit is None or len(out) < limit:
            try:
                vals = self.run([f"{node.name}:{i}" for i in range(n_comp)])
            except OutOfRange:
                break
            many = (node.op.startswith("QueueDequeueMany") or node.op.startswith("QueueDequeueUpTo")
                    or self._batched(node))
            if many:
                b = len(vals[0])
                for i in range(b):
                    out.append(Table(*[v[i] for v in vals]))
            else:
                out.append(Table(*vals))
        return out

    # ------------------------------------------------------------------ evaluation
    def _eval(self, ref: str, memo):
        ctrl = ref.startswith("^")
        name, idx = _split_ref(ref.lstrip("^"))
        if name not in memo:
            memo[name] = self._run_node(self.nodes[name], memo)
        outs = memo[name]
        if ctrl:
            return DEAD if outs is DEAD else None
        if outs is DEAD:
            return DEAD
        if isinstance(outs, tuple):
            return outs[idx]
        return outs if idx == 0 else DEAD

    def _run_node(self, node, memo):
        op = node.op
        if op == "Merge" or op == "RefMerge":
            for i, r in enumerate(node.input):
                if r.startswith("^"):
                    continue
                v = self._eval(r, memo)
                if v is not DEAD:
                    return (v, torch.tensor(i, dtype=torch.int32))
            return DEAD
        data = [r for r in node.input if not r.startswith("^")]
        for r in node.input:
            if r.startswith("^") and self._eval(r, memo) is DEAD:
                return DEAD
        if op in _QUEUE_OPS or op in _READERS:
            return node.name  # resource handle
        if op in ("QueueDequeueV2", "QueueDequeue"):
            q = self.queues[_split_ref(data[0])[0]]
            return tuple(self._dequeue(q))
        if op in ("QueueDequeueManyV2", "QueueDequeueMany", "QueueDequeueUpToV2", "QueueDequeueUpTo"):
            q = self.queues[_split_ref(data[0])[0]]
            n = int(self._eval(data[1], memo))
            items = []
            try:
                for _ in range(n):
                    items.append(self._dequeue(q))
            except OutOfRange:
                if not items or not (op.startswith("QueueDequeueUpTo") or self.partial_batches):
                    raise
            return tuple(self._stack([it[c] for it in items]) for c in range(len(items[0])))
        if op in ("QueueSizeV2", "QueueSize"):
            return torch.tensor(len(self.queues[_split_ref(data[0])[0]].items), dtype=torch.int32)
        if op in ("ReaderReadV2", "ReaderRead"):
            return self._read(_split_ref(data[0])[0], self.queues[_split_ref(data[1])[0]])
        vals = [self._eval(r, memo) for r in data]
        if any(v is DEAD for v in vals):
            return DEAD
        if op in ("Switch", "RefSwitch"):
            pred = bool(torch.as_tensor(vals[1]).reshape(-1)[0])
            return (DEAD, vals[0]) if pred else (vals[0], DEAD)
        if op in _NO_VALUE:
            if op == "Assert" and not bool(torch.as_tensor(vals[0]).all()):
                raise ValueError(f"TF Assert {node.name} failed")
            return None
        if op == "Const":
            tp = node.attr["value"].tensor
            v = tensor_to_torch(tp, self.byte_order)
            if tp.dtype % 100 == 7:
                shape = [d.size for d in tp.tensor_shape.dim]
                a = _as_str_array(v if isinstance(v, list) else [v])
                return a.reshape(shape) if shape else np.array(a.reshape(-1)[0] if a.size else b"", dtype=object)
            return v
        handler = getattr(self, "_op_" + op, None)
        if handler is not None:
            return handler(node, vals)
        if any(_is_str(v) for v in vals):
            return self._string_op(node, vals)
        if op not in _OPS:
            raise NotImplementedError(f"input pipeline: unsupported TF op {op} ({node.name})")
        m = self._mods.get(node.name)
        if m is None:
            m = self._mods[node.name] = _OPS[op](node)
        out = m.forward(vals[0] if len(vals) == 1 else Table(*vals))
        return tuple(out.values()) if isinstance(out, Table) else out

    # ------------------------------------------------------------------ queues / readers
    def _dequeue(self, q: _Queue):
        while not q.items:
            if not self._produce(q):
                raise OutOfRange(q.node.name)
        return q.pop()

    def _produce(self, q: _Queue) -> bool:
        for p in q.producers:
            if p.name in q.retired:
                continue
            try:
                memo: Dict[str, object] = {}
                comps = [self._eval(r, memo) for r in p.input[1:] if not r.startswith("^")]
            except OutOfRange:
                q.retired.add(p.name)
                continue
            if any(c is DEAD for c in comps):
                continue
            if p.op.startswith("QueueEnqueueMany"):
                n = len(comps[0])
                for i in range(n):
                    q.items.append(tuple(c[i] for c in comps))
            else:
                q.items.append(tuple(comps))
            if not self._depends_on_state(p):
                q.retired.add(p.name)  # a constant producer (file-name list) runs once
            return True
        return False

    def _batched(self, dequeue_node) -> bool:
        """True when the elements of the dequeued queue are batches (a producer's inputs come from a
        DequeueMany/UpTo): records are then split along dim 0, like the reference's RDD of samples."""
        q = self.queues.get(_split_ref(dequeue_node.input[0])[0])
        if q is None:
            return False
        todo = [r for p in q.producers for r in p.input[1:]]
        seen = set()
        while todo:
            n = _split_ref(todo.pop().lstrip("^"))[0]
            if n in seen:
                continue
            seen.add(n)
            src = self.nodes[n]
            if src.op.startswith("QueueDequeueMany") or src.op.startswith("QueueDequeueUpTo"):
                return True
            if src.op.startswith("QueueDequeue"):
                continue
            todo.extend(src.input)
        return False

    def _depends_on_state(self, node, seen=None) -> bool:
        seen = set() if seen is None else seen
        for r in node.input:
            n = _split_ref(r.lstrip("^"))[0]
            if n in seen:
                continue
            seen.add(n)
            src = self.nodes[n]
            if src.op.startswith("QueueDequeue") or src.op.startswith("ReaderRead") or src.op in (
                    "RandomUniform", "RandomShuffle"):
                if src.op != "RandomShuffle":
                    return True
            if self._depends_on_state(src, seen):
                return True
        return False

    def _read(self, reader_name, fqueue: _Queue):
        from .tfrecord import TFRecordIterator
        rd = self.readers.setdefault(reader_name, _Reader())
        while True:
            if rd.it is not None:
                try:
                    rec = next(rd.it)
                    rd.n += 1
                    key = np.array(rd.name + b":" + str(rd.n - 1).encode(), dtype=object)
                    return (key, np.array(rec, dtype=object))
                except StopIteration:
                    rd.it = None
            fname = self._dequeue(fqueue)[0]
            fname = fname.item() if isinstance(fname, np.ndarray) else fname
            rd.name = fname if isinstance(fname, bytes) else str(fname).encode()
            rd.it = iter(TFRecordIterator(rd.name.decode()))
            rd.n = 0

    @staticmethod
    def _stack(vs):
        if _is_str(vs[0]):
            return np.stack(vs)
        return torch.stack([torch.as_tensor(v) for v in vs])

    # ------------------------------------------------------------------ string-aware ops
    def _string_op(self, node, vals):
        op = node.op
        a = _as_str_array(vals[0])
        if op in ("Identity", "Snapshot", "StopGradient"):
            return a
        if op == "Reshape":
            return a.reshape([int(v) for v in torch.as_tensor(vals[1]).flatten().tolist()])
        if op == "Squeeze":
            dims = _attr(node, "squeeze_dims", []) or []
            return np.squeeze(a, axis=tuple(d % a.ndim for d in dims)) if dims else np.squeeze(a)
        if op == "ExpandDims":
            return np.expand_dims(a, int(torch.as_tensor(vals[1]).reshape(-1)[0]) % (a.ndim + 1))
        if op in ("Equal", "NotEqual"):
            b = _as_str_array(vals[1])
            eq = np.vectorize(lambda x, y: x == y, otypes=[bool])(a, b)
            return torch.from_numpy(eq if op == "Equal" else ~eq)
        if op == "Pack":
            return np.stack([_as_str_array(v) for v in vals], int(_attr(node, "axis", 0)))
        raise NotImplementedError(f"input pipeline: string op {op} ({node.name})")

    def _op_VariableV2(self, node, vals):
        if node.name not in self.variables:
            raise KeyError(f"variable {node.name} has no value (load a checkpoint or initialize_variables())")
        return self.variables[node.name]

    _op_Variable = _op_VarHandleOp = _op_VariableV2

    def _op_ReadVariableOp(self, node, vals):
        return vals[0] if not isinstance(vals[0], str) else self.variables[vals[0]]

    def _op_Assign(self, node, vals):
        self.variables[_split_ref(node.input[0])[0]] = torch.as_tensor(vals[1])
        return vals[1]

    def _op_ZerosLike(self, node, vals):
        return torch.zeros_like(torch.as_tensor(vals[0]))

    def _op_OnesLike(self, node, vals):
        return torch.ones_like(torch.as_tensor(vals[0]))

    def _op_Rank(self, node, vals):
        v = vals[0]
        return torch.tensor(v.ndim if _is_str(v) else torch.as_tensor(v).dim(), dtype=torch.int32)

    def _op_Shape(self, node, vals):
        v = vals[0]
        return torch.tensor(list(v.shape), dtype=torch.int32)

    def _op_Size(self, node, vals):
        v = vals[0]
        return torch.tensor(int(np.prod(v.shape)), dtype=torch.int32)

    def _op_RandomShuffle(self, node, vals):
        v = vals[0]
        if _is_str(v):
            idx = list(range(len(v)))
            self.rng.shuffle(idx)
            return v[idx]
        return v[torch.randperm(v.shape[0])]

    def _op_Substr(self, node, vals):
        a = _as_str_array(vals[0])
        pos = int(torch.as_tensor(vals[1]).reshape(-1)[0])
        ln = int(torch.as_tensor(vals[2]).reshape(-1)[0])
        return np.vectorize(lambda s: s[pos:pos + ln], otypes=[object])(a)

    def _op_DecodeRaw(self, node, vals):
        a = _as_str_array(vals[0])
        dt = torch_dtype(_attr(node, "out_type", 4))
        np_t = {torch.uint8: np.uint8, torch.int8: np.int8, torch.int16: np.int16, torch.int32: np.int32,
                torch.int64: np.int64, torch.float32: np.float32, torch.float64: np.float64}[dt]
        order = "<" if bool(_attr(node, "little_endian", True)) else ">"
        rows = [np.frombuffer(s, dtype=np.dtype(np_t).newbyteorder(order)).astype(np_t) for s in a.reshape(-1)]
        arr = np.stack(rows).reshape(a.shape + rows[0].shape) if a.ndim else rows[0]
        return torch.from_numpy(np.ascontiguousarray(arr))

    def _decode_image(self, node, vals):
        from ...nn.tf import DecodeImage
        a = _as_str_array(vals[0])
        return DecodeImage(int(_attr(node, "channels", 3) or 3)).forward(a.item() if a.ndim == 0 else a.reshape(-1)[0])

    _op_DecodeJpeg = _op_DecodePng = _op_DecodeGif = _op_DecodeBmp = _decode_image

    def _op_ParseExample(self, node, vals):
        """(serialized [B], names, sparse_keys × Ns, dense_keys × Nd, dense_defaults × Nd) →
        sparse indices × Ns, values × Ns, shapes × Ns, dense × Nd (dense [B, *shape])."""
        from .proto import example_classes
        Example = example_classes()["tensorflow.Example"]
        ns = int(_attr(node, "Nsparse", 0) or 0)
        nd = int(_attr(node, "Ndense", 0) or 0)
        ser = _as_str_array(vals[0]).reshape(-1)
        skeys = [_as_str_array(v).item().decode() for v in vals[2:2 + ns]]
        dkeys = [_as_str_array(v).item().decode() for v in vals[2 + ns:2 + ns + nd]]
        defaults = vals[2 + ns + nd:2 + ns + 2 * nd]
        tdense = [torch_dtype(t) for t in (_attr(node, "Tdense", []) or [])]
        shapes = [[int(d.size) for d in sh.dim] for sh in (_attr(node, "dense_shapes", []) or [])]
        exs = [Example.FromString(s) for s in ser]

        def feat(ex, k):
            if k not in ex.features.feature:
                return None, None
            f = ex.features.feature[k]
            kind = f.WhichOneof("kind")
            return kind, (list(getattr(f, kind).value) if kind else [])
        s_idx, s_val, s_shp = [], [], []
        for k in skeys:
            rows, vs = [], []
            for b, ex in enumerate(exs):
                kind, v = feat(ex, k)
                for j, x in enumerate(v or []):
                    rows.append([b, j])
                    vs.append(x)
            s_idx.append(torch.tensor(rows, dtype=torch.int64).reshape(-1, 2))
            s_val.append(_as_str_array(vs) if vs and isinstance(vs[0], bytes) else torch.tensor(vs))
            s_shp.append(torch.tensor([len(exs), max([len(feat(e, k)[1] or []) for e in exs] or [0])]))
        dense = []
        for j, k in enumerate(dkeys):
            col = []
            for ex in exs:
                kind, v = feat(ex, k)
                if kind is None:
                    d = defaults[j]
                    col.append(d if _is_str(d) else torch.as_tensor(d))
                elif kind == "bytes_list":
                    col.append(_as_str_array(v).reshape(shapes[j] if j < len(shapes) and shapes[j] else [-1]))
                else:
                    t = torch.tensor(v, dtype=tdense[j] if j < len(tdense) else None)
                    col.append(t.reshape(shapes[j]) if j < len(shapes) and shapes[j] else t)
            dense.append(np.stack(col) if _is_str(col[0]) else torch.stack(col))
        return tuple(s_idx + s_val + s_shp + dense)

    def _op_ParseSingleExample(self, node, vals):
        from .loader import _parse_single
        out = _parse_single(node).forward(Table(*[v.item() if _is_str(v) and v.ndim == 0 else v for v in vals]))
        return tuple(_as_str_array(v) if isinstance(v, list) else v for v in out.values())


__all__ = ["GraphExecutor", "OutOfRange"]
