"""TensorFlow-graph training session (``DL/utils/tf/Session.scala:43-180``, ``BigDLSessionImpl``).

A :class:`Session` holds a GraphDef plus a variable context (name → tensor, typically read from a
TF checkpoint by :func:`bigdl.utils.tf.checkpoint.read_checkpoint`):

* ``train(outputs, dataset, optim_method, criterion, end_when)`` — builds the BigDL graph from the
  Placeholder input(s) to ``outputs`` with the variables as trainable Linear / SpatialConvolution
  weights, trains it with the optimizer for this process layout (LocalOptimizer, or the RCCL
  DistriOptimizer under the launcher) and writes the trained weights back into the context;
* ``predict(outputs, data, batch_size)`` — forward of the same graph over in-memory data;
* ``saveParameters(path)`` — writes the context as a TF V2 checkpoint (``path.index`` +
  ``path.data-00000-of-00001``) — the reference dumps a Java-serialised map instead.

Queue-fed graphs (``Session.scala:132-176,536-680``): ``get_records(endpoints)`` (the reference's
``getRDD``) runs the graph's own input pipeline — file-name queue, TFRecord readers, shuffle / batch
queues, parsing and decoding ops — with :class:`~bigdl.utils.tf.executor.GraphExecutor` until the
data is exhausted and returns one Table per record (batches split along dim 0, the reference's
``splitTensorByFirstDim``); ``train_graph(end_points, optim_method, end_when, batch_size)`` trains a
TF TRAINING graph: the updater nodes under ``end_points`` (``ApplyRMSProp``, ``ApplyGradientDescent``,
…) name each variable and the graph tensor holding its gradient (TF's own backward ops —
``Conv2DBackpropFilter``, ``ReluGrad``, ``MaxPoolGrad``, …), every iteration evaluates the loss and
those gradients on a batch from the input pipeline and the BigDL OptimMethod updates the variables
(one flat parameter vector, like the reference's ``FakeCriterion`` + assigned gradients).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import torch

from .loader import TensorflowLoader, _Builder, _split_ref


class Session:
    def __init__(self, graph, context: Optional[Dict[str, torch.Tensor]] = None, byte_order: str = "little"):
        nodes = TensorflowLoader.parse(graph) if isinstance(graph, str) else list(graph)
        self.nodes = nodes
        self.context: Dict[str, torch.Tensor] = dict(context or {})
        self.byte_order = byte_order

    # ------------------------------------------------------------------ helpers
    def _placeholders(self, outputs: Sequence[str]) -> List[str]:
        by = {n.name: n for n in self.nodes}
        seen, todo, found = set(), [_split_ref(o)[0] for o in outputs], []
        while todo:
            n = todo.pop()
            if n in seen or n not in by:
                continue
            seen.add(n)
            node = by[n]
            if node.op in ("Placeholder", "PlaceholderWithDefault"):
                found.append(n)
                continue
            todo.extend(_split_ref(i.lstrip("^"))[0] for i in node.input)
        # graph order, as the reference's topological input order
        order = [n.name for n in self.nodes]
        return sorted(found, key=order.index)

    def _build(self, outputs, inputs=None):
        inputs = list(inputs) if inputs else self._placeholders(outputs)
        if not inputs:
            raise ValueError("no Placeholder feeds the requested outputs")
        b = _Builder(self.nodes, self.byte_order, self.context)
        model = b.build(inputs, list(outputs))
        return model, b

    def _write_back(self, builder):
        for var, module, attr, to_tf in builder.var_bindings:
            t = getattr(module, attr)
            self.context[var] = to_tf(t.detach().float().cpu()).contiguous().to(self.context[var].dtype)

    # ------------------------------------------------------------------ API
    def train(self, outputs: Sequence[str], dataset, optim_method, criterion, end_when, batch_size: int = 32,
              inputs: Optional[Sequence[str]] = None):
        from ...optim.optimizer import Optimizer
        model, builder = self._build(outputs, inputs)
        opt = Optimizer.create(model, dataset, criterion, end_when, batch_size, optim_method)
        opt.optimize()
        self._write_back(builder)
        return model

    def predict(self, outputs: Sequence[str], data, batch_size: int = 32, inputs: Optional[Sequence[str]] = None):
        model, _ = self._build(outputs, inputs)
        model.evaluate()
        xs = data if isinstance(data, torch.Tensor) else torch.as_tensor(data)
        outs = []
        with torch.no_grad():
            for i in range(0, xs.shape[0], batch_size):
                outs.append(model.forward(xs[i:i + batch_size]))
        return torch.cat(outs) if outs and isinstance(outs[0], torch.Tensor) else outs

    # ------------------------------------------------------------------ queue-fed graphs
    def _executor(self, seed: int = 0):
        from .executor import GraphExecutor
        return GraphExecutor(self.nodes, self.byte_order, seed, variables=self.context)

    def get_records(self, end_points: Sequence[str], has_to_batch: bool = True, seed: int = 0,
                    batch_size: Optional[int] = None):
        """``getRDD`` (BigDLSessionImpl.getRDD): one Table per record.

        * ``end_points[0]`` a dequeue node: the records its input pipeline produces.
        * otherwise (e.g. a feature layer and the label node of a transfer-learning graph): the
          records of the data dequeue feeding them are run through the graph ``batch_size`` at a
          time (default: the dequeue's own batch; a graph with a baked-in batch is filled by
          cycling records) and the end points' values are split back into per-record Tables."""
        from ..table import T
        ex = self._executor(seed)
        by = {n.name: n for n in self.nodes}
        first = by.get(_split_ref(end_points[0])[0])
        if first is not None and first.op.startswith("QueueDequeue") and len(end_points) == 1:
            return ex.records(end_points[0])
        ex.initialize_variables()  # variables without a checkpoint value take their initializers
        deq = self._data_dequeue(list(end_points))
        records = ex.records(deq.name)
        if not records:
            return []
        bs = batch_size or len(records)
        out = []
        for s in range(0, len(records), bs):
            real = records[s:s + bs]
            batch = [records[(s + j) % len(records)] for j in range(bs)]
            comps = tuple(torch.stack([torch.as_tensor(r[c + 1]) for r in batch]) for c in range(batch[0].length()))
            vals = ex.run(list(end_points), feeds={deq.name: comps})
            for j in range(len(real)):
                out.append(T(*[torch.as_tensor(v)[j] for v in vals]))
        return out

    getRDD = get_records

    _UPDATERS = {"ApplyRMSProp": 7, "ApplyGradientDescent": 2, "ApplyMomentum": 3, "ApplyAdam": 9,
                 "ApplyAdagrad": 3, "ApplyAdadelta": 6, "ApplyFtrl": 3, "ApplyProximalGradientDescent": 4,
                 "ResourceApplyRMSProp": 7, "ResourceApplyGradientDescent": 2, "ResourceApplyMomentum": 3,
                 "ResourceApplyAdam": 9}

    def _updaters(self, end_points):
        by = {n.name: n for n in self.nodes}
        seen, todo, found = set(), [_split_ref(e.lstrip("^"))[0] for e in end_points], []
        while todo:
            n = todo.pop()
            if n in seen or n not in by:
                continue
            seen.add(n)
            node = by[n]
            gi = self._UPDATERS.get(node.op)
            if gi is not None:
                found.append((_split_ref(node.input[0])[0], node.input[gi]))
                continue
            todo.extend(_split_ref(i.lstrip("^"))[0] for i in node.input)
        order = [n.name for n in self.nodes]
        return sorted(set(found), key=lambda t: order.index(t[0]))

    def _data_dequeue(self, refs):
        by = {n.name: n for n in self.nodes}
        seen, todo = set(), [_split_ref(r.lstrip("^"))[0] for r in refs]
        while todo:
            n = todo.pop(0)
            if n in seen or n not in by:
                continue
            seen.add(n)
            node = by[n]
            if node.op.startswith("QueueDequeue"):
                return node
            todo.extend(_split_ref(i.lstrip("^"))[0] for i in node.input if not i.startswith("^"))
        raise ValueError("no queue dequeue feeds the training graph")

    def train_graph(self, end_points: Sequence[str], optim_method, end_when, batch_size: int,
                    loss: Optional[str] = None, seed: int = 0):
        """Train a TF training graph from its own input pipeline and gradient ops (see module doc).
        Returns the per-iteration losses."""
        from ..table import Table
        updaters = self._updaters(end_points)
        if not updaters:
            raise ValueError("Cannot find updater nodes")
        ex = self._executor(seed)
        ex.initialize_variables()
        # one flat fp32 parameter vector; the context tensors become views of it, so the executor
        # reads the updated values every iteration
        names = [v for v, _ in updaters]
        sizes = [self.context[v].numel() for v in names]
        w = torch.cat([self.context[v].detach().float().reshape(-1) for v in names])
        g = torch.zeros_like(w)
        off = 0
        for v, n in zip(names, sizes):
            shape = self.context[v].shape
            self.context[v] = w[off:off + n].view(shape)
            off += n
        loss_ref = loss or end_points[0]
        by = {n.name: n for n in self.nodes}
        # an endpoint like ``train_op = Identity(total_loss, ^update_ops)``: take the loss through its
        # data input — the control inputs are the TF updaters this loop replaces
        while by[_split_ref(loss_ref)[0]].op in ("Identity", "Snapshot"):
            data_in = [i for i in by[_split_ref(loss_ref)[0]].input if not i.startswith("^")]
            if not data_in:
                break
            loss_ref = data_in[0]
        deq = self._data_dequeue([r for _, r in updaters])
        records = ex.records(deq.name)
        if not records:
            raise ValueError(f"the input pipeline of {deq.name} produced no data")
        state = {"epoch": 1, "neval": 1, "Loss": float("nan"), "score": 0.0, "recordsProcessedThisEpoch": 0}
        losses = []
        i = 0
        n_rec = len(records)
        while not end_when(state):
            # the data set is cycled (an epoch ends after n_rec records), so a graph with a baked-in
            # batch dimension larger than the data still trains
            batch = [records[(i + j) % n_rec] for j in range(batch_size)]
            i += batch_size
            if i >= n_rec:
                i %= n_rec
                state["epoch"] += 1
                state["recordsProcessedThisEpoch"] = 0
            comps = tuple(torch.stack([torch.as_tensor(r[c + 1]) for r in batch]) for c in range(batch[0].length()))
            outs = ex.run([loss_ref] + [r for _, r in updaters], feeds={deq.name: comps})
            off = 0
            for t, n in zip(outs[1:], sizes):
                g[off:off + n].copy_(torch.as_tensor(t).float().reshape(-1))
                off += n
            lv = torch.as_tensor(outs[0]).float().reshape(-1)[0]
            optim_method.optimize(lambda _x: (lv, g), w)
            losses.append(float(lv))
            state["Loss"] = float(lv)
            state["neval"] += 1
            state["recordsProcessedThisEpoch"] += batch_size
        return losses

    def saveParameters(self, path: str):
        from .checkpoint import write_checkpoint
        write_checkpoint(path, {k: v.detach().cpu().numpy() for k, v in self.context.items()})
        return self

    save_parameters = saveParameters


BigDLSessionImpl = Session

__all__ = ["Session", "BigDLSessionImpl"]
