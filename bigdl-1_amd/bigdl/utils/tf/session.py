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

The reference's queue/reader-fed variant (``train(endPoints, …)`` pulling from TFRecord reader
nodes on a SparkContext) maps to feeding the same graph from :mod:`bigdl.utils.tf.tfrecord` data
through ``train``'s ``dataset`` argument; in-graph queue runners are not executed.
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

    def saveParameters(self, path: str):
        from .checkpoint import write_checkpoint
        write_checkpoint(path, {k: v.detach().cpu().numpy() for k, v in self.context.items()})
        return self

    save_parameters = saveParameters


BigDLSessionImpl = Session

__all__ = ["Session", "BigDLSessionImpl"]
