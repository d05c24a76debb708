"""HIP-graph capture of a whole training iteration (forward, criterion, backward, fused optimizer
update) for launch-bound models — the MI355X replacement of per-op host dispatch.

A step of a small model (VGG-CIFAR, PTB LSTM) issues hundreds of short kernels whose host-side
launch cost exceeds their GPU time; captured once into a hipGraph the same step is one graph
launch.  Requirements, checked at capture time:

* static shapes (the batch is copied into the graph's static input buffers);
* no host synchronisation inside the step (a sync raises during capture → eager fallback);
* per-iteration scalars must not be baked in: dropout draws its Philox seed from a device counter
  advanced inside the graph, Adagrad and Adam keep their iteration counters on the device (Adam's
  fused kernel forms the decayed rate and bias corrections from it), SGD is captured
  only with a constant learning rate (``OptimMethod.prepare_graph``).

Only :class:`~bigdl.optim.optimizer.LocalOptimizer` steps are captured (the DistriOptimizer's RCCL
buckets are issued from backward hooks and stay eager).
"""
from __future__ import annotations

import torch

from ..dataset import MiniBatch
from ..utils.logger import get_logger

log = get_logger("bigdl.optim")


class GraphedTrainStep:
    """Capture ``optimizer.train_step`` into one HIP graph.

    Capture needs ``warmup`` eager steps first (allocator pools, lazily built state).  Those steps
    are NOT part of training: every tensor they change — master weights, the bf16 shadow, BN
    running statistics, optimizer state — is snapshotted before and restored IN PLACE after the
    capture (the graph keeps pointing at the same storage), host counters (``evalCounter``) are
    restored and device counters (``_dev_n``) re-synchronised, so the first :meth:`step` is the
    trajectory's first iteration.  Optimizer state that the warmup created is zeroed; SGD's
    first-iteration momentum rule (v = g) is raised through a device flag its captured kernel reads
    and clears (``_dev_first``)."""

    def __init__(self, optimizer, batch: MiniBatch, warmup: int = 3):
        if not torch.cuda.is_available():
            raise RuntimeError("HIP graph capture needs a GPU")
        for name, meth in optimizer.optim_methods.items():
            if not meth.prepare_graph():
                raise NotImplementedError(f"OptimMethod {name} ({type(meth).__name__}) is not replay-safe")
        self.opt = optimizer
        from ..ops import native_ops
        native_ops._device_seed(torch.device("cuda", torch.cuda.current_device()))  # no H2D copy while capturing
        x, y = batch.getInput(), batch.getTarget()
        self.sx = x.clone(memory_format=torch.preserve_format)
        self.sy = y.clone() if isinstance(y, torch.Tensor) else y
        b = MiniBatch(self.sx, self.sy)
        snap = self._snapshot()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                optimizer.train_step(b)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.loss = optimizer.train_step(b)
        torch.cuda.synchronize()
        self._restore(snap)
        torch.cuda.synchronize()

    # -------------------------------------------------------------------------- warmup undo
    def _tensors(self):
        opt = self.opt
        flat = getattr(opt, "flat", None)
        ts = []
        if flat is not None:
            ts += [t for t in (flat.weight, flat.shadow) if t is not None]
        ts += list(opt.model.getExtraParameter() or [])
        return ts

    def _snapshot(self):
        ts = [(t, t.detach().clone()) for t in self._tensors()]
        states = {}
        for name, meth in self.opt.optim_methods.items():
            states[name] = {k: (v.detach().clone() if isinstance(v, torch.Tensor) else v)
                            for k, v in meth.state.items()}
        return ts, states

    def _restore(self, snap):
        ts, states = snap
        for t, c in ts:
            t.copy_(c)
        flat = getattr(self.opt, "flat", None)
        if flat is not None and hasattr(flat, "shadow_gen"):
            flat.shadow_gen += 1  # the shadow changed under the weight-derived caches
        for name, meth in self.opt.optim_methods.items():
            pre = states[name]
            fresh = []
            for k in list(meth.state.keys()):
                v = meth.state[k]
                if k in pre:
                    if isinstance(v, torch.Tensor) and isinstance(pre[k], torch.Tensor) and v.shape == pre[k].shape:
                        v.copy_(pre[k])
                    else:
                        meth.state[k] = pre[k]
                elif isinstance(v, torch.Tensor):
                    v.zero_()  # created by the warmup: back to its initial (zero) value
                    fresh.append(k)
                else:
                    del meth.state[k]
            meth.sync_device_counter()
            meth.graph_state_restored(fresh)

    def step(self, batch: MiniBatch = None) -> torch.Tensor:
        if batch is not None:
            x, y = batch.getInput(), batch.getTarget()
            if x is not self.sx:
                self.sx.copy_(x, non_blocking=True)
            if isinstance(y, torch.Tensor) and y is not self.sy:
                self.sy.copy_(y, non_blocking=True)
        self.opt.state["neval"] = self.opt.state.get("neval", 0) + 1
        self.graph.replay()
        for meth in self.opt.optim_methods.values():
            meth.after_graph_replay()
        return self.loss


def graphed_train_step(optimizer, batch: MiniBatch):
    """``optimizer.train_step(batch)`` through a lazily captured graph; falls back to eager (once,
    with a log line) when the step cannot be captured."""
    g = getattr(optimizer, "_graphed", None)
    if g is None and not getattr(optimizer, "_graph_failed", False):
        try:
            g = GraphedTrainStep(optimizer, batch)
            optimizer._graphed = g
            log.info("training step captured into a HIP graph")
        except Exception as e:  # noqa: BLE001 - capture is an optimisation; eager stays correct
            optimizer._graph_failed = True
            log.warning(f"HIP graph capture failed, running eagerly: {e!r}")
            torch.cuda.synchronize()
    if g is not None:
        return g.step(batch)
    return optimizer.train_step(batch)
