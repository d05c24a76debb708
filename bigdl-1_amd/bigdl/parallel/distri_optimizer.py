"""DistriOptimizer: synchronous data-parallel SGD, one process per GPU, RCCL over xGMI.

Reference semantics (``DL/optim/DistriOptimizer.scala:97-517``, ``ParallelOptimizer.scala``):
  job 1 — every replica pulls weights, runs fwd/bwd on its slice of the global batch, pushes its
  gradient split into N chunks (bf16);  job 2 — each partition sums its chunk from all replicas
  (``aggregateGradientPartition``), runs the OptimMethod on ITS 1/N of the parameters (ZeRO-1
  style, one optimizer state per shard) and publishes the updated weight shard.
  ParallelOptimizer additionally pushes each layer group's gradient as soon as its backward is
  done (≈10 buckets, reverse execution order) and applies updates lazily before the next forward.

MI355X mapping (``bigdl.comm.*`` config keys):
  * the flat parameter arena is re-laid out into contiguous buckets of ``bucketMB`` (default 32 MB
    — large enough for RCCL's bandwidth plateau on the 7 xGMI links, few enough to overlap)
    padded to a multiple of 64·world so every bucket is directly a collective buffer;
  * module grad-ready hooks launch ``reduce_scatter_tensor`` for a bucket the moment its last
    parameter gradient is written — these run on RCCL's internal stream concurrently with the rest
    of backward;
  * after backward each bucket's shard is updated by the fused optimizer kernel (``grad_scale=1/N``
    folds the average in) and ``all_gather_into_tensor`` publishes it back into the arena;
  * the next forward waits for a bucket's all-gather only when the first layer owning parameters
    in it runs (pre-forward hook) — the reference's lazy ``updateParameter`` at forward;
  * ``comm.dtype = bf16`` reduces bf16 gradients and gathers the bf16 compute shadow directly
    (half the bytes; fp32 masters live only on the owning rank until :meth:`_flush_weights`);
    ``bf16_truncate`` reproduces the reference's truncating wire format exactly.
  * Non-sliceable methods (LBFGS, Ftrl, …) or several OptimMethods with non-SGD/Adam members fall
    back to "replicated" mode: all-reduce of the full gradient, full update on every rank.

Streams.  Every collective is issued from the comm-side stream (``_side``): it first waits for the
compute stream's work so far and for the side-stream weight-gradient kernels queued so far
(``join_wgrad(side)``), packs the bucket to the wire dtype there (one cast kernel per bucket) and
launches the RCCL op — the compute stream never blocks on a bucket; only the consumer of the
result (the shard update, or the next forward's first use of a bucket) waits.  On the CPU the side
stream is a no-op stand-in (:class:`_HostStream`), so the same early-update code path runs under
gloo in the multi-process tests.  The SGD kernel reads the bf16 reduce-scatter output directly.

Straggler drop (P5, ``DistriOptimizer.scala:240-280,343-345,421-449,510-515``): with
``setDropModuleProperty(dropPercentage, maxDropPercentage, batchsize, warmup)`` each rank times its
forward + backward; every ``batchsize`` iterations after warm-up the ranks all-gather those times and
the threshold becomes ``kthLargest(times, k − dropped)`` with ``k = dropPercentage·batchsize·N``
(or grows 1 % when enough were dropped).  A rank whose compute time exceeds the threshold
contributes a ZERO gradient and a finished-count of 0 to the same collectives; the update divides
by the all-reduced finished count, the loss is averaged over the finished ranks, and when fewer than
``(1 − maxDropPercentage)·N`` ranks finished the iteration's gradients are discarded (no update, the
iteration counter does not advance).  Unlike the reference's thread pool a rank cannot cancel its
queued GPU kernels, so a straggler still finishes its backward before the collectives proceed: the
mechanism reproduces the reference's update semantics, not its latency cut.
"""
from __future__ import annotations

import contextlib
import time
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ..optim.optimizer import BaseOptimizer
from ..utils import config
from ..utils.engine import Engine
from ..utils.logger import get_logger
from . import comm

log = get_logger("bigdl.parallel")


class _HostStream:
    """Stand-in for the comm-side HIP stream on the CPU: work issued "on" it runs in program
    order on the host, so waits are no-ops (lets the gloo tests drive the early-update path)."""

    def wait_stream(self, other):
        pass

    def wait_event(self, ev):
        pass


def _on(stream):
    return torch.cuda.stream(stream) if isinstance(stream, torch.cuda.Stream) else contextlib.nullcontext()


def _cur_stream(dev):
    return torch.cuda.current_stream(dev) if dev.type == "cuda" else _HostStream()


class _Bucket:
    __slots__ = ("idx", "lo", "hi", "slo", "shi", "pending", "expected", "rs_work", "ag_work", "ready",
                 "modules", "needs_shadow", "early", "rs_keep", "unpacked")

    def __init__(self, idx, lo, hi, slo, shi):
        self.idx, self.lo, self.hi, self.slo, self.shi = idx, lo, hi, slo, shi
        self.pending = 0
        self.expected = 0
        self.rs_work = None
        self.ag_work = None
        self.ready = False
        self.modules = []
        self.needs_shadow = False
        self.early = False
        self.rs_keep = None
        self.unpacked = False


class DistriOptimizer(BaseOptimizer):
    _alias = False

    def __init__(self, model, training_set, criterion, optim_method=None, end_trigger=None, batch_size=32,
                 bigdl_type="float"):
        super().__init__(model, training_set, criterion, batch_size)
        if optim_method is not None:
            if isinstance(optim_method, dict):
                self.setOptimMethods(optim_method)
            else:
                self.setOptimMethod(optim_method)
        if end_trigger is not None:
            self.setEndWhen(end_trigger)
        self.world = comm.world()
        self.rank = comm.rank()
        self.comm_dtype = str(config.get_property("bigdl.comm.dtype"))
        self.bucket_bytes = int(float(config.get_property("bigdl.comm.bucketMB")) * 2 ** 20)
        self.overlap = bool(config.get_property("bigdl.comm.overlap"))
        self.sharded = bool(config.get_property("bigdl.comm.sharded"))
        self._hook_counts: Dict[int, int] = {}
        self._overlap_active = False
        self._first_iter = True
        self._early = False
        self._side = None

    # ------------------------------------------------------------------------------ setup
    def _setup_model(self):
        from ..nn.fusion import fuse
        self._make_tracer()
        m = self.model
        m.to(self.device)
        m.training()
        fuse(m)
        from ..nn.fusion import mark_input_no_grad
        mark_input_no_grad(m)
        W = self.world
        self.flat = m.compactParametersBucketed(self.bucket_bytes, 64 * W)
        if self.flat is None:
            raise ValueError("DistriOptimizer needs a model with trainable parameters")
        comm.broadcast_module(m, 0)  # X1: identical initial replicas
        if self.device.type == "cuda" and self.compute_dtype != torch.float32:
            self.flat.enable_shadow(self.compute_dtype)
        self._method_slices = self._compute_method_slices()
        if self.sharded and not all(meth.supports_slices for meth in self.optim_methods.values()):
            log.info("OptimMethod without slice support: using replicated (all-reduce) mode")
            self.sharded = False
        # buckets + shard space
        self.buckets: List[_Bucket] = []
        soff = 0
        for i, (lo, hi) in enumerate(self.flat.buckets):
            per = (hi - lo) // W
            self.buckets.append(_Bucket(i, lo, hi, soff, soff + per))
            soff += per
        dev = self.flat.weight.device
        # one rank: its shard is the whole arena (slo == lo for every bucket), so the shard tensors
        # ALIAS the arena and the reduce-scatter / all-gather — identity copies on a one-rank group —
        # are not issued; hooks, buckets, side-stream early updates and the shard update path run as at
        # any world size (the fused update writes the fp32 masters and the bf16 compute shadow itself)
        self._alias = self.sharded and W == 1 and bool(config.get_property("bigdl.comm.aliasWorld1"))
        if self._alias:
            self.shard_w = self.flat.weight[:soff]
            self.shard_g = self.flat.grad[:soff]
            self.shard_shadow = self.flat.shadow[:soff] if self.flat.shadow is not None else None
            self.grad_wire = None
        elif self.sharded:
            self.shard_w = torch.empty(soff, dtype=torch.float32, device=dev)
            self.shard_g = torch.zeros(soff, dtype=torch.float32, device=dev)
            for b in self.buckets:
                per = b.shi - b.slo
                self.shard_w[b.slo:b.shi].copy_(self.flat.weight[b.lo + self.rank * per:b.lo + (self.rank + 1) * per])
            self.shard_shadow = None
            if self.flat.shadow is not None:
                self.shard_shadow = torch.empty(soff, dtype=self.flat.shadow.dtype, device=dev)
            self.grad_wire = None
            if self.comm_dtype.startswith("bf16"):
                self.grad_wire = torch.empty(self.flat.numel, dtype=torch.bfloat16, device=dev)
                self.shard_g_wire = torch.empty(soff, dtype=torch.bfloat16, device=dev)
        # shard ranges per OptimMethod: intersection of its arena range with each bucket's shard
        self._method_shard_ranges = {name: [] for name in self.optim_methods}
        for name, (off, n) in self._method_slices.items():
            for b in self.buckets:
                per = b.shi - b.slo
                own_lo = b.lo + self.rank * per
                own_hi = own_lo + per
                lo, hi = max(off, own_lo), min(off + n, own_hi)
                if lo < hi:
                    self._method_shard_ranges[name].append((b, b.slo + (lo - own_lo), b.slo + (hi - own_lo)))
        for meth in self.optim_methods.values():
            meth.grad_scale = 1.0 / W
            for k in ("epoch", "neval"):
                meth.state.setdefault(k, self.state[k])
        # per-element vectors (folded L2 regularizers, user lr/decay vectors) in the coordinate
        # space the method's update sees: arena slices (replicated) or this rank's shard (sharded)
        reg_full = self._fold_regularizers()
        for name, meth in self.optim_methods.items():
            off, n = self._method_slices[name]
            user_w = getattr(meth, "weightDecays", None)
            user_l = getattr(meth, "learningRates", None)
            if not self.sharded:
                if reg_full is not None:
                    meth._reg_decay = reg_full[off:off + n]
                continue
            def to_shard(vec, base_off):
                out = torch.zeros(soff, dtype=torch.float32, device=dev)
                for b in self.buckets:
                    per = b.shi - b.slo
                    own_lo = b.lo + self.rank * per
                    lo, hi = max(base_off, own_lo), min(base_off + vec.numel(), own_lo + per)
                    if lo < hi:
                        out[b.slo + (lo - own_lo):b.slo + (hi - own_lo)] = vec[lo - base_off:hi - base_off].to(dev)
                return out
            if reg_full is not None:
                meth._reg_decay = to_shard(reg_full, 0)
            if isinstance(user_w, torch.Tensor) and user_w.numel() == n:
                meth._space_wds = to_shard(user_w.float(), off)
            if isinstance(user_l, torch.Tensor) and user_l.numel() == n:
                meth._space_lrs = to_shard(user_l.float(), off)
        # module → buckets map, hooks
        self._mod_buckets = {}
        for (mod, w, g, off, n, shape) in self.flat.slices:
            for b in self.buckets:
                if b.lo <= off < b.hi:
                    self._mod_buckets.setdefault(id(mod), set()).add(b.idx)
                    if mod not in b.modules:
                        b.modules.append(mod)
        for b in self.buckets:
            b.expected = len(b.modules)
        self._install_hooks()
        if dev.type == "cuda":
            prio = int(config.get_property("bigdl.comm.streamPriority"))
            self._side = torch.cuda.Stream(device=dev, priority=prio)
        else:
            self._side = _HostStream()
        self._early_ok = self.sharded and bool(config.get_property("bigdl.comm.earlyUpdate"))
        # straggler drop state (P5)
        self._drop_iter = 0
        self._drop_threshold = None
        self._drop_times = [0.0] * max(1, getattr(self, "_straggler_window", 1))
        self._dropped_in_window = 0
        self._finished = self.world
        self._skipped = False
        log.info(f"DistriOptimizer: world={W} params={self.flat.numel} buckets={len(self.buckets)} "
                 f"mode={'sharded' if self.sharded else 'replicated'} comm={self.comm_dtype} overlap={self.overlap}")

    def _install_hooks(self):
        seen = set()
        for (mod, *_rest) in self.flat.slices:
            if id(mod) in seen:
                continue
            seen.add(id(mod))
            mod._grad_ready_hooks.append(self._on_grad_ready)
            mod._pre_forward_hooks.append(self._on_pre_forward)

    # ------------------------------------------------------------------------------ hooks
    def _on_grad_ready(self, mod):
        k = id(mod)
        self._hook_counts[k] = self._hook_counts.get(k, 0) + 1
        if not self._overlap_active:
            return
        for bi in self._mod_buckets.get(k, ()):
            b = self.buckets[bi]
            b.pending -= 1
            if b.pending == 0:
                self._launch_reduce(b)
                if self._early:
                    self._early_update(b)

    def _early_update(self, b: _Bucket):
        """Shard update + all-gather of bucket ``b`` on the comm-side stream, queued behind its
        reduce-scatter (issued on the same stream) while backward continues on the compute stream
        (the reference's lazy per-block ``updateParameter``, ParallelOptimizer.scala:404-470,
        without the wait)."""
        b.rs_keep = b.rs_work
        with _on(self._side):
            self._finish_reduce(b)
            self._update_bucket(b)
            self._launch_gather(b)
        b.early = True

    def _on_pre_forward(self, mod):
        for bi in self._mod_buckets.get(id(mod), ()):
            b = self.buckets[bi]
            if b.ag_work is not None:
                with self.tracer.phase("send weights"):
                    b.ag_work.wait()
                b.ag_work = None
                self._after_gather(b)

    # ------------------------------------------------------------------------------ collectives
    def _launch_reduce(self, b: _Bucket):
        """Issue bucket ``b``'s reduce-scatter (all-reduce in replicated mode) from the comm-side
        stream.  That stream waits for the compute stream's work so far and for the weight
        gradients queued so far on the wgrad side stream — events on the GPU, the compute stream
        itself never waits here."""
        from ..ops import native_ops as NO
        side = self._side
        side.wait_stream(_cur_stream(self.flat.grad.device))
        if isinstance(side, torch.cuda.Stream):
            NO.join_wgrad(side)
        if self._alias:
            return  # the gradient shard IS the arena gradient
        with _on(side):
            g = self.flat.grad[b.lo:b.hi]
            if self.sharded:
                if self.grad_wire is not None:
                    wire = self.grad_wire[b.lo:b.hi]
                    if self.comm_dtype == "bf16_truncate":
                        from ..ops import native as N
                        if not (N.has("trunc_bf16") and N.native_ops.trunc_bf16(g, wire) is not NotImplemented):
                            wire.copy_(comm.bf16_truncate(g))
                    else:
                        # RNE pack by the bigdl cast kernel (one vectorised pass; torch copy_ if the
                        # bucket slice is not 16-B aligned or off the GPU)
                        from ..ops import native_ops as NOps
                        if NOps.cast_copy(wire, g) is NotImplemented:
                            wire.copy_(g)
                    b.rs_work = dist.reduce_scatter_tensor(self.shard_g_wire[b.slo:b.shi], wire, async_op=True)
                else:
                    b.rs_work = dist.reduce_scatter_tensor(self.shard_g[b.slo:b.shi], g, async_op=True)
            else:
                b.rs_work = dist.all_reduce(g, async_op=True)

    def _finish_reduce(self, b: _Bucket, unpack: bool = False):
        """Make the current stream wait for ``b``'s reduce-scatter.  The bf16 wire shard is read
        directly by the SGD kernel; ``unpack`` widens it into the fp32 shard (other methods,
        clipping)."""
        if b.rs_work is not None:
            with self.tracer.phase("aggregate gradient"):
                b.rs_work.wait()
            b.rs_work = None
        if unpack and self.sharded and self.grad_wire is not None and not getattr(b, "unpacked", False):
            self.shard_g[b.slo:b.shi].copy_(self.shard_g_wire[b.slo:b.shi])
            b.unpacked = True

    def _bf16_gather(self) -> bool:
        return self.comm_dtype.startswith("bf16") and self.flat.shadow is not None

    def _launch_gather(self, b: _Bucket):
        if not self.sharded or self._alias:
            return
        if self._bf16_gather():
            # reference wire format: replicas compute with the bf16 copy of the weights
            b.ag_work = dist.all_gather_into_tensor(self.flat.shadow[b.lo:b.hi], self.shard_shadow[b.slo:b.shi],
                                                    async_op=True)
        else:
            b.ag_work = dist.all_gather_into_tensor(self.flat.weight[b.lo:b.hi], self.shard_w[b.slo:b.shi],
                                                    async_op=True)
        b.needs_shadow = True

    def _after_gather(self, b: _Bucket):
        if not b.needs_shadow:
            return
        from .. import ops
        from ..ops import fp32x3
        fp32x3.mark_dirty(self.flat.weight[b.lo:b.hi])  # fp32-mode weight operands derived from them
        if self._bf16_gather():
            # fp32 view of the gathered bf16 weights for layers that read fp32 params (BN γ/β);
            # exact fp32 masters stay in this rank's shard
            ops.cast_copy(self.flat.weight[b.lo:b.hi], self.flat.shadow[b.lo:b.hi])
        elif self.flat.shadow is not None:
            ops.cast_copy(self.flat.shadow[b.lo:b.hi], self.flat.weight[b.lo:b.hi])
        b.needs_shadow = False

    # ------------------------------------------------------------------------------ iteration
    def _drop_mode(self) -> bool:
        return self.drop_percentage > 0

    def _before_forward(self):
        for b in self.buckets:
            b.pending = b.expected
            b.early = False
            b.rs_keep = None
            b.unpacked = False
        # drop mode: a rank's gradient may still be zeroed after its backward, so no bucket is
        # sent during backward
        self._overlap_active = (self.overlap and not self._first_iter and self._overlap_ok
                                and not self._drop_mode())
        # early (in-backward) shard updates: sharded, no clipping (which needs the global gradient
        # norm before any update)
        self._early = (self._overlap_active and self._early_ok
                       and self.constant_clip is None and self.l2_clip is None)
        if self._drop_mode():
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            self._t_compute0 = time.perf_counter()
        if self._early:
            for meth in self.optim_methods.values():
                meth.begin_iteration(self.shard_w)
        self._hook_counts = {}

    @property
    def _overlap_ok(self):
        return getattr(self, "_overlap_checked", False)

    def _reduce_scalar(self, t):
        if not self._drop_mode():
            if self.world == 1:  # a one-rank all-reduce is the identity: no collective per step
                return t
            return comm.allreduce_scalar(t, average=True)
        return self._drop_decide(t)

    # ------------------------------------------------------------------------------ straggler drop (P5)
    def _drop_decide(self, loss_t):
        """After backward: this rank's compute time vs the threshold → keep or zero its gradient;
        all-reduce (loss·kept, kept) → loss over the finished ranks and the finished count."""
        from ..ops import native_ops as NO
        NO.join_wgrad()
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        dt = time.perf_counter() - self._t_compute0
        window = len(self._drop_times)
        warm = int(getattr(self, "_straggler_warmup", 0))
        dropped = (self._drop_threshold is not None and self._drop_iter > warm + window - 1
                   and dt > self._drop_threshold)
        if dropped:
            self.flat.grad.zero_()
        # a cancelled replica records no time (the reference leaves its slot at 0)
        self._drop_times[self._drop_iter % window] = 0.0 if dropped else dt
        kept = 0.0 if dropped else 1.0
        # a dropped rank's loss is SELECTED away, not multiplied by 0 (NaN · 0 = NaN would poison the
        # all-reduced loss and every loss-driven trigger)
        lv = loss_t.reshape(()).float()
        v = torch.stack([torch.where(torch.tensor(kept > 0, device=lv.device), lv, torch.zeros_like(lv)),
                         torch.ones((), device=loss_t.device) * kept])
        if comm.is_dist():
            dist.all_reduce(v)
        fin = int(round(float(v[1])))
        self._finished = fin
        self._dropped_in_window += self.world - fin
        self._rank_dropped = dropped
        if dropped:
            log.info(f"rank {self.rank}: compute {dt * 1e3:.1f} ms > drop threshold "
                     f"{self._drop_threshold * 1e3:.1f} ms, gradient dropped")
        return v[0] / max(fin, 1)

    def _drop_after_iteration(self):
        """Every ``batchsize`` counted iterations after warm-up: new threshold from the
        all-gathered compute times (``DistriOptimizer.scala:421-449``)."""
        self._drop_iter += 1
        window = len(self._drop_times)
        warm = int(getattr(self, "_straggler_warmup", 0))
        if not (self._drop_iter > warm and self._drop_iter % window == 0):
            return
        from ..utils.tracing import allgather_floats
        from ..utils.util import kthLargest
        per_rank = allgather_floats(self._drop_times) if comm.is_dist() else [self._drop_times]
        times = [int(t * 1e9) for r in per_rank for t in r]
        k = int(self.drop_percentage * window * self.world)
        if k > self._dropped_in_window:
            self._drop_threshold = kthLargest(times, 0, len(times) - 1, k - self._dropped_in_window) / 1e9
        elif self._drop_threshold is not None:
            self._drop_threshold *= 1.01
        if self.rank == 0:
            log.info(f"straggler drop threshold: {self._drop_threshold}")
        self._drop_times = [0.0] * window
        self._dropped_in_window = 0



    def _global_sum(self, t):
        if comm.is_dist():
            t = t.clone()
            dist.all_reduce(t)
        return t

    def _sync_and_update(self, loss_t, batch_size):
        from ..ops import native_ops as NO
        NO.join_wgrad()
        if self._first_iter:
            # enable overlap only if every parameterised module ran backward exactly once
            ok = all(self._hook_counts.get(id(m), 0) == 1 for b in self.buckets for m in b.modules)
            self._overlap_checked = ok
            if not ok and self.overlap:
                log.info("gradient/backward overlap disabled: shared or directly-driven parameter modules")
        fin = self.world
        if self._drop_mode():
            fin = self._finished
            if fin < self.world * (1.0 - self.max_drop_percentage) or fin == 0:
                log.warning(f"Warning! Not enough training samples were successfully processed in this iteration "
                            f"due to some slow tasks. The gradients computed in this iteration will be discarded. "
                            f"Only {fin}/{self.world} ranks successfully completed training.")
                self._skipped = True
                self._first_iter = False
                return
        # launch any bucket not launched during backward
        for b in reversed(self.buckets):
            if b.rs_work is None and not b.early:
                self._launch_reduce(b)
        if not self.sharded:
            for b in self.buckets:
                self._finish_reduce(b)
            self.flat.grad.mul_(1.0 / fin)
            for meth in self.optim_methods.values():
                meth.grad_scale = 1.0
            BaseOptimizer._sync_and_update(self, loss_t, batch_size)
            self._first_iter = False
            if self._drop_mode():
                self._drop_after_iteration()
            return
        for meth in self.optim_methods.values():
            meth.grad_scale = 1.0 / fin
        # sharded: clipping needs the global gradient norm before any update
        clipping = self.constant_clip is not None or self.l2_clip is not None
        if clipping:
            for b in self.buckets:
                self._finish_reduce(b, unpack=True)
            self.shard_g.mul_(1.0 / fin)
            for meth in self.optim_methods.values():
                meth.grad_scale = 1.0
            self._clip(self.shard_g, self.shard_g)
        if not self._early:
            for meth in self.optim_methods.values():
                meth.begin_iteration(self.shard_w)
        else:
            # buckets updated during backward: the compute stream must not touch their gradients /
            # weights (next zeroGrad, forward) before the comm-side stream has consumed them
            _cur_stream(self.flat.grad.device).wait_stream(self._side)
        for b in self._update_order():
            if b.early:
                continue
            self._finish_reduce(b)
            self._update_bucket(b)
            self._launch_gather(b)
        for meth in self.optim_methods.values():
            meth.grad_scale = 1.0 / self.world
        self.flat.mark_shadow_fresh()
        self._first_iter = False
        if self._drop_mode():
            self._drop_after_iteration()

    def _grad_for(self, meth, b: _Bucket):
        """The gradient shard ``meth`` reads for bucket ``b``: the bf16 wire shard itself for methods
        whose fused kernel widens a bf16 gradient on load (SGD, Adagrad), else the fp32 shard
        (unpacked once per bucket)."""
        if self.grad_wire is None:
            return self.shard_g
        if getattr(meth, "reads_bf16_grad", False) and not b.unpacked:
            return self.shard_g_wire
        self._finish_reduce(b, unpack=True)
        return self.shard_g

    def _update_bucket(self, b: _Bucket):
        with self.tracer.phase("compute weight"):
            for name, meth in self.optim_methods.items():
                for (bb, lo, hi) in self._method_shard_ranges[name]:
                    if bb is b:
                        sh = self.shard_shadow[lo:hi] if (self.shard_shadow is not None and (
                            self._alias or self.comm_dtype.startswith("bf16"))) else None
                        meth.apply_update(self.shard_w, self._grad_for(meth, b), lo, hi, shadow=sh)

    def _update_order(self):
        """Buckets in the order their shard update + all-gather is issued: readiness order (the
        reverse of the arena layout, which is backward order)."""
        return list(reversed(self.buckets))

    def _wait_all_gathers(self):
        for b in self.buckets:
            if b.ag_work is not None:
                with self.tracer.phase("send weights"):
                    b.ag_work.wait()
                b.ag_work = None
                self._after_gather(b)
        self.flat.mark_shadow_fresh()

    def _flush_weights(self):
        """Bring every rank's fp32 arena up to date (needed before validation/checkpoint when
        the bf16 wire format gathered only the compute shadow)."""
        self._wait_all_gathers()
        if self.sharded and self.comm_dtype.startswith("bf16") and not self._alias:
            for b in self.buckets:
                dist.all_gather_into_tensor(self.flat.weight[b.lo:b.hi], self.shard_w[b.slo:b.shi])
            from ..ops import fp32x3
            fp32x3.mark_dirty(self.flat.weight)
            self.flat.mark_shadow_fresh()

    def _finish(self):
        self._wait_all_gathers()
        self._flush_weights()
        super()._finish()

    def _on_restore(self):
        comm.broadcast_module(self.model, 0)
        if self.sharded and not self._alias:
            W, r = self.world, self.rank
            for b in self.buckets:
                per = b.shi - b.slo
                self.shard_w[b.slo:b.shi].copy_(self.flat.weight[b.lo + r * per:b.lo + (r + 1) * per])
        from ..ops import fp32x3
        fp32x3.mark_dirty(self.flat.weight)
        if self.flat.shadow is not None:
            self.flat.refresh_shadow()

    def checkpoint(self, asynchronous: bool = False):
        """Gather the shards (X14) then rank 0 writes ``model.<neval>`` / ``optimMethod-*``.
        Optimizer state is per shard: each rank writes its own state file next to it."""
        from ..serialization.checkpoint import save_checkpoint, save_shard_state, wait_checkpoints
        self._flush_weights()
        if Engine.rank() == 0:
            save_checkpoint(self.checkpoint_path, self.model, self.optim_methods, self.state, self.is_overwrite,
                            world_size=self.world, sharded=self.sharded, asynchronous=asynchronous,
                            slices=self._method_slices)
        if self.sharded:
            save_shard_state(self.checkpoint_path, self.optim_methods, self.state, self.rank, self.is_overwrite,
                             asynchronous=asynchronous, slices=self._method_slices)
        if not asynchronous:
            wait_checkpoints()
        comm.barrier()


class ParallelOptimizer(DistriOptimizer):
    """Layer-wise overlapped data parallelism (``DL/optim/ParallelOptimizer.scala:42-791``).

    The reference pushes each layer group's gradient as soon as its backward finishes (parameters
    split into ``parameterBlocks`` = 10 groups), aggregates and updates the groups in PRIORITY
    order and lets the next forward start on a layer as soon as its weights are fetched.  Default
    priority = execution order (the first layer of the forward is highest, ``defaultPrioritize``
    675-683); ``setPriorities({module_name: priority})`` overrides it.

    Here: the flat arena is cut into ``parameter_blocks`` RCCL buckets; reduce-scatters launch from
    the backward hooks as each bucket completes; shard updates and all-gathers are then issued in
    descending bucket priority (a bucket's priority = the highest of its modules), so the buckets
    the next forward needs first are gathered first and the forward's per-layer wait (pre-forward
    hook) releases as early as possible.  Per-sub-module OptimMethods (``setOptimMethods`` by
    module name) are supported as in DistriOptimizer.
    """

    def __init__(self, model, training_set, criterion, optim_method=None, end_trigger=None, batch_size=32,
                 parameter_blocks: int = 10, bigdl_type="float"):
        super().__init__(model, training_set, criterion, optim_method, end_trigger, batch_size, bigdl_type)
        self.parameter_blocks = max(1, int(parameter_blocks))
        self._priorities: Optional[Dict[str, int]] = None

    def setPriorities(self, priorities: Dict[str, int]):
        self._priorities = dict(priorities)
        return self

    set_priorities = setPriorities

    def _default_priorities(self) -> Dict[str, int]:
        order = [m for m in self.model.flattened_modules() if m.parameters() and m.parameters()[0]]
        n = len(order)
        return {m.get_name(): n - i for i, m in enumerate(order)}

    def _setup_model(self):
        total = 0
        for w in (self.model.parameters() or ([], []))[0]:
            total += w.numel()
        per = (total + self.parameter_blocks - 1) // self.parameter_blocks
        self.bucket_bytes = max(per * 4, 1 << 20)
        super()._setup_model()
        prio = self._default_priorities()
        if self._priorities:
            prio.update(self._priorities)
        self._bucket_prio = {}
        for b in self.buckets:
            self._bucket_prio[b.idx] = max((prio.get(m.get_name(), 0) for m in b.modules), default=0)

    def _update_order(self):
        return sorted(self.buckets, key=lambda b: (-self._bucket_prio.get(b.idx, 0), -b.idx))
