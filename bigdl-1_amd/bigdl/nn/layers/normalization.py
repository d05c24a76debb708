"""Normalisation layers.

* ``BatchNormalization`` / ``SpatialBatchNormalization`` — ``DL/nn/BatchNormalization.scala``
  (eps 1e-5, momentum 0.1, running stats ``runningMean``/``runningVar`` (variance, unbiased),
  saved ``saveMean``/``saveStd`` (=1/√(var+eps)); default init γ~U(0,1), β=0 (:107-109)) and
  ``SpatialBatchNormalization.scala`` (NCHW/NHWC; cross-replica sync via ``setParallism``).
  Device path: NHWC two-stage Welford/one-pass statistics + apply kernels with optional fused
  ReLU / residual add (K5/K7/K8/K9).
* ``SpatialCrossMapLRN`` (``SpatialCrossMapLRN.scala:96-200``), ``SpatialWithinChannelLRN``,
  ``LayerNormalization``, ``Normalize``, ``NormalizeScale``, ``SpatialSubtractive/Divisive/
  ContrastiveNormalization``.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from ... import ops
from ..abstractnn import TensorModule, AutogradModule
from ..initialization_method import RandomUniform, Zeros, Ones, VariableFormats
from .conv import to_device_layout
from ...utils import acc_float, config


_SYNCBN_COMM = {}


def _syncbn_comm():
    """The process group SyncBN statistics are all-reduced over when a layer has no explicit
    group: with ``bigdl.syncbn.ownComm`` one extra communicator over all ranks, created once (every
    rank reaches its first SyncBN forward in the same order, so the collective ``new_group`` call
    matches up) — RCCL gives each communicator its own stream, so the 2·C+1-float statistics
    collectives are not serialised behind the gradient buckets (``parallel/distri_optimizer.py``);
    otherwise the default group."""
    import torch.distributed as dist
    if not config.get_property("bigdl.syncbn.ownComm") or dist.get_world_size() == 1:
        return None
    key = id(dist.distributed_c10d._get_default_group())
    g = _SYNCBN_COMM.get(key)
    if g is None:
        g = _SYNCBN_COMM[key] = dist.new_group(list(range(dist.get_world_size())))
    return g


class BatchNormalization(TensorModule):
    def __init__(self, n_output, eps=1e-5, momentum=0.1, affine=True, init_weight=None, init_bias=None,
                 init_grad_weight=None, init_grad_bias=None, bigdl_type="float"):
        super().__init__()
        if n_output <= 0:
            raise ValueError("output feature map number must be greater than zero")
        self.nOutput = n_output
        self.eps = eps
        self.momentum = momentum
        self.affine = affine
        self.register_buffer("runningMean", torch.zeros(n_output))
        self.register_buffer("runningVar", torch.ones(n_output))
        self.saveMean = torch.zeros(n_output)
        self.saveStd = torch.zeros(n_output)
        if affine:
            self.register_parameter("weight", torch.zeros(n_output) if init_weight is None else
                                    torch.as_tensor(init_weight, dtype=torch.float32).reshape(n_output))
            self.register_parameter("bias", torch.zeros(n_output) if init_bias is None else
                                    torch.as_tensor(init_bias, dtype=torch.float32).reshape(n_output))
        else:
            self.weight = self.bias = self.gradWeight = self.gradBias = None
        self._has_init_w = init_weight is not None
        self._has_init_b = init_bias is not None
        self._init_weight_method = RandomUniform(0, 1)
        self._init_bias_method = Zeros()
        self._fused_relu = False
        self._defer_ok = False  # nn/fusion.py shortcutbn: the fused block tail applies this BN
        #: the conv consuming this BN + ReLU's output (nn/fusion.py, bnbwd): in fp32 compute the output
        #: may be handed over deferred (BNOut) and applied in that conv's operand prologues
        self._pro_consumer = None
        self._sync_group = None
        self._sync = False
        self._sync_force = False
        self.reset()

    def reset(self):
        if self.affine:
            if not self._has_init_w:
                self._init_weight_method.init(self.weight, VariableFormats.ONE_D)
            if not self._has_init_b:
                self._init_bias_method.init(self.bias, VariableFormats.ONE_D)
        self.runningMean.zero_()
        self.runningVar.fill_(1.0)
        self.zeroGradParameters()
        return self

    # --- SyncBN (P6 / X11): reference setParallism registers cross-replica sums -------------
    def setParallism(self, parallism: int):
        """Compat: in the reference this syncs ``parallism`` replica threads; on HIP it enables
        cross-rank SyncBN over the default process group."""
        self._sync = parallism is not None and parallism > 1
        return self

    def set_sync_group(self, group=None, enabled: bool = True, force: bool = False):
        """Cross-rank statistics over ``group``; ``force`` keeps the collective path even when the
        group has a single rank (a world-size-1 rehearsal of the multi-rank kernels)."""
        self._sync = enabled
        self._sync_group = group
        self._sync_force = force
        return self

    def _sync_active(self):
        if not self._sync:
            return False
        # asked ~7 times per BN call: cached against the process group, the sync settings and the
        # property version (the uncached checks cost ~37 µs of host time per BN call, enough to make
        # the ResNet-50 step host-bound under SyncBN)
        import torch.distributed as dist
        pg = dist.distributed_c10d.GroupMember.WORLD if dist.is_available() else None
        token = (id(pg), id(self._sync_group), self._sync_force, config.version())
        c = self.__dict__.get("_sa_cache")
        if c is not None and c[0] == token:
            return c[1]
        on = _dist_ready(self._sync_force)
        if on and config.get_property("bigdl.bn.syncOneRankLocal") and self._sync_world() == 1:
            # a one-rank group: the all-reduce is the identity and the global statistics ARE the
            # local ones, so the local finalize+apply kernels run (the launch count of local BN)
            on = False
        self.__dict__["_sa_cache"] = (token, on)
        return on

    def _sync_world(self):
        import torch.distributed as dist
        grp = self._sync_group
        return dist.get_world_size(grp) if grp is not None else dist.get_world_size()

    def _to_nchw_like(self, x):
        return x

    def _shape_in(self, input):
        """BN over dim 1 of (N, C) or (N, C, ...)."""
        return input

    # --- fusion hooks (set by bigdl.nn.fusion) ---------------------------------------------
    #: conv whose bias was folded into this BN (its output excludes the bias)
    _bias_producer = None
    #: (data_ptr, shape, partials, G) left by the producing conv's epilogue for the next forward
    _pending_stats = None
    #: forward scale/shift (2C fp32) of the last training forward, and its input (device layout)
    _coef = None
    _last_input = None
    #: (gm data_ptr, partials, G) left by the consuming conv's dgrad epilogue for this backward
    _pending_grad = None
    #: ReLU mask of the last fused-tail forward output as bits (uint8, one byte per 8 channels)
    _relu_bits = None

    def _atomic_sums(self, kind, C, device):
        """Persistent zeroed fp32 [2C + 1] buffer (Σ, Σ², arrival counter) a conv epilogue ADDS this BN's
        statistics into — ``kind`` "fwd": the producing conv's Σ(y−K), Σ(y−K)²; "bwd": the consuming
        conv's dgrad Σg', Σg'·(x − μ) — consumed (and re-zeroed) by the one-launch finalize+apply.
        None when the per-tile partials path is required (SyncBN, bigdl.deterministic, off)."""
        if device.type != "cuda" or config.get_property("bigdl.deterministic"):
            return None
        rep = int(config.get_property("bigdl.bn.statReplicas"))
        if self._sync_active() and not (rep > 0 and config.get_property("bigdl.bn.shiftedStats")):
            return None
        if rep > 0 and (self._sync_active() or not config.get_property("bigdl.bn.atomicStats")):
            # replicated form: [2][R][C] zeroed, tile tm adds into replica tm % R.  Two sets used in
            # alternate steps: a one-launch BN (bigdl.bn.foldFinalize) reduces its set in every apply
            # block and clears the OTHER set for the next producer; a separate finalize clears the set
            # it read.  R ≤ 16384 / C keeps the per-block reduction at ≤ 32k floats.
            rep = min(rep, 512)
            if config.get_property("bigdl.bn.foldFinalize"):
                rep = min(rep, max(4, 16384 // max(C, 1)))
            attr = "_rep_" + kind
            sets = self.__dict__.get(attr)
            if sets is None or sets[0].numel() != 2 * rep * C or sets[0].device != device:
                sets = self.__dict__[attr] = [torch.zeros(2 * rep * C, dtype=torch.float32, device=device)
                                              for _ in range(2)]
                self.__dict__["_repi_" + kind] = 0
            return sets[self.__dict__["_repi_" + kind]], rep
        if not config.get_property("bigdl.bn.atomicStats"):
            return None
        attr = "_sums_" + kind
        buf = self.__dict__.get(attr)
        if buf is None or buf.numel() != 2 * C + 1 or buf.device != device:
            buf = self.__dict__[attr] = torch.zeros(2 * C + 1, dtype=torch.float32, device=device)
        return buf

    def _drop_sums(self, pending, g_index):
        """A conv left atomically accumulated sums this BN is not consuming: clear them, or the next
        producer would add onto stale values."""
        if pending is not None and (pending[g_index] == 0 or self._is_rep(pending[g_index - 1])):
            pending[g_index - 1].zero_()

    def _is_rep(self, part):
        """``part`` is one of this BN's replicated atomic-statistics buffers (cleared by the finalize
        that reads it)."""
        return part is not None and any(part is b for a in ("_rep_fwd", "_rep_bwd") for b in (self.__dict__.get(a) or ()))

    def _rep_next(self, kind, part):
        """The other replica set of ``kind`` when ``part`` is the current one (what a one-launch BN
        clears for the next producer), else None."""
        sets = self.__dict__.get("_rep_" + kind)
        if not sets or not config.get_property("bigdl.bn.foldFinalize"):
            return None
        i = self.__dict__["_repi_" + kind]
        return sets[1 - i] if part is sets[i] else None

    def _rep_flip(self, kind, part):
        """``part`` (the current set of ``kind``) was consumed: the next producer adds into the other."""
        sets = self.__dict__.get("_rep_" + kind)
        if sets and part is sets[self.__dict__["_repi_" + kind]]:
            self.__dict__["_repi_" + kind] ^= 1

    def _advance_shift(self, mean):
        """This step's batch mean becomes the next step's statistics shift (the ring of
        :meth:`_stat_shift`)."""
        kb = self.__dict__.get("_kbuf")
        if kb is None or mean is None:
            return
        i = self.__dict__["_kidx"]
        nxt = kb[1 - i]
        if mean is not nxt:
            nxt.copy_(mean.detach().reshape(nxt.shape))
        self.__dict__["_kidx"] = 1 - i

    def _shift_next(self, shift):
        """The ring buffer the kernel may write this step's mean into (when ``shift`` is the ring's
        current K), else None."""
        kb = self.__dict__.get("_kbuf")
        if kb is None or shift is not kb[self.__dict__["_kidx"]]:
            return None
        return kb[1 - self.__dict__["_kidx"]]

    def _stat_shift(self, device=None):
        """The K the shifted statistics Σ(x − K), Σ(x − K)² subtract (every producer of this BN's
        sums — the conv epilogue, the stats pass — must use the same one).  Local BN: the running
        mean.  SyncBN: the previous step's GLOBAL batch mean (identical on every rank), held in a
        two-buffer ring — the one-launch finalize+apply then never writes what its blocks read, so
        block 0 updates the running statistics up front (batchnorm.hip BnFwdFin::early)."""
        if not (self._sync_active() or (config.get_property("bigdl.bn.foldFinalize") and self.train)):
            return self.runningMean
        kb = self.__dict__.get("_kbuf")
        rm = self.runningMean
        if kb is None or kb[0].shape != rm.shape or kb[0].device != rm.device:
            kb = self.__dict__["_kbuf"] = [rm.detach().to(torch.float32).clone(), torch.empty_like(rm, dtype=torch.float32)]
            self.__dict__["_kidx"] = 0
        return kb[self.__dict__["_kidx"]]

    def _in_bias(self):
        p = self._bias_producer
        if p is None or not getattr(p, "withBias", False):
            return None
        return p.cw("bias", torch.float32)

    def _pro_deferrable(self, x, relu, residual, coef):
        """fp32 compute: hand this BN + ReLU's output to its consumer conv deferred (bigdl.fp32.bnPrologue)."""
        c = self._pro_consumer
        if (c is None or not relu or residual is not None or not x.is_cuda or x.dtype != torch.float32
                or c._bn_bwd_target is not self or not c.train):
            return False
        if not config.get_property("bigdl.fp32.bnPrologue") or not config.get_property("bigdl.fusion.bnbwd"):
            return False
        from ...ops import fp32x3 as F3
        return F3.pro_ok(x, coef)

    def forward_residual(self, x, residual, relu):
        """y = [relu](BN(x) + residual) — the fused ResNet block tail (K9)."""
        self._residual_mode = True
        self._res_relu = relu
        try:
            self.output = self._forward_impl(x, residual, relu)
        finally:
            self._residual_mode = False
        return self.output

    def updateOutput(self, input):
        return self._forward_impl(input, None, self._fused_relu)

    def _forward_impl(self, input, residual, relu):
        from ...ops.reference import BNOut
        x = input
        if x.dim() == 1:
            x = x.unsqueeze(0)
        x = to_device_layout(x) if x.dim() == 4 else x
        # a deferred shortcut-BN output: only the native fused tail consumes it as is
        defer = (self.__dict__.pop("_defer_next", False) and residual is None and not relu and x.is_cuda
                 and x.dtype == torch.bfloat16)  # the bf16 native path only (fp32 keeps its own kernels)
        deferred_res = isinstance(residual, BNOut)
        if deferred_res and not self.train:
            residual, deferred_res = residual.dense(), False
        if residual is not None and not deferred_res and residual.dim() == 4:
            residual = to_device_layout(residual)
        pdt = torch.float64 if x.dtype == torch.float64 else torch.float32  # statistics dtype
        g = self.cw("weight", pdt) if self.affine else None
        b = self.cw("bias", pdt) if self.affine else None
        ib = self._in_bias()
        self._last_relu = relu
        if self.train:
            if self._sync_active():
                y, mean, invstd = self._sync_forward(x, g, b, relu, residual, ib, defer=defer)
            else:
                r = NotImplemented
                C_ = x.shape[1]
                coef = self._coef
                if coef is None or coef.numel() != 2 * C_ or coef.device != x.device:
                    coef = self._coef = torch.empty(2 * C_, dtype=torch.float32, device=x.device)
                ps, self._pending_stats = self._pending_stats, None
                bits = self._tail_bits(x, relu, residual)
                self._relu_bits = None
                if ps is not None and ps[0] == x.data_ptr() and ps[1] == tuple(x.shape):
                    special = defer or deferred_res
                    # fp32: a mid-block BN + ReLU whose consumer conv applies it on load
                    pdefer = not special and self._pro_deferrable(x, relu, residual, coef)
                    r = ops.native_ops.batchnorm_forward_train_partials(
                        x, ps[2], ps[3], g, b, self.runningMean, self.runningVar, self.momentum, self.eps,
                        relu=relu, residual=residual, in_bias=ib, coef_out=coef, shift=ps[4],
                        bits_out=None if pdefer else bits,
                        rezero=self._is_rep(ps[2]), zero_next=None if special else self._rep_next("fwd", ps[2]),
                        mean_out=self._shift_next(ps[4]), apply=not (defer or pdefer))
                    if r is not NotImplemented and not special:
                        # (the special path finalizes without the one-launch fold: it cleared the set
                        # it read, the other set may still hold a folded step's sums — stay on this one)
                        self._rep_flip("fwd", ps[2])
                if r is NotImplemented:
                    if deferred_res:
                        residual = residual.dense()
                    self._drop_sums(ps, 3)
                    r = ops.batchnorm_forward_train(x, g, b, self.runningMean, self.runningVar,
                                                    self.momentum, self.eps, relu=relu, residual=residual,
                                                    in_bias=ib, coef_out=coef, bits_out=bits)
                self._relu_bits = bits
                y, mean, invstd = r
                if y is None:  # finalize only: the consumer (fused block tail / conv prologue) applies it
                    y = BNOut(x, coef, relu=bool(relu))
                self._advance_shift(mean)
                self._last_input = x
            self.saveMean, self.saveStd = mean, invstd
        else:
            y = ops.batchnorm_forward_infer(x, g, b, self.runningMean, self.runningVar, self.eps, relu=False,
                                            in_bias=ib)
            if residual is not None:
                y = y + residual
            if relu:
                y = torch.relu(y)
        return y.reshape(input.shape) if input.dim() == 1 else y

    def _tail_bits(self, x, relu, residual):
        """A fused block tail (ReLU(BN(x) + shortcut)) on the GPU also emits its output's ReLU mask
        as bits: the next block's dgrad epilogue reads 1/16 of the bytes of the output."""
        if not (residual is not None and relu and x.is_cuda and x.dim() == 4 and x.shape[1] % 8 == 0
                and getattr(self, "_residual_mode", False)):
            return None
        n = x.numel() // 8
        bits = self._relu_bits
        if bits is None or bits.numel() != n or bits.device != x.device:
            bits = torch.empty(n, dtype=torch.uint8, device=x.device)
        return bits

    def _lazy_grad_ok(self, input, x):
        """Return the input gradient deferred (a BNGrad) when the producing conv — the only consumer
        of that gradient — is a 1×1 stride-1 native conv that applies it in its backward prologues."""
        prod = self._bias_producer
        if prod is None or input is not x or x.dim() != 4 or not x.is_cuda or x.dtype != torch.bfloat16:
            return False
        mode = int(config.get_property("bigdl.fusion.bnprologue"))
        if mode <= 0 or (mode == 1 and x.shape[1] >= getattr(prod, "nInputPlane", 0)):
            return False
        k = (getattr(prod, "kernelH", 0), getattr(prod, "kernelW", 0), getattr(prod, "strideH", 0),
             getattr(prod, "strideW", 0), getattr(prod, "padH", -1), getattr(prod, "padW", -1),
             getattr(prod, "nGroup", 0))
        return (k == (1, 1, 1, 1, 0, 0, 1) and prod.format == "NCHW" and x.shape[1] % 32 == 0
                and x.is_contiguous(memory_format=torch.channels_last))

    def _sync_allreduce(self, t):
        """Sum ``t`` over the sync group in place; a one-rank group (the forced world-size-1
        rehearsal) is the identity, so no collective is issued.  Without an explicit group the
        statistics go over a communicator of their own (:func:`_syncbn_comm`): its stream is not
        the one the data-parallel gradient reduce-scatter / all-gather buckets queue on, so a
        forward BN never waits behind the previous step's late all-gathers."""
        import torch.distributed as dist
        ws = self.__dict__.get("_sync_ws")
        if ws is None or ws[0] is not self._sync_group:
            grp = self._sync_group if self._sync_group is not None else _syncbn_comm()
            ws = self.__dict__["_sync_ws"] = (self._sync_group, dist.get_world_size(grp), grp)
        if ws[1] > 1:
            dist.all_reduce(t, group=ws[2])

    def _sync_ops(self, x):
        """The SyncBN sums contract (``bn_local_sums`` → all-reduce → ``bn_forward_from_sums``; the
        backward twins): the HIP kernels for a native bf16 NHWC activation, otherwise the reference
        implementation of the same contract (CPU, fp32), so every device issues the same host
        sequence and collectives — the gloo multi-rank tests run exactly the GPU path's logic."""
        from ...ops import native_ops as NO, reference as R
        if (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] % 8 == 0
                and ops.native_has("batchnorm_forward_train")):
            return NO
        return R

    def _sync_forward(self, x, g, b, relu=False, residual=None, in_bias=None, defer=False):
        """SyncBN forward (``SpatialBatchNormalization.scala:1114-1151``): this rank's shifted sums
        [Σ(x−K), Σ(x−K)², rows] (from the producing conv's epilogue partials when it left them) →
        ONE all-reduce of 2·C + 1 floats → finalize over the global row count (read on the device:
        no host sync, and ranks with uneven batches still issue identical collectives) → apply
        (+residual, ReLU).  K is the running mean, identical on every rank.  As in the local path, a
        projection-shortcut BN (``defer``) only finalizes and returns its output deferred
        (:class:`~bigdl.ops.reference.BNOut`), and the block tail applies it inside its own pass."""
        from ...ops import reference as R
        impl = self._sync_ops(x)
        C_ = x.shape[1]
        coef = self._coef
        if coef is None or coef.numel() != 2 * C_ or coef.device != x.device:
            coef = self._coef = torch.empty(2 * C_, dtype=torch.float32, device=x.device)
        ps, self._pending_stats = self._pending_stats, None
        bits = self._tail_bits(x, relu, residual) if impl is not R else None
        self._relu_bits = None
        r = NotImplemented
        for m in ((impl, R) if impl is not R else (R,)):
            if m is not R and ps is not None and ps[0] == x.data_ptr() and ps[1] == tuple(x.shape) \
                    and ps[4] is not None:
                shift = ps[4]
                sums = m.bn_local_sums(x, shift, ps[2], ps[3], rezero=self._is_rep(ps[2]))
                ps = None  # consumed
            else:
                shift = self._stat_shift()
                sums = m.bn_local_sums(x, shift)
            if sums is NotImplemented:
                continue
            self._sync_allreduce(sums)  # the ONE collective of this call: a failed apply reuses its sums
            kb = self.__dict__.get("_kbuf")
            nxt = kb[1 - self.__dict__["_kidx"]] if (kb is not None and shift is kb[self.__dict__["_kidx"]]) else None
            kw = dict(mean_out=nxt) if (m is not R and nxt is not None) else {}
            r = m.bn_forward_from_sums(x, sums, 0, shift, g, b, self.runningMean, self.runningVar, self.momentum,
                                       self.eps, relu=relu, residual=residual, in_bias=in_bias, coef_out=coef,
                                       bits_out=bits if (m is not R and not defer) else None, apply=not defer, **kw)
            if r is NotImplemented and m is not R:
                m = R
                r = R.bn_forward_from_sums(x, sums, 0, shift, g, b, self.runningMean, self.runningVar,
                                           self.momentum, self.eps, relu=relu, residual=residual, in_bias=in_bias,
                                           coef_out=coef, apply=not defer)
            if r is not NotImplemented:
                if r[0] is None:  # finalize only: the fused block tail applies it
                    r = (R.BNOut(x, coef, relu=bool(relu)),) + tuple(r[1:])
                self._relu_bits = bits if m is not R else None
                self._sync_path = "native" if m is not R else "reference"
                self._last_input = x
                if nxt is not None:  # this step's global mean is the next step's shift
                    if r[1] is not nxt:
                        nxt.copy_(r[1])
                    self.__dict__["_kidx"] ^= 1
                break
        self._drop_sums(ps, 3)  # replicated statistics left by the conv and not read: clear them
        return r

    def _bwd(self, input, gradOutput, need_input, acc, want_gres=False):
        x = input if input.dim() > 1 else input.unsqueeze(0)
        gy = gradOutput if gradOutput.dim() > 1 else gradOutput.unsqueeze(0)
        if x.dim() == 4:
            x = to_device_layout(x)
            gy = to_device_layout(gy)
        relu = getattr(self, "_last_relu", self._fused_relu)
        y = self.output if relu else None
        from ...ops.reference import BNOut
        if isinstance(y, BNOut):
            y = None if (self._pending_grad is not None and self._pending_grad[0] == gy.data_ptr()) else y.dense()
        if y is not None and y.dim() == 1:
            y = y.unsqueeze(0)
        g = self.cw("weight", torch.float64 if x.dtype == torch.float64 else torch.float32) if self.affine else None
        prod = self._bias_producer
        cb = prod.gradBias if (acc and prod is not None and getattr(prod, "withBias", False)) else None
        cbs = prod.scale_b if prod is not None else 0.0
        gres = None
        if self._sync_active() and self.train:
            # gy already ReLU-masked by the consumer conv's dgrad epilogue (which also left the
            # backward partials): it is then also exactly the residual branch's gradient
            pg = self._pending_grad
            pre_masked = pg is not None and pg[0] == gy.data_ptr()
            gi, cb_done = self._sync_backward(x, gy, g, y, need_input, acc, relu, cb, cbs)
            if cb is not None and gi is not None and not cb_done:
                cb.add_(acc_float(gi).sum([d for d in range(gi.dim()) if d != 1]), alpha=cbs)
            if want_gres:
                gres = gy * (y > 0).to(gy.dtype) if (relu and not pre_masked) else gy
        else:
            same = self.scale_w == self.scale_b
            pg, self._pending_grad = self._pending_grad, None
            if pg is not None and pg[0] == gy.data_ptr() and relu and same:
                # gy is already ReLU-masked (by the consumer conv's dgrad epilogue), which is also
                # exactly the gradient a fused residual shortcut receives
                gi = ops.native_ops.batchnorm_backward_partials(
                    gy, x, g, self.saveMean, self.saveStd, pg[1], pg[2], need_input=need_input,
                    gg_acc=self.gradWeight if (acc and self.affine) else None,
                    gb_acc=self.gradBias if (acc and self.affine) else None,
                    scale=self.scale_w if acc else 0.0, cbias_acc=cb, cbias_scale=cbs,
                    lazy=self._lazy_grad_ok(input, x), rezero=self._is_rep(pg[1]),
                    zero_next=self._rep_next("bwd", pg[1]))
                if gi is not NotImplemented:
                    self._rep_flip("bwd", pg[1])
                    if gi is not None and input.dim() == 1:
                        gi = gi.reshape(input.shape)
                    return (gi, gy) if want_gres else gi
            self._drop_sums(pg, 2)  # (reached only when the sums were not consumed)
            gi, gres = ops.batchnorm_backward(gy, x, g, self.saveMean, self.saveStd, y=y, relu=relu,
                                              need_input=need_input,
                                              gg_acc=self.gradWeight if (acc and self.affine) else None,
                                              gb_acc=self.gradBias if (acc and self.affine and same) else None,
                                              scale=self.scale_w if acc else 0.0, cbias_acc=cb, cbias_scale=cbs,
                                              want_gres=want_gres)
            if acc and self.affine and not same and self.scale_b != 0:
                gf = acc_float(gy) * ((y > 0).float() if relu else 1.0)
                dims = [d for d in range(gf.dim()) if d != 1]
                self.gradBias.add_(gf.sum(dims), alpha=self.scale_b)
        if gi is not None and input.dim() == 1:
            gi = gi.reshape(input.shape)
        if want_gres:
            return gi, gres
        return gi

    def backward_residual(self, input, gradOutput):
        """Backward of :meth:`forward_residual`: returns (gradInput, gradient for the residual)."""
        gi, gres = self._bwd(input, gradOutput, True, True, want_gres=True)
        self.gradInput = gi
        for h in self._grad_ready_hooks:
            h(self)
        return gi, gres

    def _sync_backward(self, x, gy, g, y, need_input, acc, relu=None, cb=None, cbs=0.0):
        """SyncBN backward (``SpatialBatchNormalization.scala:1257-1329``): local [Σg', Σg'·(x − μ)]
        → this rank's dγ/dβ (the data-parallel gradient all-reduce sums them across ranks); the
        same sums + the row count all-reduced (2·C + 1 floats) → the input-gradient coefficients
        → one apply pass.  → (gradInput, whether the folded producer bias ``cb`` was accumulated)."""
        from ...ops import reference as R
        relu = self._fused_relu if relu is None else relu
        impl = self._sync_ops(x)
        pg, self._pending_grad = self._pending_grad, None
        C = x.shape[1]
        rows = x.numel() // C
        for m in ((impl, R) if impl is not R else (R,)):
            rl = relu
            both = NotImplemented
            if m is not R and pg is not None and pg[0] == gy.data_ptr() and relu:
                # gy is already ReLU-masked by the consumer conv's dgrad epilogue, which also left
                # the backward partial sums: reduce those instead of re-reading gy, x, y
                both = m.bn_bwd_partials_sums(pg[1], pg[2], C, x.device, rows=rows, rezero=self._is_rep(pg[1]))
                if both is not NotImplemented:
                    rl = False
                    pg = None  # consumed
            if both is NotImplemented:
                both = m.bn_bwd_local_sums(gy, x, self.saveMean, y=y, relu=rl)
            if both is NotImplemented:
                continue
            loc, glob = both[:2 * C], both[2 * C:]
            self._sync_allreduce(glob)  # the ONE collective of this call: a failed apply reuses its sums
            kw = dict(need_input=need_input, gg_acc=self.gradWeight if (acc and self.affine) else None,
                      gb_acc=self.gradBias if (acc and self.affine) else None, scale=self.scale_w if acc else 0.0,
                      cbias_acc=cb, cbias_scale=cbs)
            gi = m.bn_backward_from_sums(gy, x, g, self.saveMean, self.saveStd, loc, glob, 0, y=y, relu=rl, **kw)
            if gi is NotImplemented and m is not R:
                m = R
                gi = R.bn_backward_from_sums(gy, x, g, self.saveMean, self.saveStd, loc, glob, 0, y=y, relu=rl, **kw)
            if gi is NotImplemented:
                raise RuntimeError("SyncBN backward: no implementation accepted the all-reduced sums")
            if acc and self.affine and self.scale_b != self.scale_w:
                self.gradBias.add_(loc[:C], alpha=self.scale_b - self.scale_w)
            self._sync_bwd_path = "native" if m is not R else "reference"
            self._drop_sums(pg, 2)  # replicated statistics left by the dgrad and not read
            return gi, cb is not None
        raise RuntimeError("SyncBN backward: no implementation accepted the input")

    def updateGradInput(self, input, gradOutput):
        gi = self._bwd(input, gradOutput, True, True)
        self._gi_done = True
        return gi

    def accGradParameters(self, input, gradOutput):
        if not getattr(self, "_gi_done", False):
            self._bwd(input, gradOutput, False, True)
        self._gi_done = False

    def set_running_mean(self, v):
        self.runningMean.copy_(torch.as_tensor(v))
        return self

    def set_running_std(self, v):
        self.runningVar.copy_(torch.as_tensor(v))
        return self

    def __repr__(self):
        return f"{type(self).__name__}[{self.get_name()}]({self.nOutput}, {self.eps}, {self.momentum}, {self.affine})"


class SpatialBatchNormalization(BatchNormalization):
    def __init__(self, n_output, eps=1e-5, momentum=0.1, affine=True, init_weight=None, init_bias=None,
                 init_grad_weight=None, init_grad_bias=None, data_format="NCHW", bigdl_type="float"):
        super().__init__(n_output, eps, momentum, affine, init_weight, init_bias, init_grad_weight, init_grad_bias)
        self.dataFormat = data_format

    def updateOutput(self, input):
        if self.dataFormat == "NHWC":
            y = super().updateOutput(input.permute(0, 3, 1, 2))
            return y.permute(0, 2, 3, 1)
        return super().updateOutput(input)

    def updateGradInput(self, input, gradOutput):
        if self.dataFormat == "NHWC":
            saved = self.output
            self.output = saved.permute(0, 3, 1, 2)
            gi = super().updateGradInput(input.permute(0, 3, 1, 2), gradOutput.permute(0, 3, 1, 2))
            self.output = saved
            return gi.permute(0, 2, 3, 1)
        return super().updateGradInput(input, gradOutput)

    def accGradParameters(self, input, gradOutput):
        if self.dataFormat == "NHWC":
            if not getattr(self, "_gi_done", False):
                saved = self.output
                self.output = saved.permute(0, 3, 1, 2)
                self._bwd(input.permute(0, 3, 1, 2), gradOutput.permute(0, 3, 1, 2), False, True)
                self.output = saved
            self._gi_done = False
            return
        super().accGradParameters(input, gradOutput)


def _dist_ready(single_rank_ok=False):
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized() and (single_rank_ok or dist.get_world_size() > 1)


class SpatialCrossMapLRN(TensorModule):
    """Cross-channel LRN: y = x / (k + α/size·Σ x²)^β (``SpatialCrossMapLRN.scala:96-200``)."""

    def __init__(self, size=5, alpha=1.0, beta=0.75, k=1.0, data_format="NCHW", bigdl_type="float"):
        super().__init__()
        self.size, self.alpha, self.beta, self.k = size, alpha, beta, k
        self.format = data_format

    def _f(self, x):
        nhwc = self.format == "NHWC"
        if nhwc:
            x = x.permute(0, 3, 1, 2)
        batched = x.dim() == 4
        if not batched:
            x = x.unsqueeze(0)
        y = ops.lrn_forward(x, self.size, self.alpha, self.beta, self.k)
        if not batched:
            y = y.squeeze(0)
        return y.permute(0, 2, 3, 1) if nhwc else y

    def updateOutput(self, input):
        return self._f(input)

    def updateGradInput(self, input, gradOutput):
        nhwc = self.format == "NHWC"
        x, gy = input, gradOutput
        if nhwc:
            x, gy = x.permute(0, 3, 1, 2), gy.permute(0, 3, 1, 2)
        batched = x.dim() == 4
        if not batched:
            x, gy = x.unsqueeze(0), gy.unsqueeze(0)
        gx = ops.lrn_backward(gy, x, self.size, self.alpha, self.beta, self.k)
        if not batched:
            gx = gx.squeeze(0)
        return gx.permute(0, 2, 3, 1) if nhwc else gx


class SpatialWithinChannelLRN(AutogradModule):
    """LRN inside each channel over a size×size spatial window (``SpatialWithinChannelLRN.scala``)."""

    def __init__(self, size=5, alpha=1.0, beta=0.75, bigdl_type="float"):
        super().__init__()
        self.size, self.alpha, self.beta = size, alpha, beta

    def _forward(self, x):
        batched = x.dim() == 4
        if not batched:
            x = x.unsqueeze(0)
        p = (self.size - 1) // 2
        sq = F.avg_pool2d(x * x, self.size, 1, p, count_include_pad=True)
        y = x * torch.pow(1 + self.alpha * sq, -self.beta)
        return y if batched else y.squeeze(0)


class LayerNormalization(AutogradModule):
    """Transformer layer norm (``LayerNormalization.scala``): weight init 1, bias 0, eps 1e-6."""

    def __init__(self, hidden_size, bigdl_type="float"):
        super().__init__()
        self.hiddenSize = hidden_size
        self.register_parameter("weight", torch.ones(hidden_size))
        self.register_parameter("bias", torch.zeros(hidden_size))

    def _forward(self, x):
        if x.is_cuda and ops.native_has("layer_norm"):
            # fused one-wave-per-row kernel (layernorm.hip) instead of 8 composed launches
            y = ops.native_ops.layer_norm(x, self.P("weight"), self.P("bias"), 1e-6)
            if y is not NotImplemented:
                return y
            ops.native.note_fallback("layer_norm", "geometry", (x,))
        mean = x.mean(-1, keepdim=True)
        var = ((x - mean) ** 2).mean(-1, keepdim=True)
        return (x - mean) * torch.rsqrt(var + 1e-6) * self.P("weight").to(x.dtype) + self.P("bias").to(x.dtype)


class Normalize(AutogradModule):
    """Lp-normalise along the feature dim (``Normalize.scala``)."""

    def __init__(self, p, eps=1e-10, bigdl_type="float"):
        super().__init__()
        self.p, self.eps = p, eps

    def _forward(self, x):
        dim = 1 if x.dim() > 1 else 0
        if math.isinf(self.p):
            n = x.abs().amax(dim, keepdim=True)
        else:
            n = (x.abs().pow(self.p).sum(dim, keepdim=True) + self.eps).pow(1.0 / self.p)
        return x / n


class NormalizeScale(AutogradModule):
    """L2-normalise then per-channel scale (SSD, ``NormalizeScale.scala``)."""

    def __init__(self, p, scale, size, w_regularizer=None, eps=1e-10, bigdl_type="float"):
        super().__init__()
        self.p, self.eps = p, eps
        self.register_parameter("weight", torch.full(tuple(size), float(scale)))

    def _forward(self, x):
        n = (x.abs().pow(self.p).sum(1, keepdim=True) + self.eps).pow(1.0 / self.p)
        return x / n * self.P("weight").to(x.dtype)


def _gauss_kernel(size):
    if isinstance(size, torch.Tensor):
        return acc_float(size)
    k = torch.ones(size, size)
    return k


class SpatialSubtractiveNormalization(AutogradModule):
    """x − weighted local mean (``SpatialSubtractiveNormalization.scala``)."""

    def __init__(self, n_input_plane=1, kernel=None, bigdl_type="float"):
        super().__init__()
        self.nInputPlane = n_input_plane
        k = torch.ones(9, 9) if kernel is None else torch.as_tensor(kernel, dtype=torch.float32)
        if k.dim() == 1:
            k = torch.outer(k, k)
        self.kernel = k / (k.sum() * n_input_plane)

    def _mean(self, x):
        kh, kw = self.kernel.shape
        w = self.kernel.to(x.device, x.dtype).expand(1, self.nInputPlane, kh, kw)
        pad = (kw // 2, (kw - 1) // 2, kh // 2, (kh - 1) // 2)
        xp = F.pad(x, pad)
        m = F.conv2d(xp, w)
        ones = torch.ones(1, self.nInputPlane, x.shape[2], x.shape[3], device=x.device, dtype=x.dtype)
        coef = F.conv2d(F.pad(ones, pad), w)
        return m / coef

    def _forward(self, x):
        batched = x.dim() == 4
        if not batched:
            x = x.unsqueeze(0)
        y = x - self._mean(x)
        return y if batched else y.squeeze(0)


class SpatialDivisiveNormalization(SpatialSubtractiveNormalization):
    def __init__(self, n_input_plane=1, kernel=None, threshold=1e-4, thresval=1e-4, bigdl_type="float"):
        super().__init__(n_input_plane, kernel)
        self.threshold, self.thresval = threshold, thresval

    def _forward(self, x):
        batched = x.dim() == 4
        if not batched:
            x = x.unsqueeze(0)
        std = torch.sqrt(self._mean(x * x))
        mean_std = std.mean(dim=(1, 2, 3), keepdim=True)
        div = torch.maximum(std, mean_std)
        div = torch.where(div > self.threshold, div, torch.full_like(div, self.thresval))
        y = x / div
        return y if batched else y.squeeze(0)


class SpatialContrastiveNormalization(AutogradModule):
    def __init__(self, n_input_plane=1, kernel=None, threshold=1e-4, thresval=1e-4, bigdl_type="float"):
        super().__init__()
        self.sub = SpatialSubtractiveNormalization(n_input_plane, kernel)
        self.div = SpatialDivisiveNormalization(n_input_plane, kernel, threshold, thresval)

    def _forward(self, x):
        return self.div._forward(self.sub._forward(x))
