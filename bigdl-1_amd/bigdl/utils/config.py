"""Typed configuration registry.

The reference reads ~30 ``-Dbigdl.*`` JVM system properties ad hoc (e.g.
``DL/utils/Engine.scala:45-46,191-252``, ``DL/optim/DistriOptimizer.scala:882-883``,
``DL/optim/ParallelOptimizer.scala:404``).  Here every key is declared once with a type and a
default; the environment variable ``BIGDL_<KEY with . → _ upper-cased>`` overrides it, and
``set_property`` overrides both at runtime.
"""
from __future__ import annotations

import os
import threading

_lock = threading.Lock()

# key -> (type, default, doc)
_REGISTRY = {
    # engine / topology
    "bigdl.localMode": (bool, False, "run without a process group"),
    "bigdl.coreNumber": (int, 0, "host threads for CPU ops (0 = auto)"),
    "bigdl.engineType": (str, "hip", "kept for compatibility: 'mklblas'/'mkldnn' map to the native engine"),
    "bigdl.multiModels": (bool, False, "compat flag (one replica per GPU here)"),
    "bigdl.utils.Engine.defaultPoolSize": (int, 0, "host pool size"),
    "bigdl.check.singleton": (bool, False, "compat"),
    # failure handling
    "bigdl.failure.retryTimes": (int, 5, "optimizer retry budget"),
    "bigdl.graph.capture": (bool, False, "LocalOptimizer on a GPU: capture the training step into a HIP graph"),
    "bigdl.comm.timeout": (float, 600.0, "collective watchdog: seconds before a hung RCCL/gloo collective raises"),
    "bigdl.failure.retryTimeInterval": (int, 120, "retry window seconds"),
    "bigdl.failure.resume": (bool, False, "resume from the latest checkpoint at optimize() start (automatic after a launcher restart)"),
    # straggler monitor (P5, DistriOptimizer.scala:246-278,421-449)
    "bigdl.embedding.syncCheck": (bool, False, "check LookupTable ids synchronously after every GPU lookup (debug; default: the out-of-range flag is read back asynchronously and raised at the next lookup)"),
    "bigdl.straggler.window": (int, 20, "iterations between straggler checks (all-gather of per-rank step times)"),
    "bigdl.straggler.factor": (float, 1.5, "a rank is slow when its step time exceeds factor x the kthLargest threshold"),
    # parameter sync
    "bigdl.Parameter.syncPoolSize": (int, 4, "compat"),
    "bigdl.Parameter.computePoolSize": (int, 0, "compat"),
    "bigdl.parallelOptimizer.parameterBlocks": (int, 10, "number of gradient buckets for overlap mode"),
    # device / precision (new)
    "bigdl.compute.dtype": (str, "auto", "auto (bf16 on a GPU, fp32 on the host) | fp32 | bf16 compute dtype"),
    "bigdl.comm.dtype": (str, "fp32", "fp32 | bf16 | bf16_truncate wire format for gradient reduction"),
    "bigdl.comm.bucketMB": (float, 32.0, "gradient bucket size for RCCL collectives"),
    "bigdl.comm.overlap": (bool, True, "overlap gradient reduce-scatter with backward"),
    "bigdl.comm.sharded": (bool, True, "reduce-scatter + sharded update + all-gather (ZeRO-1)"),
    "bigdl.comm.channels": (int, 0, "RCCL channel cap (NCCL_MIN/MAX_NCHANNELS, set by the launcher before any GPU call; 0 = RCCL default): bounds the CUs collectives take from compute"),
    "bigdl.comm.streamPriority": (int, -1, "priority of the comm-side stream that runs the shard update + all-gather (-1 = high, 0 = normal)"),
    "bigdl.comm.aliasWorld1": (bool, True, "sharded mode with one rank: the shard tensors alias the parameter arena and the identity reduce-scatter / all-gather are skipped"),
    "bigdl.comm.earlyUpdate": (bool, True, "sharded mode on a GPU: issue each bucket's shard update + all-gather on the comm-side stream as soon as its reduce-scatter is launched (overlaps the rest of backward)"),
    # observability
    "bigdl.metrics.jsonPath": (str, "", "per-rank JSON metrics stream: one line per iteration to <path>.rank<r>.jsonl ('' = off)"),
    "bigdl.metrics.deviceTimers": (bool, False, "time the distributed phases with HIP events (adds no host sync)"),
    "bigdl.bn.atomicStats": (bool, False, "conv epilogues ADD the BN statistics into a [2C] buffer with fp32 atomics and the BN runs as ONE finalize+apply launch (forward and backward); off (or bigdl.deterministic) = per-tile partial rows + fold/finalize kernels, bit-reproducible. Off by default: the same-address atomics from thousands of tiles cost more conv time than the fold launches they remove (25.04 vs 23.09 ms/step, profiles/r4_bn_atomic_ab.txt)"),
    "bigdl.syncbn.ownComm": (bool, True, "SyncBN statistics all-reduces run over a communicator of their own (own RCCL stream), not the one the gradient buckets use"),
    "bigdl.bn.statReplicas": (int, 32, "R > 0 (with atomicStats off): conv epilogues ADD the BN statistics into R replicas (tile tm → replica tm % R) of a zeroed buffer — R-fold less same-address atomic contention than atomicStats, and the BN finalizes from R rows with no fold pass; 0 = per-tile partial rows. Default 32: 22.50 vs 22.94 ms/step (profiles/r4_bn_replicas_ab.txt)"),
    "bigdl.bn.foldFinalize": (bool, False, "training BN from a conv's replicated statistics in ONE launch per pass: every apply block reduces the replicas itself (no finalize kernel), block 0 updates the running statistics and clears the other of two alternating replica sets; the statistics shift is the previous step's batch mean (a two-buffer ring), so no block reads what block 0 writes. Off: 22.45 vs 21.05 ms/step — re-reducing the R·C replica rows in each of ~1000 apply blocks costs more than the finalize launches it removes (profiles/r5_bn_fold_ab.txt)"),
    "bigdl.bn.syncOneRankLocal": (bool, True, "a SyncBN whose sync group has ONE rank (also the forced world-size-1 rehearsal) runs the local BN kernels: the all-reduce is the identity there, so the compaction of the statistics replicas and the one-launch global finalize+apply are skipped; False rehearses the multi-rank kernels at one rank"),
    "bigdl.bn.shiftedStats": (bool, True, "conv-epilogue BN statistics as Σ(y−K), Σ(y−K)² with K = the BN running mean"),
    "bigdl.checkpoint.async": (bool, True, "trigger-driven checkpoints: host snapshot on the training thread, serialise + write on a writer thread"),
    "bigdl.predict.compiled": (bool, True, "LocalPredictor / Predictor / PredictionService on a GPU: lower the model through the IR (BN fold, conv+sum+ReLU), plan each batch shape once and replay its forward as a HIP graph (the reference's predictors always convert, LocalPredictor.scala:66)"),
    "bigdl.compile.lower": (bool, True, "nn.compiled.compile (inference phase): lower the model through the IR first (utils/intermediate.ConversionUtils: BN folded into convs / Linears, conv+sum+ReLU epilogues)"),
    "bigdl.roctx": (bool, False, "emit roctx ranges around forward / backward / reduce-scatter / update / all-gather"),
    "bigdl.native.require": (bool, True, "fail loudly on a GPU if the HIP extension is missing"),
    "bigdl.native.strict": (bool, False, "raise instead of warning when a device-tensor op falls back to the torch reference"),
    "bigdl.step.overlapMinMs": (float, 8.0, "enable the high-priority step stream and async wgrad once the measured step period is at least this long (GPU-bound steps; launch-bound ones lose to the extra host work)"),
    "bigdl.step.maxInflight": (int, 2, "GPU training iterations the host may queue ahead of the device (0 = unbounded): a host far ahead of a GPU-bound step piles up cross-stream events and fresh allocations (blocks still read by the wgrad side stream cannot be recycled) and was measured to stall for seconds (profiles/r6_fp32_runahead.txt)"),
    "bigdl.step.highPriority": (bool, True, "run each GPU training iteration on a high-priority HIP stream (the critical path outranks side-stream wgrad work)"),
    "bigdl.fp32.native": (bool, True, "fp32 compute on a GPU: convolutions and Linear run the bf16x3 split on the MFMA kernels (ops/fp32x3.py; ≤2^-16 relative per product) instead of torch/MIOpen fp32"),
    "bigdl.fp32.twoPart": (bool, True, "fp32 compute: activation splits stored as [hi | lo] and read by the conv kernels as [hi | hi | lo] (ConvParams::cdup); false = the three-part [hi | hi | lo] buffers"),
    "bigdl.fp32.producerSplit": (bool, True, "fp32 compute: the BN apply passes also write the [hi | lo] split of their output for the consuming conv (forward input, backward dY), so the conv skips its own split pass"),
    "bigdl.fp32.bnPrologue": (bool, True, "fp32 compute: a training BN + ReLU whose only consumer is a conv hands its output over deferred (ops.reference.BNOut); the conv applies relu(x·scale + shift) in its forward B-operand and weight-gradient X-operand prologues (conv_x3 / conv_wgrad PRO) and its dgrad epilogue recomputes the ReLU mask — the BN output is never written or read"),
    "bigdl.fp32.stemC4": (bool, True, "fp32 compute: a conv with ≤ 4 input channels (the RGB stem) reads a 4-channel NHWC copy of its input and gathers 8 taps × 4 channels per k-tile (conv_x3.hip MODE 2, conv_wgrad.hip C4 F32): 224 reduction indices for the 7×7 stem instead of the space-to-depth image's 512"),
    "bigdl.fp32.direct": (bool, True, "fp32 compute: convolutions with C % 32 == 0 read the fp32 activations and gradients directly (csrc/conv_x3.hip: hi / lo split while reading the MFMA fragments; conv_wgrad.hip F32: split between load and LDS store) — no [hi | lo] split is materialised and the BN passes write fp32 only"),
    "bigdl.fp32.convStats": (bool, True, "fp32 compute: a conv followed by a training BN adds the BN statistics into the BN's replicated buffer from its fp32 epilogue (the BN skips its statistics pass)"),
    "bigdl.compile.trainAutotune": (bool, True, "training compile phase: the first GPU training iteration records its conv launches (forward, backward-data, weight-gradient) and pins the fastest kernel candidate per geometry"),
    "bigdl.compile.autotune": (bool, True, "nn.compiled.compile on a GPU (inference): time every implicit-GEMM conv tile candidate per conv geometry and pin the fastest (kernel selection)"),
    "bigdl.conv.asyncWgrad": (bool, True, "inside optimizer steps run conv backward-weight kernels on a second HIP stream, overlapping the backward-data / BatchNorm chain"),
    "bigdl.deterministic": (bool, False, "bit-reproducible kernels: single-writer reductions instead of split-K float atomics (slower wgrad / embedding backward)"),
    "bigdl.native.enable": (bool, True, "False routes device tensors to the torch reference ops (debug/A-B only)"),
    "bigdl.profile.sync": (bool, False, "synchronize the device around per-module timers"),
    "bigdl.profile.deviceTimers": (bool, False, "per-module HIP-event forward/backward timers (resolved lazily by getDeviceTimes)"),
    "bigdl.optim.foldRegularizers": (bool, True, "apply pure-L2 layer regularizers inside the fused SGD update"),
    # fusion flags (bigdl.mkldnn.fusion.* equivalents, nn/mkldnn/Fusion.scala:34)
    "bigdl.int8.calibration": (str, "p99.999", "static int8 activation scale rule of quantize() after calcScales: max (max|x|, the reference's) or p99.9 / p99.99 / p99.999 (that percentile of |x|)"),
    "bigdl.int8.unsignedActivations": (bool, True, "a quantised conv whose ReLU is fused writes its non-negative int8 output as unsigned 8-bit (offset -128, scale clip/255); the consumer corrects the offset with per-tap weight sums"),
    "bigdl.int8.foldBN": (bool, True, "quantize() folds evaluation BatchNorms into the preceding convolution before quantising its weights (the reference's int8 conv + BN fusion)"),
    "bigdl.int8.residual": (bool, True, "quantize() turns ConcatTable(branch, shortcut) + CAddTable + ReLU blocks into int8 residual blocks (conv + sum epilogue, int8 block outputs chained to the next block)"),
    "bigdl.int8.quantizeLinear": (bool, True, "quantize() converts Linear layers too (int8 GEMM, per-row dynamic input scales); False keeps them in the compute dtype"),
    "bigdl.fusion": (bool, True, "enable layer fusion"),
    "bigdl.fusion.convbn": (bool, True, "fold BN into conv for inference"),
    "bigdl.fusion.bnrelu": (bool, True, "fuse BN + ReLU"),
    "bigdl.fusion.convrelu": (bool, True, "fuse conv + ReLU"),
    "bigdl.fusion.lstmstack": (bool, True, "run two stacked Recurrent(LSTM) layers on the layer wavefront"),
    "bigdl.fusion.convsum": (bool, True, "fuse residual add"),
    "bigdl.fusion.convstats": (bool, True, "conv epilogue emits the following training BN's statistics"),
    "bigdl.fusion.shortcutbn": (bool, True, "a ResNet block's conv->BN shortcut hands its BN output to the fused tail deferred (input + coefficients), applied inside the tail's pass"),
    "bigdl.fusion.bnbwd": (bool, True, "dgrad epilogue applies the producing BN's ReLU mask and its backward reductions"),
    "bigdl.fusion.bnprologue": (int, 0, "a BN whose producer is a 1x1 stride-1 conv hands it the input gradient "
                                         "deferred (A*g + B*x + C applied in the conv's dgrad / wgrad operand loads): "
                                         "0 off, 1 when the BN is narrower than the conv input, 2 always "
                                         "(profiles/r3_bn_prologue_ab.txt)"),
    # logging
    "bigdl.utils.LoggerFilter.disable": (bool, False, "disable log redirect"),
    "bigdl.utils.LoggerFilter.logFile": (str, "bigdl.log", "log file"),
    "bigdl.utils.LoggerFilter.enableSparkLog": (bool, True, "compat"),
}

_overrides: dict = {}
_listeners: dict = {}


def on_change(key: str, fn):
    """Call ``fn(value)`` whenever ``set_property``/``clear_property`` changes ``key`` (used to push
    flags such as ``bigdl.deterministic`` into the native library once instead of per call)."""
    _listeners.setdefault(key, []).append(fn)


def _env_name(key: str) -> str:
    return "BIGDL_" + key.replace("bigdl.", "", 1).replace(".", "_").upper()


def _coerce(typ, v):
    if typ is bool:
        if isinstance(v, bool):
            return v
        return str(v).strip().lower() in ("1", "true", "yes", "on")
    return typ(v)


def get_property(key: str, default=None):
    with _lock:
        if key in _overrides:
            return _overrides[key]
    typ, dflt, _ = _REGISTRY.get(key, (str, default, ""))
    env = os.environ.get(_env_name(key))
    if env is not None:
        return _coerce(typ, env)
    sysprop = os.environ.get(key)  # allow literal "bigdl.x.y" names too
    if sysprop is not None:
        return _coerce(typ, sysprop)
    return dflt if default is None else default


_VERSION = [0]


def version() -> int:
    """A counter bumped by every ``set_property`` / ``clear_property``: per-call decisions derived
    from properties can be cached against it (environment overrides are read at first use)."""
    return _VERSION[0]


def set_property(key: str, value):
    typ = _REGISTRY.get(key, (type(value), None, ""))[0]
    with _lock:
        _overrides[key] = _coerce(typ, value)
        _VERSION[0] += 1
    for fn in _listeners.get(key, ()):
        fn(get_property(key))


def clear_property(key: str):
    with _lock:
        _overrides.pop(key, None)
        _VERSION[0] += 1
    for fn in _listeners.get(key, ()):
        fn(get_property(key))


def describe() -> dict:
    return {k: get_property(k) for k in _REGISTRY}
