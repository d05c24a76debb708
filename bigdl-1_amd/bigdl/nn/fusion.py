"""Graph-level fusion for the device path (the reference's MKL-DNN fusion,
``DL/nn/mkldnn/Fusion.scala:32-332`` and ``mkldnn/Sequential.scala:195-267``; flags
``bigdl.fusion[.convbn|.bnrelu|.convsum]``).

The module tree is NOT rewritten (serialisation, ``parameters()`` order and user-visible structure
stay identical); matched modules get execution flags instead:

* conv → ReLU (``convrelu``, Sequential chains and Graph edges): the conv applies the ReLU in its
  epilogue; the ReLU module keeps only the gradient mask (taken from its input, which is now
  ReLU(conv) — positive exactly where the conv output was).
* conv → BN (``convbn``): the conv skips its bias add and the BN folds the bias in (batch
  normalisation is shift-invariant, so only the running mean sees it); the conv-bias gradient
  Σ_rows gx is produced by the BN backward's finalize kernel from its closed form.
* BN → ReLU (``bnrelu``): the ReLU becomes a pass-through; BN applies it in its apply kernel and
  masks the gradient in its backward apply kernel.
* ResNet block tail ``ConcatTable(branch…BN, shortcut) → CAddTable → ReLU`` (``convsum``): the
  shortcut runs first and the branch's last BN computes ReLU(BN(x) + shortcut) in one pass; in
  backward the same kernel emits both the branch gradient and the masked gradient for the shortcut.
* shortcut BN → block tail (``shortcutbn``): a ``conv → BN`` shortcut's BN only finalizes its
  statistics in training; the tail computes ReLU(BN(x) + x_s·a_s + b_s) from the shortcut conv's
  output and the shortcut BN's coefficients in the same pass.
* block tail → next block (``bnbwd``): the next block's first conv computes, in its dgrad
  epilogue, (dgrad + shortcut gradient) · [block output > 0] and the tail BN's Σg, Σg·(x − mean),
  so the tail BN backward is a single apply pass and the masked gradient IS the shortcut gradient.

Each fusion removes one full read+write pass over an activation tensor from HBM.
"""
from __future__ import annotations

from ..utils import config
from .containers import Sequential, ConcatTable
from .layers.activation import Threshold
from .layers.conv import SpatialConvolution
from .layers.normalization import BatchNormalization, SpatialBatchNormalization
from .layers.table_ops import CAddTable


def _is_relu(m):
    return isinstance(m, Threshold) and m.threshold == 0.0 and m.value == 0.0


from .layers.conv import SpatialShareConvolution  # noqa: E402

_PLAIN_CONVS = (SpatialConvolution, SpatialShareConvolution)


def _is_nchw_bn(m):
    return isinstance(m, BatchNormalization) and getattr(m, "dataFormat", "NCHW") == "NCHW"


def _relu_fusable_conv(m):
    return type(m) in _PLAIN_CONVS and m.format == "NCHW" and m._bias_folded_into is None


def _fuse_conv_relu(a, b):
    a._fused_relu = True
    b._passthrough = "mask"


def _fuse_graphs(model, convrelu):
    """conv → ReLU edges inside Graphs (Caffe/TF-loaded models are graphs): the ReLU must be the
    conv's only consumer."""
    from .graph import Graph
    for g in model.flattened_modules():
        if not isinstance(g, Graph) or not hasattr(g, "forward_order"):
            continue
        g._plans = None  # concat plans depend on the fusion state
        for n in g.forward_order:
            if (convrelu and _relu_fusable_conv(n.element) and len(n.next_nodes) == 1
                    and _is_relu(n.next_nodes[0].element) and len(n.next_nodes[0].prev_nodes) == 1
                    and not n.element._fused_relu):
                _fuse_conv_relu(n.element, n.next_nodes[0].element)


def _stackable(a, b):
    from .layers.recurrent import Recurrent, LSTM
    return (type(a) is Recurrent and type(b) is Recurrent and type(a.topology) is LSTM and type(b.topology) is LSTM
            and a.topology.p == 0 and b.topology.p == 0 and not a.maskZero and not b.maskZero
            and b.batchNormParams is None and a._stack_next is None and a._stack_prev is None
            and b._stack_next is None and b._stack_prev is None)


def _link_stack(a, b):
    a._stack_next = b
    b._stack_prev = a


def _fuse_lstm_stacks(model):
    """Two stacked Recurrent(LSTM) layers, the upper one's only input being the lower one's output
    (Sequential neighbours or a Graph edge): flag the pair for the layer-wavefront execution
    (nn/layers/recurrent.py ``_lstm2_forward``; the runtime re-checks shapes / dtypes and falls
    back to layer-by-layer execution otherwise)."""
    from .graph import Graph
    for s in model.flattened_modules():
        if isinstance(s, Sequential):
            mods = s.modules
            for i in range(len(mods) - 1):
                if _stackable(mods[i], mods[i + 1]):
                    _link_stack(mods[i], mods[i + 1])
        elif isinstance(s, Graph) and hasattr(s, "forward_order"):
            for n in s.forward_order:
                if len(n.next_nodes) != 1:
                    continue
                m = n.next_nodes[0]
                if len(m.prev_nodes) == 1 and _stackable(n.element, m.element):
                    _link_stack(n.element, m.element)


def fuse(model, convbn=None, bnrelu=None, convsum=None, bnbwd=None, convrelu=None):
    if not config.get_property("bigdl.fusion"):
        return model
    if getattr(model, "_fused", False):
        return model
    model._fused = True
    convrelu = config.get_property("bigdl.fusion.convrelu") if convrelu is None else convrelu
    convbn = config.get_property("bigdl.fusion.convbn") if convbn is None else convbn
    bnrelu = config.get_property("bigdl.fusion.bnrelu") if bnrelu is None else bnrelu
    convsum = config.get_property("bigdl.fusion.convsum") if convsum is None else convsum
    bnbwd = config.get_property("bigdl.fusion.bnbwd") if bnbwd is None else bnbwd
    tails, heads = [], []
    for s in model.flattened_modules():
        if not isinstance(s, Sequential):
            continue
        mods = s.modules
        for i in range(len(mods) - 1):
            a, b = mods[i], mods[i + 1]
            if convbn and isinstance(a, SpatialConvolution) and type(a) in (SpatialConvolution,) + tuple(
                    SpatialConvolution.__subclasses__()) and a.format == "NCHW" and a.withBias and _is_nchw_bn(b) \
                    and b._bias_producer is None:
                a._bias_folded_into = b
                b._bias_producer = a
            if convrelu and _relu_fusable_conv(a) and _is_relu(b) and not b._passthrough:
                _fuse_conv_relu(a, b)
            if bnrelu and _is_nchw_bn(a) and _is_relu(b):
                a._fused_relu = True
                b._passthrough = True
                c = mods[i + 2] if i + 2 < len(mods) else None
                if bnbwd and isinstance(c, SpatialConvolution) and c.format == "NCHW" and c.nGroup == 1:
                    c._bn_bwd_target = a
                    if type(c) in _PLAIN_CONVS:
                        a._pro_consumer = c  # fp32: its output may reach c deferred (bigdl.fp32.bnPrologue)
        if not convsum:
            continue
        for i in range(len(mods) - 1):
            ct, add = mods[i], mods[i + 1]
            if not (isinstance(ct, ConcatTable) and len(ct.modules) == 2 and isinstance(add, CAddTable)):
                continue
            br = ct.modules[0]
            if not (isinstance(br, Sequential) and br.modules and _is_nchw_bn(br.modules[-1])):
                continue
            bn = br.modules[-1]
            if bn._fused_relu:
                continue
            relu = mods[i + 2] if i + 2 < len(mods) and _is_relu(mods[i + 2]) else None
            ct._residual = (br, bn, ct.modules[1], relu is not None)
            sc = ct.modules[1]
            if (config.get_property("bigdl.fusion.shortcutbn") and isinstance(sc, Sequential) and len(sc.modules) >= 2
                    and _is_nchw_bn(sc.modules[-1]) and not sc.modules[-1]._fused_relu):
                sc.modules[-1]._defer_ok = True
            add._passthrough = True
            if relu is not None:
                relu._passthrough = True
                tails.append(bn)
            first = br.modules[0]
            if isinstance(first, SpatialConvolution) and len(br.modules) > 1:
                heads.append(first)
                # 1×1 strided shortcut conv: its input gradient (nonzero only on the stride grid)
                # reaches `first`'s dgrad epilogue as a strided residual, never zero-filled
                sc = ct.modules[1]
                sc0 = sc.modules[0] if isinstance(sc, Sequential) and sc.modules else None
                if (isinstance(sc0, SpatialConvolution) and type(sc0) in _PLAIN_CONVS and sc0.format == "NCHW"
                        and sc0.kernelW == 1 and sc0.kernelH == 1 and sc0.padW == 0 and sc0.padH == 0
                        and sc0.nGroup == 1 and (sc0.strideW > 1 or sc0.strideH > 1)):
                    sc0._lazy_strided_ok = True
    # block tail → next block: the first conv of a fused block (whose dgrad epilogue already sums
    # the shortcut gradient) also applies the previous tail's ReLU mask and produces that BN's
    # backward reductions; the match is made at backward time by tensor identity
    if bnbwd and tails:
        for h in heads:
            h._tail_candidates = tails
    _fuse_graphs(model, convrelu)
    if config.get_property("bigdl.fusion.lstmstack"):
        _fuse_lstm_stacks(model)
    return model


def mark_input_no_grad(model):
    """The optimizer discards the model's gradInput, so the first layer need not compute it: flag
    the conv(s) that consume the model input (first module of nested Sequentials / the input nodes
    of a Graph) to skip their backward-data pass.  For an RGB (C = 3) stem that pass is also the
    one shape the native dgrad does not cover.  Execution flag only, like :func:`fuse`."""
    from .graph import Graph
    todo, seen = [model], set()
    while todo:
        m = todo.pop()
        if id(m) in seen:
            continue
        seen.add(id(m))
        if isinstance(m, Sequential):
            if m.modules:
                todo.append(m.modules[0])
        elif isinstance(m, Graph) and hasattr(m, "forward_order"):
            for n in m.forward_order:
                if not n.prev_nodes:
                    todo.append(n.element)
        elif isinstance(m, SpatialConvolution):
            m._input_grad_needed = False
    return model


def unfuse(model):
    model._fused = False
    for m in model.flattened_modules():
        if hasattr(m, "_plans"):
            m._plans = None
        if hasattr(m, "_plan"):
            m._plan = None
        if isinstance(m, SpatialConvolution):
            m._bias_folded_into = None
            m._fused_relu = False
            m._bn_bwd_target = None
            m._tail_candidates = None
            m._input_grad_needed = True
            m._lazy_strided_ok = False
        if isinstance(m, BatchNormalization):
            m._bias_producer = None
            m._fused_relu = False
            m._defer_ok = False
            m._pro_consumer = None
            m._pending_stats = None
            m._pending_grad = None
        if isinstance(m, Threshold):
            m._passthrough = False
        if isinstance(m, ConcatTable):
            m._residual = None
        if isinstance(m, CAddTable):
            m._passthrough = False
    return model
