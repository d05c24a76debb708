"""Recurrent family: ``Cell``, ``LSTM``, ``LSTMPeephole``, ``GRU``, ``RnnCell``, ``ConvLSTMPeephole``
(2-D / 3-D), ``MultiRNNCell``, ``Recurrent``, ``BiRecurrent``, ``RecurrentDecoder``,
``TimeDistributed``.

Reference semantics: ``DL/nn/Recurrent.scala`` (preTopology run **once** over all steps at
:251-255, time loop :283-307, BPTT :327-400, ``maskZero`` :273-304), ``DL/nn/Cell.scala``
(hidden resize, ``includePreTopology``), ``DL/nn/LSTM.scala:124-187`` (gate order i, g, f, o),
``GRU.scala``, ``RNN.scala`` (``RnnCell``), ``LSTMPeephole.scala``, ``ConvLSTMPeephole.scala``,
``MultiRNNCell.scala``, ``BiRecurrent.scala``, ``RecurrentDecoder.scala``, ``TimeDistributed.scala``.

Design (MI355X-first, not the reference's clone-a-cell-per-step scheme):

* The input projection (``preTopology``, i2g) runs as ONE GEMM over all B·T rows.
* **LSTM fast path** (``p == 0``, default Tanh/Sigmoid): per step one h·Uᵀ GEMM (hipBLASLt) plus
  one fused pointwise HIP kernel (gate add + activations + cell update, writes h straight into
  the (B, T, H) output); BPTT runs per step one fused backward kernel plus one dgrad GEMM, and
  the recurrent weight gradient dU = Σ_t dgates_tᵀ·h_{t-1} is ONE (4H × B·T) · (B·T × H) GEMM
  after the loop instead of T small ones.
* Every other cell (GRU, RnnCell, peephole, ConvLSTM, MultiRNNCell, custom cells) declares a
  differentiable ``step(x, hidden, tape)`` on torch device ops; the time loop is recorded once
  and BPTT is a single autograd pass.  Parameters enter through a ``_Tape`` that hands out
  compute-dtype leaves, fires the owning modules' pre-forward hooks (the DistriOptimizer's
  all-gather wait) and, after backward, accumulates gradients with the module's scale and
  regulariser and fires grad-ready hooks (bucketed reduce-scatter launch).
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.nn.functional as F

from ... import ops
from ...utils.table import Table, T
from ..abstractnn import AbstractModule, AutogradModule, TensorModule
from ..containers import Container, Sequential
from .activation import Tanh, Sigmoid, ReLU, Threshold
from .conv import SpatialConvolution, same_padding, to_device_layout
from .dropout import Dropout
from .linear import Linear
from .math_ops import CMul
from .shape import Identity
from ...utils import acc_float


# ============================================================================ tape
class _Tape:
    """Parameter leaves + dropout masks for one recorded recurrence (see module docstring)."""

    def __init__(self, train: bool):
        self.train = train
        self.leaves = {}  # (id(m), name) -> (m, name, leaf)
        self.masks = {}

    def W(self, m: AbstractModule, name: str):
        key = (id(m), name)
        ent = self.leaves.get(key)
        if ent is None:
            for h in m._pre_forward_hooks:
                h(m)
            t = m.cw(name)
            if self.train:
                t = t.detach().requires_grad_(True)
            ent = (m, name, t)
            self.leaves[key] = ent
        return ent[2]

    def dropout(self, m: Dropout, x: torch.Tensor):
        """Dropout whose mask is sampled once per sequence and shared by all time steps
        (``Recurrent.share``: ``current.noise = noise; isResampling = false``)."""
        if not (self.train and m.train) or m.p <= 0:
            return x if m.scale or m.p <= 0 else x * (1 - m.p)
        key = id(m)
        mask = self.masks.get(key)
        if mask is None or mask.shape != x.shape:
            keep = 1.0 - m.p
            mask = (torch.rand(x.shape, device=x.device) < keep).to(x.dtype)
            if m.scale:
                mask = mask / keep
            self.masks[key] = mask
        return x * mask

    def apply(self, m, x):
        """Differentiable application of module ``m`` to ``x`` inside the tape."""
        if isinstance(m, Linear):
            w = self.W(m, "weight")
            b = self.W(m, "bias") if m.withBias else None
            return F.linear(x.to(w.dtype), w, None if b is None else b.to(w.dtype))
        if isinstance(m, SpatialConvolution):
            w = m._w4(self.W(m, "weight"))
            b = self.W(m, "bias") if m.withBias else None
            xx = x.to(w.dtype)
            pt, pb, pl, pr = m._pads(xx)
            if pt != pb or pl != pr:
                xx = F.pad(xx, (pl, pr, pt, pb))
                pad = (0, 0)
            else:
                pad = (pt, pl)
            return F.conv2d(xx, w, None if b is None else b.to(w.dtype), (m.strideH, m.strideW), pad,
                            (m.dilationH, m.dilationW), m.nGroup)
        if isinstance(m, Dropout):
            return self.dropout(m, x)
        if isinstance(m, Tanh):
            return torch.tanh(x)
        if isinstance(m, Sigmoid):
            return torch.sigmoid(x)
        if isinstance(m, Threshold):
            return torch.where(x > m.threshold, x, torch.full_like(x, m.value))
        if isinstance(m, Identity):
            return x
        if isinstance(m, AutogradModule):
            leaves = {w: self.W(m, w) for w, _ in m._param_slots}
            m._leaves = leaves
            try:
                return m._forward(x)
            finally:
                m._leaves = None
        if isinstance(m, Sequential):
            for sub in m.modules:
                x = self.apply(sub, x)
            return x
        raise TypeError(f"recurrent cell: module {type(m).__name__} is not usable inside a recurrent step")

    def param_leaves(self):
        return [e[2] for e in self.leaves.values()]

    def accumulate(self, grads, regularize: bool = True):
        """Add leaf gradients into the owning modules' grad slots; fire grad-ready hooks."""
        mods = {}
        for (m, name, _), g in zip(self.leaves.values(), grads):
            gname = dict(m._param_slots)[name]
            scale = m.scale_b if name == "bias" else m.scale_w
            if g is not None and scale != 0:
                gt = getattr(m, gname)
                gt.add_(g.to(gt.dtype).reshape(gt.shape), alpha=scale)
            reg = getattr(m, "bRegularizer" if name == "bias" else "wRegularizer", None)
            if regularize and reg is not None and scale != 0:
                reg.accRegularization(getattr(m, name), getattr(m, gname), scale)
            mods[id(m)] = m
        for m in mods.values():
            for h in m._grad_ready_hooks:
                h(m)


def _fire_pre_forward(mods):
    for m in mods:
        for h in m._pre_forward_hooks:
            h(m)


def _fire_grad_ready(mods):
    for m in mods:
        for h in m._grad_ready_hooks:
            h(m)


def _acc_recurrent_grad(m, DG, h0, out, U):
    """dU += Σ_t dg_tᵀ h_{t-1} as ONE GEMM over all B·T rows, then the module's grad-ready hooks."""
    B, Tn, H = out.shape
    if m.scale_w != 0:
        hprev = torch.cat([h0.unsqueeze(1), out[:, :-1]], 1) if Tn > 1 else h0.unsqueeze(1)
        ops.linear_backward(DG.reshape(B * Tn, 4 * H), hprev.reshape(B * Tn, H), U, False, m.gradWeight, None,
                            m.scale_w)
        if m.wRegularizer is not None:
            m.wRegularizer.accRegularization(m.weight, m.gradWeight, m.scale_w)
    _fire_grad_ready([m])


def _fused_rnn32_ok(H, *ts) -> bool:
    """fp32 device recurrence on the bf16x3 fused step (rnn_step.hip k_rnn_step<…, F32>)."""
    if not all(isinstance(t, torch.Tensor) for t in ts) or not ts[0].is_cuda:
        return False
    from ...ops import native_ops as NO
    return NO.rnn_fast32_ok(H, *ts)


def _fused_rnn_ok(H, *ts) -> bool:
    """Fused MFMA recurrent step applies: bf16 device rows, H % 8 == 0, native library loaded."""
    if not all(isinstance(t, torch.Tensor) for t in ts) or not ts[0].is_cuda:
        return False
    from ...ops import native_ops as NO
    return NO.rnn_fast_ok(H, *ts)


def _cdtype(t: torch.Tensor):
    if t.is_cuda:
        from ...utils.engine import Engine
        return Engine.compute_dtype()
    return torch.float64 if t.dtype == torch.float64 else torch.float32


def _state_dt(dtype):
    """Cell-state dtype: fp32 under bf16/fp32 compute, float64 for a float64 model."""
    return torch.float64 if dtype == torch.float64 else torch.float32


# ============================================================================ cells
class Cell(Container):
    """Abstract recurrent cell (``DL/nn/Cell.scala``).  ``hiddensShape`` lists the hidden
    state sizes (LSTM: [H, H] → hidden Table(h, c); GRU/RNN: [H] → hidden Tensor).

    Subclasses implement ``step(x, hidden: list, tape) -> (out, new_hidden: list)`` where ``x``
    is the step input AFTER the preTopology (i2g) projection.  Standalone use
    ``cell.forward(T(x, hidden))`` → ``T(out, hidden')`` is supported (``Cell.updateOutput``)."""

    def __init__(self, hiddens_shape, regularizers=None):
        super().__init__()
        self.hiddensShape = list(hiddens_shape)
        self.regularizers = regularizers
        self.preTopology: Optional[AbstractModule] = None
        self.includePreTopology = False

    # -- hidden state --------------------------------------------------------------------
    def hiddenSizeOfPreTopo(self):
        return self.hiddensShape[0]

    def init_hidden(self, batch, step_shape, device, dtype) -> List[torch.Tensor]:
        """Zero hidden state(s) of shape (batch, hiddensShape[i], *step_shape[1:])."""
        rest = list(step_shape[1:]) if step_shape else []
        return [torch.zeros([batch, h] + rest, device=device, dtype=dtype) for h in self.hiddensShape]

    def hidResize(self, hidden, batch_size, step_shape=None):
        hs = self.init_hidden(batch_size, step_shape or [self.hiddensShape[0]], "cpu", torch.float32)
        return self.pack_hidden(hs)

    def pack_hidden(self, hs: List[torch.Tensor]):
        if len(self.hiddensShape) == 1:
            return hs[0]
        return T(*hs)

    def unpack_hidden(self, hidden) -> List[torch.Tensor]:
        if isinstance(hidden, torch.Tensor):
            return [hidden]
        return [hidden[i + 1] for i in range(len(hidden))]

    # -- step ----------------------------------------------------------------------------
    def step(self, x, hidden, tape: _Tape):  # pragma: no cover - abstract
        raise NotImplementedError

    def step_full(self, x, hidden, tape: _Tape):
        """Step on the RAW input (applies the preTopology when ``includePreTopology``)."""
        if self.includePreTopology and self.preTopology is not None:
            x = tape.apply(self.preTopology, x)
        return self.step(x, hidden, tape)

    def _param_entries(self):
        out = []
        if self.includePreTopology and self.preTopology is not None:
            out.extend(self.preTopology._param_entries())
        out.extend(super()._param_entries())
        return out

    def _set_arena_recursive(self, arena):
        super()._set_arena_recursive(arena)
        if self.includePreTopology and self.preTopology is not None:
            self.preTopology._set_arena_recursive(arena)

    def children(self):
        ch = list(self.modules)
        if self.includePreTopology and self.preTopology is not None:
            ch = [self.preTopology] + ch
        return ch

    # -- standalone Table API (one step) ---------------------------------------------------
    def updateOutput(self, input):
        x, hidden = input[1], input[2]
        hs = self.unpack_hidden(hidden)
        tape = _Tape(self.train)
        if self.train:
            xl = x.detach().requires_grad_(x.is_floating_point())
            hl = [h.detach().requires_grad_(True) for h in hs]
            with torch.enable_grad():
                out, nh = self.step_full(xl, hl, tape)
            self._rec = (tape, xl, hl, out, nh)
            return T(out.detach(), self.pack_hidden([h.detach() for h in nh]))
        self._rec = None
        with torch.no_grad():
            out, nh = self.step_full(x, hs, tape)
        return T(out, self.pack_hidden(nh))

    def _cell_backward(self, input, gradOutput):
        rec = getattr(self, "_rec", None)
        if rec is None:
            self.updateOutput(input)
            rec = self._rec
        tape, xl, hl, out, nh = rec
        go = gradOutput[1]
        gh = self.unpack_hidden(gradOutput[2]) if 2 in gradOutput else [None] * len(nh)
        outs, gos = [out], [go]
        for h, g in zip(nh, gh):
            if g is not None and h.requires_grad:
                outs.append(h)
                gos.append(g)
        targets = ([xl] if xl.requires_grad else []) + hl + tape.param_leaves()
        grads = torch.autograd.grad(outs, targets, [g.to(o.dtype) for o, g in zip(outs, gos)], allow_unused=True)
        k = 0
        gx = None
        if xl.requires_grad:
            gx = grads[0]
            k = 1
        ghid = [torch.zeros_like(h) if g is None else g for h, g in zip(hl, grads[k:k + len(hl)])]
        self._pgrads = grads[k + len(hl):]
        self._rec = None
        return T(torch.zeros_like(xl) if gx is None else gx, self.pack_hidden(ghid)), tape

    def updateGradInput(self, input, gradOutput):
        gi, tape = self._cell_backward(input, gradOutput)
        self._pending_tape = tape
        return gi

    def accGradParameters(self, input, gradOutput):
        tape = getattr(self, "_pending_tape", None)
        if tape is None:
            _, tape = self._cell_backward(input, gradOutput)
        tape.accumulate(self._pgrads)
        self._pending_tape = None

    def regluarized(self, is_regularized: bool):
        """Kept for API parity (``Cell.regluarized``); the tape applies regularisers once per
        sequence, which is what the reference achieves by enabling them only on cell 1."""
        return self


def _is_default(act, cls):
    return act is None or type(act) is cls


class LSTM(Cell):
    """``DL/nn/LSTM.scala``: gates (i, g, f, o); ``p`` > 0 builds per-gate Linear layers with
    dropout (no preTopology), otherwise i2g is one Linear(input, 4H) preTopology and h2g one
    Linear(H, 4H, no bias)."""

    def __init__(self, input_size, hidden_size, p=0.0, activation=None, inner_activation=None,
                 wRegularizer=None, uRegularizer=None, bRegularizer=None, bigdl_type="float"):
        super().__init__([hidden_size, hidden_size], [wRegularizer, uRegularizer, bRegularizer])
        self.inputSize, self.hiddenSize, self.p = input_size, hidden_size, p
        self.activation = activation if activation is not None else Tanh()
        self.innerActivation = inner_activation if inner_activation is not None else Sigmoid()
        self.wRegularizer, self.uRegularizer, self.bRegularizer = wRegularizer, uRegularizer, bRegularizer
        H = hidden_size
        if p != 0:
            self.i2g = [Linear(input_size, H, wRegularizer=wRegularizer, bRegularizer=bRegularizer) for _ in range(4)]
            self.h2g = [Linear(H, H, wRegularizer=wRegularizer, bRegularizer=bRegularizer) for _ in range(4)]
            self.drops = [Dropout(p) for _ in range(8)]
            for m in self.i2g + self.h2g:
                self.add(m)
            self.preTopology = None
        else:
            self.h2g = Linear(H, 4 * H, with_bias=False, wRegularizer=uRegularizer)
            self.add(self.h2g)
            self.preTopology = Linear(input_size, 4 * H, wRegularizer=wRegularizer, bRegularizer=bRegularizer)

    def hiddenSizeOfPreTopo(self):
        return 4 * self.hiddenSize

    @property
    def fused(self) -> bool:
        return self.p == 0 and _is_default(self.activation, Tanh) and _is_default(self.innerActivation, Sigmoid)

    def step(self, x, hidden, tape):
        h, c = hidden
        H = self.hiddenSize
        if self.p != 0:
            i2g = torch.cat([tape.apply(l, tape.dropout(d, x)) for l, d in zip(self.i2g, self.drops[:4])], -1)
            h2g = torch.cat([tape.apply(l, tape.dropout(d, h)) for l, d in zip(self.h2g, self.drops[4:])], -1)
        else:
            i2g = x
            h2g = tape.apply(self.h2g, h)
        if self.fused:
            hn, cn = _LSTMCellFn.apply(i2g, h2g, c)
            return hn, [hn, cn]
        gates = acc_float(i2g) + acc_float(h2g)
        act, inner = self.activation, self.innerActivation
        i = tape.apply(inner, gates[:, :H])
        g = tape.apply(act, gates[:, H:2 * H])
        f = tape.apply(inner, gates[:, 2 * H:3 * H])
        o = tape.apply(inner, gates[:, 3 * H:])
        cn = i * g + f * acc_float(c)
        hn = (o * tape.apply(act, cn)).to(x.dtype)
        return hn, [hn, cn]

    def init_hidden(self, batch, step_shape, device, dtype):
        H = self.hiddenSize
        return [torch.zeros(batch, H, device=device, dtype=dtype), torch.zeros(batch, H, device=device,
                                                                               dtype=_state_dt(dtype))]

    def __repr__(self):
        return f"LSTM({self.inputSize}, {self.hiddenSize}, {self.p})"


class _LSTMCellFn(torch.autograd.Function):
    """Fused LSTM pointwise step as an autograd node (native HIP kernel on GPU)."""

    @staticmethod
    def forward(ctx, xg, hg, c_prev):
        h, c, act, tc = ops.lstm_cell_forward(xg, hg, c_prev)
        ctx.save_for_backward(act, tc, c_prev)
        return h, c

    @staticmethod
    def backward(ctx, gh, gc):
        act, tc, c_prev = ctx.saved_tensors
        if gh is None:
            gh = torch.zeros(act.shape[0], act.shape[1] // 4, device=act.device, dtype=act.dtype)
        dg, dc = ops.lstm_cell_backward(gh.contiguous(), None, gc, act, tc, c_prev)
        return dg, dg, dc.to(c_prev.dtype)


class LSTMPeephole(Cell):
    """``DL/nn/LSTMPeephole.scala``: i = σ(Wi x + Ui h + ci∘c), f = σ(Wf x + Uf h + cf∘c),
    g = tanh(Wg x + Ug h), c' = f∘c + i∘g, o = σ(Wo x + Uo h + co∘c'), h' = o∘tanh(c').
    preTopology Linear(input, 4H) with blocks (i, f, g, o)."""

    def __init__(self, input_size, hidden_size, p=0.0, wRegularizer=None, uRegularizer=None, bRegularizer=None,
                 bigdl_type="float"):
        super().__init__([hidden_size, hidden_size], [wRegularizer, uRegularizer, bRegularizer])
        self.inputSize, self.hiddenSize, self.p = input_size, hidden_size, p
        self.wRegularizer, self.uRegularizer, self.bRegularizer = wRegularizer, uRegularizer, bRegularizer
        H = hidden_size
        if p != 0:
            self.i2g = [Linear(input_size, H, wRegularizer=wRegularizer, bRegularizer=bRegularizer) for _ in range(4)]
            self.drops = [Dropout(p) for _ in range(8)]
            self.preTopology = None
        else:
            self.i2g = None
            self.preTopology = Linear(input_size, 4 * H, wRegularizer=wRegularizer, bRegularizer=bRegularizer)
        self.h2g = [Linear(H, H, with_bias=False, wRegularizer=uRegularizer) for _ in range(4)]
        self.peep = [CMul([H]) for _ in range(3)]  # input, forget, output
        for m in (self.i2g or []) + self.h2g + self.peep:
            self.add(m)

    def hiddenSizeOfPreTopo(self):
        return 4 * self.hiddenSize

    def init_hidden(self, batch, step_shape, device, dtype):
        H = self.hiddenSize
        return [torch.zeros(batch, H, device=device, dtype=dtype), torch.zeros(batch, H, device=device,
                                                                               dtype=_state_dt(dtype))]

    def step(self, x, hidden, tape):
        h, c = hidden
        H = self.hiddenSize
        if self.p != 0:
            xs = [acc_float(tape.apply(l, tape.dropout(d, x))) for l, d in zip(self.i2g, self.drops[:4])]
            hs = [tape.dropout(d, h) for d in self.drops[4:]]
        else:
            xf = acc_float(x)
            xs = [xf[:, k * H:(k + 1) * H] for k in range(4)]
            hs = [h] * 4
        u = [acc_float(tape.apply(l, hh)) for l, hh in zip(self.h2g, hs)]
        cf = acc_float(c)
        i = torch.sigmoid(xs[0] + u[0] + tape.apply(self.peep[0], cf))
        f = torch.sigmoid(xs[1] + u[1] + tape.apply(self.peep[1], cf))
        g = torch.tanh(xs[2] + u[2])
        cn = f * cf + i * g
        o = torch.sigmoid(xs[3] + u[3] + tape.apply(self.peep[2], cn))
        hn = (o * torch.tanh(cn)).to(x.dtype)
        return hn, [hn, cn]


class GRU(Cell):
    """``DL/nn/GRU.scala``: r = σ(x_r + U_r h), z = σ(x_z + U_z h), ĥ = tanh(x_h + U_h (h∘r)),
    h' = (1 − z)∘ĥ + z∘h.  preTopology Linear(input, 3H) with blocks (r, z, h)."""

    def __init__(self, input_size, output_size, p=0.0, activation=None, inner_activation=None,
                 wRegularizer=None, uRegularizer=None, bRegularizer=None, bigdl_type="float"):
        super().__init__([output_size], [wRegularizer, uRegularizer, bRegularizer])
        self.inputSize, self.outputSize, self.p = input_size, output_size, p
        self.activation = activation if activation is not None else Tanh()
        self.innerActivation = inner_activation if inner_activation is not None else Sigmoid()
        self.wRegularizer, self.uRegularizer, self.bRegularizer = wRegularizer, uRegularizer, bRegularizer
        H = output_size
        if p != 0:
            self.i2g = [Linear(input_size, H, wRegularizer=wRegularizer, bRegularizer=bRegularizer) for _ in range(3)]
            self.h2g = [Linear(H, H, with_bias=False, wRegularizer=wRegularizer) for _ in range(2)]
            self.drops = [Dropout(p) for _ in range(6)]
            self.preTopology = None
            mods = self.i2g[:2] + self.h2g + self.i2g[2:]
        else:
            self.i2g = None
            self.h2g = [Linear(H, 2 * H, with_bias=False, wRegularizer=uRegularizer)]
            self.preTopology = Linear(input_size, 3 * H, wRegularizer=wRegularizer, bRegularizer=bRegularizer)
            self.drops = [Dropout(p)]
            mods = list(self.h2g)
        self.u_h = Linear(H, H, with_bias=False, wRegularizer=uRegularizer)
        for m in mods + [self.u_h]:
            self.add(m)

    def hiddenSizeOfPreTopo(self):
        return 3 * self.outputSize

    def step(self, x, hidden, tape):
        (h,) = hidden
        H = self.outputSize
        if self.p != 0:
            xr = acc_float(tape.apply(self.i2g[0], tape.dropout(self.drops[0], x)))
            xz = acc_float(tape.apply(self.i2g[1], tape.dropout(self.drops[1], x)))
            ur = acc_float(tape.apply(self.h2g[0], tape.dropout(self.drops[2], h)))
            uz = acc_float(tape.apply(self.h2g[1], tape.dropout(self.drops[3], h)))
            xh = acc_float(tape.apply(self.i2g[2], tape.dropout(self.drops[4], x)))
            rz = torch.cat([xr + ur, xz + uz], -1)
            hd = self.drops[5]
        else:
            xf = acc_float(x)
            rz = xf[:, :2 * H] + acc_float(tape.apply(self.h2g[0], h))
            xh = xf[:, 2 * H:]
            hd = self.drops[0]
        r = tape.apply(self.innerActivation, rz[:, :H])
        z = tape.apply(self.innerActivation, rz[:, H:])
        hh = tape.apply(self.activation, xh + acc_float(tape.apply(self.u_h, tape.dropout(hd, (acc_float(h) * r).to(h.dtype)))))
        hn = ((1 - z) * hh + z * acc_float(h)).to(x.dtype)
        return hn, [hn]


class RnnCell(Cell):
    """``DL/nn/RNN.scala``: h' = act(W x + b_i + U h + b_h)."""

    SCALA_NAME = "RnnCell"

    def __init__(self, input_size=4, hidden_size=3, activation=None, isInputWithBias=True, isHiddenWithBias=True,
                 wRegularizer=None, uRegularizer=None, bRegularizer=None, bigdl_type="float"):
        super().__init__([hidden_size], [wRegularizer, uRegularizer, bRegularizer])
        self.inputSize, self.hiddenSize = input_size, hidden_size
        self.activation = activation if activation is not None else Tanh()
        self.isInputWithBias, self.isHiddenWithBias = isInputWithBias, isHiddenWithBias
        self.preTopology = Linear(input_size, hidden_size, with_bias=isInputWithBias, wRegularizer=wRegularizer,
                                  bRegularizer=bRegularizer)
        self.h2h = Linear(hidden_size, hidden_size, with_bias=isHiddenWithBias, wRegularizer=uRegularizer)
        self.add(self.h2h)

    def step(self, x, hidden, tape):
        (h,) = hidden
        hn = tape.apply(self.activation, acc_float(x) + acc_float(tape.apply(self.h2h, h))).to(x.dtype)
        return hn, [hn]


RNN = RnnCell


class ConvLSTMPeephole(Cell):
    """``DL/nn/ConvLSTMPeephole.scala``: convolutional LSTM over (B, T, C, H, W); each gate is
    conv_i(x) (with bias) + conv_h(h) (no bias) [+ peephole CMul(1, C, 1, 1)∘c]."""

    _conv = SpatialConvolution

    def __init__(self, input_size, output_size, kernel_i, kernel_c, stride=1, padding=-1, activation=None,
                 inner_activation=None, wRegularizer=None, uRegularizer=None, bRegularizer=None, cRegularizer=None,
                 with_peephole=True, bigdl_type="float"):
        super().__init__([output_size, output_size], [wRegularizer, uRegularizer, bRegularizer, cRegularizer])
        self.inputSize, self.outputSize = input_size, output_size
        self.kernelI, self.kernelC, self.stride, self.padding = kernel_i, kernel_c, stride, padding
        self.activation = activation if activation is not None else Tanh()
        self.innerActivation = inner_activation if inner_activation is not None else Sigmoid()
        self.withPeephole = with_peephole
        self.preTopology = None
        self.gx = [self._mk(input_size, kernel_i, True, wRegularizer, bRegularizer) for _ in range(4)]  # i f o h
        self.gh = [self._mk(output_size, kernel_c, False, uRegularizer, None) for _ in range(4)]
        self.peep = [CMul(self._peep_shape(), cRegularizer) for _ in range(3)] if with_peephole else []
        for m in self.gx + self.gh + self.peep:
            self.add(m)

    def _peep_shape(self):
        return [1, self.outputSize, 1, 1]

    def _mk(self, cin, k, bias, wreg, breg):
        return SpatialConvolution(cin, self.outputSize, k, k, self.stride, self.stride, self.padding, self.padding,
                                  wRegularizer=wreg, bRegularizer=breg, with_bias=bias)

    def init_hidden(self, batch, step_shape, device, dtype):
        rest = list(step_shape[1:])
        return [torch.zeros([batch, self.outputSize] + rest, device=device, dtype=dtype),
                torch.zeros([batch, self.outputSize] + rest, device=device, dtype=_state_dt(dtype))]

    def step(self, x, hidden, tape):
        h, c = hidden
        cf = acc_float(c)
        gate = [acc_float(tape.apply(a, x)) + acc_float(tape.apply(b, h)) for a, b in zip(self.gx, self.gh)]
        inner, act = self.innerActivation, self.activation
        if self.withPeephole:
            i = tape.apply(inner, gate[0] + tape.apply(self.peep[0], cf))
            f = tape.apply(inner, gate[1] + tape.apply(self.peep[1], cf))
        else:
            i = tape.apply(inner, gate[0])
            f = tape.apply(inner, gate[1])
        g = tape.apply(act, gate[3])
        cn = f * cf + i * g
        o = tape.apply(inner, gate[2] + (tape.apply(self.peep[2], cn) if self.withPeephole else 0))
        hn = (o * tape.apply(act, cn)).to(x.dtype)
        return hn, [hn, cn]


class ConvLSTMPeephole3D(ConvLSTMPeephole):
    """``DL/nn/ConvLSTMPeephole3D.scala``: the same cell over (B, T, C, D, H, W)."""

    def _peep_shape(self):
        return [1, self.outputSize, 1, 1, 1]

    def _mk(self, cin, k, bias, wreg, breg):
        from .conv import VolumetricConvolution
        p = self.padding if self.padding >= 0 else (k - 1) // 2
        return VolumetricConvolution(cin, self.outputSize, k, k, k, self.stride, self.stride, self.stride, p, p, p,
                                     with_bias=bias, wRegularizer=wreg, bRegularizer=breg)


class MultiRNNCell(Cell):
    """``DL/nn/MultiRNNCell.scala``: a stack of cells run as one cell; each inner cell applies
    its own preTopology (``includePreTopology = true``).  Hidden = Table of the inner hiddens."""

    def __init__(self, cells, bigdl_type="float"):
        super().__init__(cells[-1].hiddensShape)
        self.cells = list(cells)
        for c in self.cells:
            if c.preTopology is not None:
                c.includePreTopology = True
            self.add(c)

    def init_hidden(self, batch, step_shape, device, dtype):
        return [c.init_hidden(batch, step_shape, device, dtype) for c in self.cells]

    def pack_hidden(self, hs):
        return T(*[c.pack_hidden(h) for c, h in zip(self.cells, hs)])

    def unpack_hidden(self, hidden):
        return [c.unpack_hidden(hidden[i + 1]) for i, c in enumerate(self.cells)]

    def step(self, x, hidden, tape):
        new = []
        for c, h in zip(self.cells, hidden):
            x, nh = c.step_full(x, h, tape)
            new.append(nh)
        return x, new


def _flat_hidden(hs):
    out = []
    for h in hs:
        if isinstance(h, (list, tuple)):
            out.extend(_flat_hidden(h))
        else:
            out.append(h)
    return out


def _rebuild_hidden(template, flat, pos=0):
    out = []
    for h in template:
        if isinstance(h, (list, tuple)):
            sub, pos = _rebuild_hidden(h, flat, pos)
            out.append(sub)
        else:
            out.append(flat[pos])
            pos += 1
    return out, pos


# ============================================================================ TimeDistributed
class TimeDistributed(TensorModule):
    """Apply ``layer`` to every time step by folding (B, T) into one batch dim
    (``DL/nn/TimeDistributed.scala``); ``maskZero`` zeroes outputs of all-zero input steps."""

    def __init__(self, layer, maskZero=False, bigdl_type="float"):
        super().__init__()
        self.layer = layer
        self.maskZero = maskZero

    def children(self):
        return [self.layer]

    def _param_entries(self):
        return self.layer._param_entries()

    def parameters(self):
        return self.layer.parameters()

    def _set_arena_recursive(self, arena):
        self._arena = arena
        self.layer._set_arena_recursive(arena)

    def zeroGradParameters(self):
        self.layer.zeroGradParameters()

    def getParametersTable(self):
        return self.layer.getParametersTable()

    def _fold(self, t):
        return t.reshape((t.shape[0] * t.shape[1],) + tuple(t.shape[2:]))

    def _mask(self, input):
        return input.reshape(input.shape[0], input.shape[1], -1).abs().amax(-1) != 0

    def updateOutput(self, input):
        if input.dim() < 3:
            raise ValueError(f"TimeDistributed: input should be at least a 3D Tensor, got {input.dim()}D")
        B, Tn = input.shape[0], input.shape[1]
        y = self.layer.forward(self._fold(input.contiguous()))
        y = y.reshape((B, Tn) + tuple(y.shape[1:]))
        if self.maskZero:
            m = self._mask(input)
            y = y * m.reshape(B, Tn, *([1] * (y.dim() - 2))).to(y.dtype)
        return y

    def _gy(self, input, gradOutput):
        g = self._fold(gradOutput.contiguous())
        return g

    def updateGradInput(self, input, gradOutput):
        gi = self.layer.updateGradInput(self._fold(input.contiguous()), self._gy(input, gradOutput))
        return gi.reshape(input.shape)

    def accGradParameters(self, input, gradOutput):
        self.layer.accGradParameters(self._fold(input.contiguous()), self._gy(input, gradOutput))

    def backward(self, input, gradOutput):
        gi = self.layer.backward(self._fold(input.contiguous()), self._gy(input, gradOutput)).reshape(input.shape)
        if self.maskZero:
            m = self._mask(input)
            gi = gi * m.reshape(input.shape[0], input.shape[1], *([1] * (gi.dim() - 2))).to(gi.dtype)
        self.gradInput = gi
        for h in self._grad_ready_hooks:
            h(self)
        return gi

    def __repr__(self):
        return f"TimeDistributed({self.layer!r})"


class BatchNormParams:
    """``Recurrent(batchNormParams)``: BN applied to the preTopology output."""

    def __init__(self, eps=1e-5, momentum=0.1, affine=True, initWeight=None, initBias=None, initGradWeight=None,
                 initGradBias=None):
        self.eps, self.momentum, self.affine = eps, momentum, affine
        self.initWeight, self.initBias = initWeight, initBias
        self.initGradWeight, self.initGradBias = initGradWeight, initGradBias


# ============================================================================ Recurrent
class Recurrent(Container):
    """Runs a ``Cell`` over the time dimension of a (B, T, ...) input (``DL/nn/Recurrent.scala``).

    ``modules`` = [TimeDistributed(preTopology) (if any), cell], so ``parameters()`` order is
    (i2g weight, i2g bias, cell weights...) as in the reference."""

    def __init__(self, batchNormParams=None, maskZero=False, bigdl_type="float"):
        super().__init__()
        self.batchNormParams = batchNormParams
        self.maskZero = maskZero
        self.topology: Optional[Cell] = None
        self.preTopology = None
        self._init_hidden_state = None
        self._grad_hidden_state = None
        self._rec = None

    def add(self, module):
        if not isinstance(module, Cell):
            raise ValueError("Recurrent: added module should be Cell type!")
        if isinstance(module, MultiRNNCell):
            raise ValueError("Recurrent: added module cannot be MultiRNNCell, use Sequential().add(Recurrent(cell))"
                             ".add(Recurrent(cell))... instead!")
        self.topology = module
        pre = TimeDistributed(module.preTopology, maskZero=self.maskZero) if module.preTopology is not None else None
        if self.batchNormParams is not None:
            if pre is None:
                raise ValueError(f"{type(module).__name__} does not support BatchNormalization; add a preTopology")
            from .normalization import BatchNormalization
            bp = self.batchNormParams
            bn = BatchNormalization(module.hiddenSizeOfPreTopo(), bp.eps, bp.momentum, bp.affine, bp.initWeight,
                                    bp.initBias, bp.initGradWeight, bp.initGradBias)
            pre = Sequential().add(pre).add(TimeDistributed(bn))
        self.preTopology = pre
        self.modules = ([pre] if pre is not None else []) + [module]
        return self

    def getCell(self):
        return self.topology

    def setHiddenState(self, hidden_state):
        self._init_hidden_state = hidden_state
        return self

    def getHiddenState(self):
        if self._last_hidden is None:
            raise RuntimeError("getHiddenState need to be called after updateOutput")
        return self._last_hidden

    def getGradHiddenState(self):
        return self._grad_hidden_state

    _last_hidden = None

    # -- forward -------------------------------------------------------------------------
    def _h0(self, B, step_shape, device, dtype):
        cell = self.topology
        if self._init_hidden_state is not None:
            hs = cell.unpack_hidden(self._init_hidden_state)
            return [h.to(device) if isinstance(h, torch.Tensor) else [x.to(device) for x in h] for h in hs]
        return cell.init_hidden(B, step_shape, device, dtype)

    #: use the explicit BPTT path for plain LSTM cells (False → generic autograd path; tests
    #: compare the two)
    fast_lstm = True

    def _use_fast_lstm(self):
        c = self.topology
        return self.fast_lstm and type(c) is LSTM and c.fused and not self.maskZero

    def _use_fast_gru(self, x2):
        c = self.topology
        if not (self.fast_lstm and type(c) is GRU and c.p == 0 and not self.maskZero and x2.dim() == 3):
            return False
        if not (_is_default(c.activation, Tanh) and _is_default(c.innerActivation, Sigmoid)):
            return False
        w1, w2 = c.h2g[0].cw("weight"), c.u_h.cw("weight")
        return _fused_rnn_ok(c.outputSize, x2, w1, w2) or _fused_rnn32_ok(c.outputSize, x2, w1, w2)

    # -- stacked-LSTM fusion (bigdl.nn.fusion ``lstmstack``) ----------------------------------
    #: lower layer: the next Recurrent(LSTM) whose only input is this layer's output; upper layer:
    #: the layer feeding it.  The pair then runs on the layer wavefront (rnn_step.hip
    #: bigdl_lstm2_seq_*): the upper layer's input projection h·W + b becomes a second reduction
    #: segment of its recurrent step and both layers advance in the same launches.
    _stack_next = None
    _stack_prev = None
    #: upper layer: (lower output, upper output) of the fused forward, consumed by its own forward
    _stack_fwd = None
    #: lower layer: its gate gradients, produced by the upper layer's fused backward
    _stack_gx2 = None

    def _stack_ready(self, x2):
        nxt = self._stack_next
        if nxt is None or not (self._use_fast_lstm() and nxt._use_fast_lstm()) or bool(self.train) != bool(nxt.train):
            return False
        pre = nxt.preTopology
        if not (isinstance(pre, TimeDistributed) and type(pre.layer) is Linear and not pre.maskZero):
            return False
        H0, H1 = self.topology.hiddenSize, nxt.topology.hiddenSize
        W1 = pre.layer.cw("weight")
        return (x2.dim() == 3 and tuple(W1.shape) == (4 * H1, H0) and H1 % 8 == 0 and nxt._init_hidden_state is None
                and self._init_hidden_state is None
                and _fused_rnn_ok(H0, x2, self.topology.h2g.cw("weight"), W1, nxt.topology.h2g.cw("weight")))

    def updateOutput(self, input):
        sf = self._stack_fwd
        if sf is not None:
            self._stack_fwd = None
            if sf[0] is input:  # computed by the lower layer's fused forward for exactly this input
                return sf[1]
        if input.dim() not in (3, 5, 6):
            raise ValueError(f"Recurrent: input should be a 3D/5D/6D Tensor, e.g [batch, times, nDim], "
                             f"current input.dim = {input.dim()}")
        x2 = self.preTopology.forward(input) if self.preTopology is not None else input
        if x2.is_cuda and x2.dtype != _cdtype(x2) and x2.is_floating_point():
            x2 = x2.to(_cdtype(x2))
        self._x2 = x2
        if self._use_fast_lstm():
            if self._stack_next is not None and self._stack_ready(x2):
                return self._lstm2_forward(x2)
            return self._lstm_forward(x2)
        if self._use_fast_gru(x2):
            return self._gru_forward(x2)
        return self._generic_forward(input, x2)

    def _lstm_forward(self, x2):
        cell: LSTM = self.topology
        B, Tn, G = x2.shape
        H = cell.hiddenSize
        _fire_pre_forward([cell.h2g])
        U = cell.h2g.cw("weight")  # (4H, H)
        h0, c0 = self._h0(B, [H], x2.device, x2.dtype)
        h0 = h0.to(x2.dtype)
        c0 = acc_float(c0)
        out = torch.empty(B, Tn, H, device=x2.device, dtype=x2.dtype)
        train = self.train
        if train:
            acts = torch.empty(Tn, B, G, device=x2.device, dtype=_state_dt(x2.dtype))
            tcs = torch.empty(Tn, B, H, device=x2.device, dtype=_state_dt(x2.dtype))
            cs = torch.empty(Tn, B, H, device=x2.device, dtype=_state_dt(x2.dtype))
        if _fused_rnn_ok(H, x2, U):
            # one launch per step (h·Uᵀ on MFMA + the cell update in the GEMM epilogue, rnn_step.hip),
            # the time loop itself in C++: one host call for the whole sequence
            from ...ops import native_ops as NO
            x2 = x2.contiguous()
            h0 = h0.contiguous()
            c0 = c0.contiguous()
            cbuf = None if train else torch.empty(2, B, H, device=x2.device, dtype=_state_dt(x2.dtype))
            NO.lstm_seq_forward(x2, h0, c0, U, out, cs if train else None, acts if train else None,
                                tcs if train else None, cbuf)
            h = out[:, Tn - 1]
            c = cs[Tn - 1] if train else cbuf[(Tn - 1) % 2]
        elif _fused_rnn32_ok(H, x2, U):
            # fp32: the same one-launch-per-step loop with bf16x3 recurrent products
            from ...ops import native_ops as NO
            x2 = x2.contiguous()
            h0 = h0.contiguous()
            c0 = c0.contiguous()
            cbuf = None if train else torch.empty(2, B, H, device=x2.device, dtype=torch.float32)
            NO.lstm_seq_forward32(x2, h0, c0, U.contiguous(), out, cs if train else None, acts if train else None,
                                  tcs if train else None, cbuf)
            h = out[:, Tn - 1]
            c = cs[Tn - 1] if train else cbuf[(Tn - 1) % 2]
        else:
            h, c = h0, c0
            for t in range(Tn):
                hg = torch.mm(h, U.t())
                if train:
                    h, c, _, _ = ops.lstm_cell_forward(x2[:, t], hg, c, h_out=out[:, t], c_out=cs[t],
                                                       act_out=acts[t], tc_out=tcs[t])
                else:
                    h, c, _, _ = ops.lstm_cell_forward(x2[:, t], hg, c, h_out=out[:, t])
        self._last_hidden = T(h, c)
        self._rec = ("lstm", h0, c0, out, acts, tcs, cs) if train else None
        return out

    def _lstm2_forward(self, x2):
        """This layer and ``_stack_next`` in one wavefront sequence (T + 1 launches); returns this
        layer's output and parks the upper layer's for its own forward call."""
        from ...ops import native_ops as NO
        nxt = self._stack_next
        c0m, c1m = self.topology, nxt.topology
        lin = nxt.preTopology.layer
        B, Tn, _ = x2.shape
        H0, H1 = c0m.hiddenSize, c1m.hiddenSize
        _fire_pre_forward([c0m.h2g, lin, c1m.h2g])
        U0, U1, W1 = c0m.h2g.cw("weight"), c1m.h2g.cw("weight"), lin.cw("weight")
        dev, dt = x2.device, x2.dtype
        if lin.withBias:
            b1 = lin.bias.detach().to(torch.float32).contiguous()
        else:
            b1 = torch.zeros(4 * H1, dtype=torch.float32, device=dev)
        h00, c00 = self._h0(B, [H0], dev, dt)
        h01, c01 = nxt._h0(B, [H1], dev, dt)
        h00, h01 = h00.to(dt).contiguous(), h01.to(dt).contiguous()
        c00, c01 = acc_float(c00).contiguous(), acc_float(c01).contiguous()
        out0 = torch.empty(B, Tn, H0, device=dev, dtype=dt)
        out1 = torch.empty(B, Tn, H1, device=dev, dtype=dt)
        sdt = _state_dt(dt)
        train = self.train
        if train:
            sv0 = [torch.empty(Tn, B, 4 * H0, device=dev, dtype=sdt), torch.empty(Tn, B, H0, device=dev, dtype=sdt),
                   torch.empty(Tn, B, H0, device=dev, dtype=sdt)]  # acts, tcs, cs
            sv1 = [torch.empty(Tn, B, 4 * H1, device=dev, dtype=sdt), torch.empty(Tn, B, H1, device=dev, dtype=sdt),
                   torch.empty(Tn, B, H1, device=dev, dtype=sdt)]
            cb0 = cb1 = None
        else:
            sv0 = sv1 = [None, None, None]
            cb0 = torch.empty(2, B, H0, device=dev, dtype=sdt)
            cb1 = torch.empty(2, B, H1, device=dev, dtype=sdt)
        x2 = x2.contiguous()
        NO.lstm2_seq_forward(x2, h00, c00, U0, out0, sv0[2], sv0[0], sv0[1], cb0, b1, W1, h01, c01, U1, out1, sv1[2],
                             sv1[0], sv1[1], cb1)
        last = Tn - 1
        self._last_hidden = T(out0[:, last], sv0[2][last] if train else cb0[last % 2])
        nxt._last_hidden = T(out1[:, last], sv1[2][last] if train else cb1[last % 2])
        self._rec = ("lstm", h00, c00, out0, sv0[0], sv0[1], sv0[2]) if train else None
        nxt._x2 = None
        nxt._rec = ("lstm2", h01, c01, out1, sv1[0], sv1[1], sv1[2], self, out0) if train else None
        nxt._stack_fwd = (out0, out1)
        return out0

    def _gru_forward(self, x2):
        """GRU time loop on two fused launches per step (rnn_step.hip cells 2 and 3)."""
        from ...ops import native_ops as NO
        cell: GRU = self.topology
        B, Tn, _ = x2.shape
        H = cell.outputSize
        urz, uh = cell.h2g[0], cell.u_h
        _fire_pre_forward([urz, uh])
        Urz, Uh = urz.cw("weight"), uh.cw("weight")
        (h0,) = self._h0(B, [H], x2.device, x2.dtype)
        h0 = h0.to(x2.dtype).contiguous()
        dev = x2.device
        out = torch.empty(B, Tn, H, device=dev, dtype=x2.dtype)
        train = self.train
        nS = Tn if train else 1
        R = torch.empty(nS, B, H, device=dev, dtype=torch.float32)
        Z = torch.empty(nS, B, H, device=dev, dtype=torch.float32)
        Nn = torch.empty(nS, B, H, device=dev, dtype=torch.float32) if train else None
        RH = torch.empty(B, Tn if train else 1, H, device=dev, dtype=x2.dtype)
        if x2.dtype == torch.float32:
            NO.gru_seq_forward32(x2.contiguous(), h0, Urz.contiguous(), Uh.contiguous(), out, R, Z, Nn, RH, train)
        else:
            NO.gru_seq_forward(x2.contiguous(), h0, Urz, Uh, out, R, Z, Nn, RH, train)
        self._last_hidden = out[:, Tn - 1]
        self._rec = ("gru", h0, out, R, Z, Nn, RH) if train else None
        return out

    def _generic_forward(self, input, x2):
        cell = self.topology
        B, Tn = x2.shape[0], x2.shape[1]
        step_shape = [cell.hiddensShape[0]] + list(x2.shape[3:])
        hdt = x2.dtype if x2.is_floating_point() else torch.float32
        h0 = self._h0(B, step_shape, x2.device, hdt)
        train = self.train
        tape = _Tape(train)
        mask = None
        if self.maskZero:
            if input.dim() != 3:
                raise ValueError("If maskZero set to true, input should be a 3D Tensor, e.g [batch, times, nDim]")
            mask = input.abs().amax(-1) != 0  # (B, T)
        ctx = torch.enable_grad() if train else torch.no_grad()
        with ctx:
            xl = x2.detach().requires_grad_(train and x2.is_floating_point())
            flat0 = [h.detach().requires_grad_(train) for h in _flat_hidden(h0)]
            hid, _ = _rebuild_hidden(h0, flat0)
            outs = []
            for t in range(Tn):
                o, nh = cell.step(xl[:, t], hid, tape)
                if mask is not None:
                    m = mask[:, t]
                    fo, fn = _flat_hidden([o]), _flat_hidden(nh)
                    fp = _flat_hidden(hid)
                    mm = [m.reshape(-1, *([1] * (v.dim() - 1))) for v in fn]
                    fn = [torch.where(k, v, p.to(v.dtype)) for k, v, p in zip(mm, fn, fp)]
                    nh, _ = _rebuild_hidden(nh, fn)
                    o = o * m.reshape(-1, *([1] * (o.dim() - 1))).to(o.dtype)
                outs.append(o)
                hid = nh
            out = torch.stack(outs, 1)
        self._last_hidden = cell.pack_hidden(_rebuild_hidden(hid, [v.detach() for v in _flat_hidden(hid)])[0])
        self._rec = ("generic", tape, xl, flat0, out) if train else None
        return out.detach()

    # -- backward ------------------------------------------------------------------------
    def _bptt(self, gradOutput):
        """Run BPTT once; returns the gradient w.r.t. the preTopology output (x2)."""
        g = self._stack_gx2
        if g is not None:  # produced by the upper layer's fused backward
            self._stack_gx2 = None
            return g
        rec = self._rec
        if rec is None:
            raise RuntimeError("Recurrent: backward called without a training-mode forward")
        if rec[0] == "lstm":
            return self._lstm_backward(gradOutput)
        if rec[0] == "lstm2":
            return self._lstm2_backward(gradOutput)
        if rec[0] == "gru":
            return self._gru_backward(gradOutput)
        _, tape, xl, flat0, out = rec
        targets = ([xl] if xl.requires_grad else []) + flat0 + tape.param_leaves()
        grads = torch.autograd.grad([out], targets, [gradOutput.to(out.dtype)], allow_unused=True)
        k = 1 if xl.requires_grad else 0
        gx = grads[0] if k else None
        gh = grads[k:k + len(flat0)]
        self._grad_hidden_state = [g for g in gh]
        tape.accumulate(grads[k + len(flat0):])
        self._rec = None
        return torch.zeros_like(xl) if gx is None else gx

    def _lstm_backward(self, gradOutput):
        _, h0, c0, out, acts, tcs, cs = self._rec
        cell: LSTM = self.topology
        U = cell.h2g.cw("weight")
        B, Tn, H = out.shape
        gy = gradOutput.to(out.dtype)
        if not gy.is_contiguous():
            gy = gy.contiguous()
        DG = torch.empty(B, Tn, 4 * H, device=out.device, dtype=out.dtype)
        if _fused_rnn_ok(H, out, U, gy):
            # one launch per step: dh = gy_t + dg_{t+1}·U on MFMA, cell backward in the epilogue
            from ...ops import native_ops as NO
            Ut = NO.transpose_bf16(U)  # (H, 4H)
            gc = torch.empty(B, H, device=out.device, dtype=_state_dt(out.dtype))
            NO.lstm_seq_backward(gy, Ut, acts, tcs, cs, c0, DG, gc)
            gh_rec = NO.gemm(DG[:, 0], Ut)
        elif _fused_rnn32_ok(H, out, U, gy):
            from ...ops import native_ops as NO
            Ut = U.t().contiguous()  # (H, 4H) fp32
            gc = torch.empty(B, H, device=out.device, dtype=torch.float32)
            NO.lstm_seq_backward32(gy, Ut, acts, tcs, cs, c0.contiguous(), DG, gc)
            gh_rec = DG[:, 0] @ U  # the initial hidden state's gradient (one product per sequence)
        else:
            gh_rec, gc = None, None
            for t in range(Tn - 1, -1, -1):
                c_prev = cs[t - 1] if t > 0 else c0
                dg, gc = ops.lstm_cell_backward(gy[:, t], gh_rec, gc, acts[t], tcs[t], c_prev, dg_out=DG[:, t])
                gh_rec = torch.mm(dg, U)
        self._grad_hidden_state = [gh_rec, gc]
        _acc_recurrent_grad(cell.h2g, DG, h0, out, U)
        self._rec = None
        return DG

    def _lstm2_backward(self, gradOutput):
        """Upper layer of a fused stack: BPTT of BOTH layers on the wavefront (T + 1 launches);
        accumulates both recurrent weights, returns this layer's gate gradients (for its input
        projection's weight gradient) and parks the lower layer's for its backward."""
        from ...ops import native_ops as NO
        _, h01, c01, out1, acts1, tcs1, cs1, low, out0 = self._rec
        _, h00, c00, _, acts0, tcs0, cs0 = low._rec
        c1m, c0m = self.topology, low.topology
        U1, U0, W1 = c1m.h2g.cw("weight"), c0m.h2g.cw("weight"), self.preTopology.layer.cw("weight")
        B, Tn, H1 = out1.shape
        H0 = out0.shape[2]
        dev, dt = out1.device, out1.dtype
        gy = gradOutput.to(dt)
        if not gy.is_contiguous():
            gy = gy.contiguous()
        DG1 = torch.empty(B, Tn, 4 * H1, device=dev, dtype=dt)
        DG0 = torch.empty(B, Tn, 4 * H0, device=dev, dtype=dt)
        U1t, U0t, W1t = NO.transpose_bf16(U1), NO.transpose_bf16(U0), NO.transpose_bf16(W1)
        gc1 = torch.empty(B, H1, device=dev, dtype=_state_dt(dt))
        gc0 = torch.empty(B, H0, device=dev, dtype=_state_dt(dt))
        NO.lstm2_seq_backward(gy, U1t, acts1, tcs1, cs1, c01, DG1, gc1, U0t, W1t, acts0, tcs0, cs0, c00, DG0, gc0)
        self._grad_hidden_state = [NO.gemm(DG1[:, 0], U1t), gc1]
        low._grad_hidden_state = [NO.gemm(DG0[:, 0], U0t), gc0]
        _acc_recurrent_grad(c1m.h2g, DG1, h01, out1, U1)
        _acc_recurrent_grad(c0m.h2g, DG0, h00, out0, U0)
        low._stack_gx2 = DG0
        low._rec = None
        self._rec = None
        return DG1

    def _gru_backward(self, gradOutput):
        from ...ops import native_ops as NO
        _, h0, out, R, Z, Nn, RH = self._rec
        cell: GRU = self.topology
        urz, uh = cell.h2g[0], cell.u_h
        Urz, Uh = urz.cw("weight"), uh.cw("weight")
        B, Tn, H = out.shape
        gy = gradOutput.to(out.dtype)
        if not gy.is_contiguous():
            gy = gy.contiguous()
        dev = out.device
        DG = torch.empty(B, Tn, 3 * H, device=dev, dtype=out.dtype)  # (da_r, da_z, da_n) per step
        carry = torch.zeros(B, H, device=dev, dtype=torch.float32)
        if out.dtype == torch.float32:
            Urz_t, Uh_t = Urz.t().contiguous(), Uh.t().contiguous()
            NO.gru_seq_backward32(gy, Urz_t, Uh_t, R, Z, Nn, out, h0, DG, carry)
            carry.add_(DG[:, 0, :2 * H] @ Urz)  # dh0 = carry + da_rz_0 · U_rz
        else:
            Urz_t, Uh_t = NO.transpose_bf16(Urz), NO.transpose_bf16(Uh)  # (H, 2H), (H, H)
            NO.gru_seq_backward(gy, Urz_t, Uh_t, R, Z, Nn, out, h0, DG, carry)
            NO.gemm(DG[:, 0, :2 * H], Urz_t, out=carry, beta=1.0)  # dh0 = carry + da_rz_0 · U_rz
        self._grad_hidden_state = [carry]
        hprev = torch.cat([h0.unsqueeze(1), out[:, :-1]], 1) if Tn > 1 else h0.unsqueeze(1)
        if urz.scale_w != 0:
            ops.linear_backward(DG[:, :, :2 * H].reshape(B * Tn, 2 * H), hprev.reshape(B * Tn, H), Urz, False,
                                urz.gradWeight, None, urz.scale_w)
            if urz.wRegularizer is not None:
                urz.wRegularizer.accRegularization(urz.weight, urz.gradWeight, urz.scale_w)
        if uh.scale_w != 0:
            ops.linear_backward(DG[:, :, 2 * H:].reshape(B * Tn, H), RH.reshape(B * Tn, H), Uh, False,
                                uh.gradWeight, None, uh.scale_w)
            if uh.wRegularizer is not None:
                uh.wRegularizer.accRegularization(uh.weight, uh.gradWeight, uh.scale_w)
        _fire_grad_ready([urz, uh])
        self._rec = None
        return DG

    def _stacked_upper(self):
        return self._rec is not None and self._rec[0] == "lstm2"

    @staticmethod
    def _stack_placeholder(input):
        """gradInput of a fused upper layer: its input gradient went straight into the lower layer's
        steps, so the lower layer ignores what it receives — a zero-stride view of the right shape."""
        return torch.zeros((), dtype=input.dtype, device=input.device).expand(input.shape)

    def updateGradInput(self, input, gradOutput):
        stacked = self._stacked_upper()
        self._gx2 = self._bptt(gradOutput)
        if stacked:
            return self._stack_placeholder(input)
        if self.preTopology is not None:
            return self.preTopology.updateGradInput(input, self._gx2)
        return self._gx2

    def accGradParameters(self, input, gradOutput):
        if self.preTopology is not None:
            self.preTopology.accGradParameters(input, self._gx2)
        self._gx2 = None

    def backward(self, input, gradOutput):
        import time
        t0 = time.perf_counter()
        stacked = self._stacked_upper()
        gx2 = self._bptt(gradOutput)
        if stacked:
            self.preTopology.accGradParameters(input, gx2)
            _fire_grad_ready([self.preTopology.layer])
            gi = self._stack_placeholder(input)
        else:
            gi = self.preTopology.backward(input, gx2) if self.preTopology is not None else gx2
        self.gradInput = gi
        self.backward_time += time.perf_counter() - t0
        for h in self._grad_ready_hooks:
            h(self)
        return gi

    def __repr__(self):
        return f"Recurrent({self.topology!r})"


class RecurrentDecoder(Recurrent):
    """``DL/nn/RecurrentDecoder.scala``: the input (B, H) is the step-1 input; each step's
    output is the next step's input, for ``seqLength`` steps.  The cell applies its own
    preTopology (``includePreTopology``)."""

    def __init__(self, output_length, bigdl_type="float"):
        super().__init__()
        self.seqLength = output_length

    def add(self, module):
        if not isinstance(module, Cell):
            raise ValueError("Recurrent: contained module should be Cell type")
        self.topology = module
        if module.preTopology is not None:
            module.includePreTopology = True
        self.preTopology = None
        self.modules = [module]
        return self

    def updateOutput(self, input):
        if input.dim() not in (2, 4, 5):
            raise ValueError("RecurrentDecoder: input should be a 2D/4D/5D Tensor, e.g [batch, nDim]")
        cell = self.topology
        if cell.hiddensShape[0] != input.shape[1]:
            raise ValueError("hiddenSize is not the same with input size!! Please update cell settings or use "
                             "Recurrent instead!")
        x = input
        if x.is_cuda and x.dtype != _cdtype(x):
            x = x.to(_cdtype(x))
        B = x.shape[0]
        h0 = self._h0(B, list(x.shape[1:]), x.device, x.dtype)
        train = self.train
        tape = _Tape(train)
        with (torch.enable_grad() if train else torch.no_grad()):
            xl = x.detach().requires_grad_(train)
            flat0 = [h.detach().requires_grad_(train) for h in _flat_hidden(h0)]
            hid, _ = _rebuild_hidden(h0, flat0)
            outs = []
            cur = xl
            for _ in range(self.seqLength):
                cur, hid = cell.step_full(cur, hid, tape)
                outs.append(cur)
            out = torch.stack(outs, 1)
        self._last_hidden = cell.pack_hidden(_rebuild_hidden(hid, [v.detach() for v in _flat_hidden(hid)])[0])
        self._rec = ("generic", tape, xl, flat0, out) if train else None
        return out.detach()

    def updateGradInput(self, input, gradOutput):
        return self._bptt(gradOutput)

    def accGradParameters(self, input, gradOutput):
        pass

    def backward(self, input, gradOutput):
        gi = self._bptt(gradOutput)
        self.gradInput = gi
        for h in self._grad_ready_hooks:
            h(self)
        return gi


class BiRecurrent(Container):
    """``DL/nn/BiRecurrent.scala``: forward Recurrent + time-reversed Recurrent, merged by
    ``merge`` (default CAddTable).  ``isSplitInput`` splits the features in two halves."""

    def __init__(self, merge=None, batchNormParams=None, isSplitInput=False, bigdl_type="float"):
        super().__init__()
        from .table_ops import CAddTable
        self.merge = merge if merge is not None else CAddTable(True)
        self.batchNormParams = batchNormParams
        self.isSplitInput = isSplitInput
        self.layer = Recurrent(batchNormParams)
        self.revLayer = Recurrent(batchNormParams)

    def add(self, module):
        import copy
        self.layer.add(module)
        self.revLayer.add(copy.deepcopy(module))  # cloneModule: same initial weights
        self.modules = [self.layer, self.revLayer, self.merge]
        return self

    def getMerge(self):
        return self.merge

    def _split(self, input):
        if self.isSplitInput:
            half = input.shape[2] // 2
            return input[:, :, :half], input[:, :, half:]
        return input, input

    def updateOutput(self, input):
        a, b = self._split(input)
        self._fa, self._fb = a, torch.flip(b, [1])
        ya = self.layer.forward(a)
        yb = torch.flip(self.revLayer.forward(self._fb), [1])
        self._merge_in = T(ya, yb)
        return self.merge.forward(self._merge_in)

    def _grads(self, gradOutput):
        gm = self.merge.backward(self._merge_in, gradOutput)
        return gm[1], torch.flip(gm[2], [1])

    def _join(self, ga, gb):
        gb = torch.flip(gb, [1])
        if self.isSplitInput:
            return torch.cat([ga, gb], 2)
        return ga + gb

    def updateGradInput(self, input, gradOutput):
        ga, gb = self._grads(gradOutput)
        self._ga, self._gb = ga, gb
        return self._join(self.layer.updateGradInput(self._fa, ga), self.revLayer.updateGradInput(self._fb, gb))

    def accGradParameters(self, input, gradOutput):
        self.layer.accGradParameters(self._fa, self._ga)
        self.revLayer.accGradParameters(self._fb, self._gb)

    def backward(self, input, gradOutput):
        ga, gb = self._grads(gradOutput)
        gi = self._join(self.layer.backward(self._fa, ga), self.revLayer.backward(self._fb, gb))
        self.gradInput = gi
        for h in self._grad_ready_hooks:
            h(self)
        return gi
