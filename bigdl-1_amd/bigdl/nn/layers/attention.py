"""Attention / Transformer family: ``Attention``, ``FeedForwardNetwork``, ``Transformer``
(LanguageModel and Translation), ``SequenceBeamSearch`` and the position/mask helpers.

Reference: ``DL/nn/Attention.scala:30-111`` (dense q/k/v/out projections, split heads with
q·depth^-0.5, QKᵀ + bias → softmax → dropout → ·V → combine heads, KV cache for inference at
:114+), ``FeedForwardNetwork.scala``, ``TransformerOperation.scala`` (Xavier dense layers, the
sinusoid position signal, padding / lower-triangle biases with −1e9), ``Transformer.scala``
(pre-norm blocks: x + Dropout(Sublayer(LayerNorm(x))), final LayerNorm), ``SequenceBeamSearch.scala``.

Reference quirks kept on purpose (parity): every Dropout in these layers is built as
``Dropout(1 - rate)``, i.e. the configured rate is the KEEP probability; the beam-search length
penalty is ``(5 + len/6)^alpha``; token ids produced by the search are 1-based.

MI355X path (device tensors, bf16 compute): ``Attention`` runs the Q/K/V projections as ONE
GEMM on the MFMA kernel (gemm.hip) over the adjacent query/key/value weight rows of the
parameter arena (self-attention; K/V fused for encoder-decoder attention), the fused attention
kernels of ``ops/csrc/attention.hip`` read Q/K/V straight out of that [B·L][3H] buffer (no
split/combine-heads copies; causal masking, padding bias and attention dropout in-kernel), and
the output projection is one more GEMM; the backward writes dQ/dK/dV into one [B·L][3H] buffer
that feeds a single weight-gradient GEMM.  ``FeedForwardNetwork`` is GEMM+bias+ReLU epilogue →
dropout → GEMM+bias, backward on the same kernels.  Host tensors (and cached incremental
decoding) use the torch composition below.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from ...utils.table import Table, T
from ..abstractnn import AbstractModule, AutogradModule, TensorModule
from ..initialization_method import Xavier, Zeros, VariableFormats

_MASK = -1e9


def _dense_param(mod, name, out_f, in_f, bias):
    mod.register_parameter(f"{name}Weight", torch.zeros(out_f, in_f), f"{name}GradWeight")
    Xavier().init(getattr(mod, f"{name}Weight"), VariableFormats.OUT_IN)
    if bias:
        mod.register_parameter(f"{name}Bias", torch.zeros(out_f), f"{name}GradBias")


def _drop(x, keep_rate, train):
    """``Dropout(initP = 1 - rate)`` of the reference: drop probability 1 - rate."""
    p = 1.0 - keep_rate
    if not train or p <= 0:
        return x
    if p >= 1:
        return torch.zeros_like(x)
    return F.dropout(x, p, True)


def _native_dense_ok(x):
    """Device activations with bf16 compute and the native attention/GEMM kernels loaded."""
    from ... import ops
    from ...utils.engine import Engine
    return (isinstance(x, torch.Tensor) and x.is_cuda and x.dim() >= 2 and Engine.compute_dtype() == torch.bfloat16
            and ops.native_has("attention_forward"))


def _fused_rows(ts):
    """One [Σrows][cols] view over row blocks that sit back to back in memory (consecutive
    parameters of one flat arena / shadow), else None."""
    t0 = ts[0]
    cols, n = t0.shape[-1], 0
    st0 = t0.untyped_storage()
    for t in ts:
        # adjacency must be WITHIN one storage: separately cast copies can sit back to back by
        # allocator coincidence, and a view over them would run past the first storage
        if (t.dim() != 2 or t.shape[1] != cols or not t.is_contiguous() or t.dtype != t0.dtype
                or t.device != t0.device or t.untyped_storage().data_ptr() != st0.data_ptr()
                or t.data_ptr() != t0.data_ptr() + n * cols * t0.element_size()):
            return None
        n += t.shape[0]
    if (t0.storage_offset() + n * cols) * t0.element_size() > st0.nbytes():
        return None
    return torch.as_strided(t0, (n, cols), (cols, 1))


def _proj_bwd(dbuf, src, ws, gws, scale, need_input):
    """Backward of ``dbuf = src · [W₀; W₁; …]ᵀ`` (one GEMM over the stacked weights when they are
    adjacent): weight gradients accumulated with ``scale``, returns d(src) (or None)."""
    from ...ops import native_ops as NO
    H = src.shape[1]
    wf = _fused_rows(ws)
    if scale != 0:
        gf = _fused_rows(gws)
        if gf is not None:
            NO.wgrad_rows(dbuf, src, gf, scale)
        else:
            for i, g in enumerate(gws):
                NO.wgrad_rows(dbuf[:, i * H:(i + 1) * H].contiguous(), src, g, scale)
    if not need_input:
        return None
    if wf is not None:
        return NO.gemm(dbuf, NO.transpose_bf16(wf))
    d = None
    for i, w in enumerate(ws):
        r = NO.gemm(dbuf[:, i * H:(i + 1) * H], NO.transpose_bf16(w))
        d = r if d is None else d.add_(r)
    return d


def split_heads(x, n_heads):
    B, L, Hd = x.shape
    return x.reshape(B, L, n_heads, Hd // n_heads).transpose(1, 2)


def combine_heads(x):
    B, n, L, d = x.shape
    return x.transpose(1, 2).reshape(B, L, n * d)


class DecodeCache:
    """Preallocated KV cache of cached incremental decoding: ``k`` / ``v`` [rows, Lmax, H] with the
    first ``length`` positions valid, appended to IN PLACE each step (the reference concatenates
    ``[new; cache]`` into a fresh tensor every step, ``DL/nn/Attention.scala:136-141``) and read by
    the decode-attention kernel (``ops/csrc/attn_decode.hip``).  One object serves both the
    ``<name>_k`` and ``<name>_v`` entries of the cache Table.  :meth:`reorder` applies a beam
    search's surviving-beam selection to the valid rows."""

    def __init__(self, rows: int, max_len: int, hidden: int, device=None):
        self.rows, self.max_len, self.hidden, self.device = rows, max(1, int(max_len)), hidden, device
        self.k = self.v = None
        self.length = 0
        self.chunks: list = []  # positions per append, oldest first (the reference order is per chunk)

    def append(self, k, v):
        n = k.shape[1]
        if self.k is None or self.k.dtype != k.dtype:
            self.k = torch.empty((self.rows, self.max_len, self.hidden), dtype=k.dtype, device=k.device)
            self.v = torch.empty_like(self.k)
            self.length = 0
            self.chunks = []
        if self.length + n > self.k.shape[1]:  # grow (amortised doubling) keeping the history
            cap = max(self.length + n, 2 * self.k.shape[1])
            nk = torch.empty((self.rows, cap, self.hidden), dtype=self.k.dtype, device=self.k.device)
            nv = torch.empty_like(nk)
            nk[:, :self.length].copy_(self.k[:, :self.length])
            nv[:, :self.length].copy_(self.v[:, :self.length])
            self.k, self.v = nk, nv
        self.k[:, self.length:self.length + n].copy_(k)
        self.v[:, self.length:self.length + n].copy_(v)
        self.length += n
        self.chunks.append(n)

    def ref_order(self):
        """Storage positions in the reference's key order: the reference concatenates ``[new; cache]``
        per call, so appends are newest first but each multi-position append keeps its own order."""
        order, start = [], 0
        spans = []
        for n in self.chunks:
            spans.append((start, n))
            start += n
        for s0, n in reversed(spans):
            order.extend(range(s0, s0 + n))
        return order

    def kernel_bias(self, bias):
        """``bias`` (last dim = the reference key order) rearranged for the decode kernel, which reads
        key position p's bias at index L − 1 − p (a fully reversed cache): identical unless an append
        held more than one position."""
        L = self.length
        if bias is None or not isinstance(bias, torch.Tensor) or bias.shape[-1] != L or all(n == 1 for n in self.chunks):
            return bias
        r = self.ref_order()  # r[i] = storage position of reference key i
        idx = [0] * L
        for i, pos in enumerate(r):
            idx[L - 1 - pos] = i
        return bias.index_select(-1, torch.tensor(idx, device=bias.device))

    def reorder(self, rows_idx):
        """Row i ← row rows_idx[i] over the valid positions (beam survivors)."""
        L = self.length
        if L and self.k is not None:
            self.k[:, :L] = self.k[rows_idx, :L]
            self.v[:, :L] = self.v[rows_idx, :L]

    def keys(self):
        """The cached keys in the reference's order (newest append first), [rows, L, H]."""
        return self.k[:, self.ref_order()]

    def values(self):
        return self.v[:, self.ref_order()]


class Attention(AutogradModule):
    """Multi-head attention.  Input ``T(x, y, bias)``: queries from ``x`` (B, Lq, H), keys and
    values from ``y`` (B, Lk, H), additive ``bias`` broadcastable to (B, heads, Lq, Lk).  For
    cached incremental decoding pass ``T(x, y, T(bias, cache))`` (inference only); the cache
    Table is updated with ``<name>_k`` / ``<name>_v``."""

    def __init__(self, hidden_size, num_heads, attention_dropout, bigdl_type="float"):
        super().__init__()
        if hidden_size % num_heads:
            raise ValueError("hidden_size must be a multiple of num_heads")
        self.hiddenSize, self.numHeads, self.attentionDropout = hidden_size, num_heads, attention_dropout
        for n in ("query", "key", "value", "output"):
            _dense_param(self, n, hidden_size, hidden_size, False)

    def _proj(self, x, name):
        w = self.P(f"{name}Weight")
        return F.linear(x.to(w.dtype), w)

    def _attend(self, q, k, v, bias):
        depth = self.hiddenSize // self.numHeads
        if q.is_cuda:  # a device tensor reached the torch path: count it like any other fallback
            from ...ops import native as N
            N.note_fallback("attention_forward", "torch-attention", (q, k))
        q = split_heads(q, self.numHeads) * depth ** -0.5
        k = split_heads(k, self.numHeads)
        v = split_heads(v, self.numHeads)
        bias = bias.to(q.dtype) if bias is not None else None
        if not self.train or self.attentionDropout >= 1.0:
            o = F.scaled_dot_product_attention(q, k, v, attn_mask=bias, scale=1.0)
        else:
            logits = q @ k.transpose(-1, -2)
            if bias is not None:
                logits = logits + bias
            w = torch.softmax(logits.float(), -1).to(q.dtype)
            o = _drop(w, self.attentionDropout, True) @ v
        return self._proj(combine_heads(o), "output")

    def _forward(self, input):
        x, y, b = input[1], input[2], input.get(3)  # the bias input is optional
        if isinstance(b, Table):
            return self._forward_cached(x, y, b[1], b[2])
        return self._attend(self._proj(x, "query"), self._proj(y, "key"), self._proj(y, "value"), b)

    # ---- native (device) path -----------------------------------------------------------------
    def _nat_ok(self, x, y, b):
        D = self.hiddenSize // self.numHeads
        return (D in (32, 64, 96, 128) and _native_dense_ok(x) and x.dim() == 3 and isinstance(y, torch.Tensor)
                and y.is_cuda and y.dim() == 3 and (b is None or isinstance(b, torch.Tensor)))

    def updateOutput(self, input):
        x, y, b = input[1], input[2], input.get(3)  # the bias input is optional
        if not isinstance(b, Table) and self._nat_ok(x, y, b):
            return self._nat_forward(x, y, b)
        self._nat = None
        return super().updateOutput(input)

    def _nat_forward(self, x, y, b):
        from ... import ops
        from ...ops import native_ops as NO
        bf = torch.bfloat16
        H, nh = self.hiddenSize, self.numHeads
        D = H // nh
        B, Lq, _ = x.shape
        Lk = y.shape[1]
        x2 = x.reshape(B * Lq, H).to(bf).contiguous()
        same = y is x or (y.data_ptr() == x.data_ptr() and y.shape == x.shape and y.stride() == x.stride())
        y2 = x2 if same else y.reshape(B * Lk, H).to(bf).contiguous()
        ws = [self.cw(n + "Weight", bf) for n in ("query", "key", "value")]
        wqkv = _fused_rows(ws) if same else None
        if wqkv is not None:  # self-attention: one [B·L][3H] projection
            qkv = NO.gemm(x2, wqkv)
            q, k, v = qkv[:, :H], qkv[:, H:2 * H], qkv[:, 2 * H:]
        else:
            q = NO.gemm(x2, ws[0])
            wkv = _fused_rows(ws[1:])
            if wkv is not None:
                kv = NO.gemm(y2, wkv)
                k, v = kv[:, :H], kv[:, H:]
            else:
                k, v = NO.gemm(y2, ws[1]), NO.gemm(y2, ws[2])
        causal = bool(getattr(b, "_bigdl_causal", False)) and Lq == Lk
        bias = None if (causal or b is None) else b
        keep = float(self.attentionDropout) if (self.train and self.attentionDropout < 1.0) else 1.0
        seed = NO.attention_seed(x.device) if keep < 1.0 else 0
        o, lse = ops.attention_forward(q, k, v, B, nh, Lq, Lk, D, D ** -0.5, bias, causal, keep, seed)
        out = NO.gemm(o, self.cw("outputWeight", bf))
        self._nat = (x2, y2, same, q, k, v, o, lse, bias, causal, keep, seed, B, Lq, Lk, x.dtype, y.dtype,
                     b) if self.train else None
        self._gi_done = False
        return out.view(B, Lq, H)

    def _nat_backward(self, gradOutput, need_input):
        from ... import ops
        from ...ops import native_ops as NO
        (x2, y2, same, q, k, v, o, lse, bias, causal, keep, seed, B, Lq, Lk, xdt, ydt, b) = self._nat
        self._nat = None
        bf = torch.bfloat16
        H, nh = self.hiddenSize, self.numHeads
        D = H // nh
        s = self.scale_w
        gy = gradOutput.reshape(B * Lq, H).to(bf).contiguous()
        do = NO.linear_backward(gy, o, self.cw("outputWeight", bf), True, self.outputGradWeight, None, s)
        names = ("query", "key", "value")
        ws = [self.cw(n + "Weight", bf) for n in names]
        gws = [getattr(self, n + "GradWeight") for n in names]
        if same:
            dqkv = torch.empty((B * Lq, 3 * H), dtype=bf, device=gy.device)
            ops.attention_backward(do, q, k, v, o, lse, B, nh, Lq, Lk, D, D ** -0.5, bias, causal, keep, seed,
                                   dq=dqkv[:, :H], dk=dqkv[:, H:2 * H], dv=dqkv[:, 2 * H:])
            if s != 0:
                gf = _fused_rows(gws)
                if gf is not None:
                    NO.wgrad_rows(dqkv, x2, gf, s)
                else:
                    for i, g in enumerate(gws):
                        NO.wgrad_rows(dqkv[:, i * H:(i + 1) * H].contiguous(), x2, g, s)
            dx = dy = None
            if need_input:
                wf = _fused_rows(ws)
                wt = NO.transpose_bf16(wf) if wf is not None else torch.cat([NO.transpose_bf16(w) for w in ws], 1)
                dx = NO.gemm(dqkv[:, :H], wt[:, :H])
                dy = NO.gemm(dqkv[:, H:], wt[:, H:])
        else:
            dq = torch.empty((B * Lq, H), dtype=bf, device=gy.device)
            dkv = torch.empty((B * Lk, 2 * H), dtype=bf, device=gy.device)
            ops.attention_backward(do, q, k, v, o, lse, B, nh, Lq, Lk, D, D ** -0.5, bias, causal, keep, seed,
                                   dq=dq, dk=dkv[:, :H], dv=dkv[:, H:])
            dx = _proj_bwd(dq, x2, ws[:1], gws[:1], s, need_input)
            dy = _proj_bwd(dkv, y2, ws[1:], gws[1:], s, need_input)
        self._gi_done = True
        if not need_input:
            return None
        gi = [dx.view(B, Lq, H).to(xdt), dy.view(B, Lk, H).to(ydt)]
        if b is not None:  # the mask inputs (PaddingMask / SelfAttentionMask) take no gradient
            gi.append(torch.zeros_like(b))
        return T(*gi)

    def updateGradInput(self, input, gradOutput):
        if getattr(self, "_nat", None) is not None:
            return self._nat_backward(gradOutput, True)
        return super().updateGradInput(input, gradOutput)

    def accGradParameters(self, input, gradOutput):
        if getattr(self, "_gi_done", False):
            self._gi_done = False
            return
        if getattr(self, "_nat", None) is not None:
            self._nat_backward(gradOutput, False)
            self._gi_done = False
            return
        super().accGradParameters(input, gradOutput)

    def _forward_cached(self, x, y, bias, cache):
        if self.train:
            raise RuntimeError("Only support input cache for model inference")
        kn, vn = f"{self.get_name()}_k", f"{self.get_name()}_v"
        dc = cache.get(kn) if isinstance(cache, Table) else None
        if isinstance(dc, DecodeCache):
            return self._forward_decode(x, y, bias, cache, dc, kn, vn)
        q = self._proj(x, "query")
        k = self._proj(y, "key")
        v = self._proj(y, "value")
        kn, vn = f"{self.get_name()}_k", f"{self.get_name()}_v"
        if isinstance(cache, Table) and len(list(cache.keys())) > 0:
            ck, cv = cache.get(kn), cache.get(vn)
            if ck is not None and ck.numel() > 0:
                k = torch.cat([k, ck.to(k.dtype)], 1)
                v = torch.cat([v, cv.to(v.dtype)], 1)
            cache[kn] = k
            cache[vn] = v
        return self._attend(q, k, v, bias)


    def _forward_decode(self, x, y, bias, cache, dc, kn, vn):
        """One decoding step on a :class:`DecodeCache`: project the new token(s), append K/V in
        place, attend over the whole cache with the decode kernel (``ops.attention_decode``)."""
        from ... import ops
        H, nh = self.hiddenSize, self.numHeads
        D = H // nh
        rows, Lq, Ly = x.shape[0], x.shape[1], y.shape[1]
        native = _native_dense_ok(x) and isinstance(y, torch.Tensor) and y.is_cuda and H % 8 == 0
        q = k = v = None
        if native:
            # bf16 compute on the native GEMMs; any shape a GEMM refuses (NotImplemented) takes the
            # reference projections below in x's dtype
            from ...ops import native_ops as NO
            bf = torch.bfloat16
            x2 = x.reshape(rows * Lq, H).to(bf).contiguous()
            y2 = x2 if (y is x) else y.reshape(rows * Ly, H).to(bf).contiguous()
            q = NO.gemm(x2, self.cw("queryWeight", bf))
            wkv = _fused_rows([self.cw("keyWeight", bf), self.cw("valueWeight", bf)])
            if wkv is not None:
                kv = NO.gemm(y2, wkv)
                if kv is not NotImplemented:
                    kv = kv.view(rows, Ly, 2 * H)
                    k, v = kv[..., :H], kv[..., H:]
            else:
                k = NO.gemm(y2, self.cw("keyWeight", bf))
                v = NO.gemm(y2, self.cw("valueWeight", bf))
                k = k.view(rows, Ly, H) if k is not NotImplemented else None
                v = v.view(rows, Ly, H) if v is not NotImplemented else None
            q = q.view(rows, Lq, H) if q is not NotImplemented else None
            native = q is not None and k is not None and v is not None
        if not native:
            q, k, v = self._proj(x, "query"), self._proj(y, "key"), self._proj(y, "value")
        dc.append(k, v)
        cache[kn] = dc
        cache[vn] = dc
        o = ops.attention_decode(q.contiguous(), dc.k, dc.v, dc.length, nh, D, D ** -0.5, dc.kernel_bias(bias), True)
        if native:
            from ...ops import native_ops as NO
            out = NO.gemm(o.reshape(rows * Lq, H).to(torch.bfloat16).contiguous(),
                          self.cw("outputWeight", torch.bfloat16))
            if out is not NotImplemented:
                return out.view(rows, Lq, H)
            o = o.to(x.dtype)
        return self._proj(o, "output")


class FeedForwardNetwork(AutogradModule):
    """dense(H→F, ReLU) → Dropout(1 - reluDropout) → dense(F→H) (``FeedForwardNetwork.scala``)."""

    def __init__(self, hidden_size, filter_size, relu_dropout, bigdl_type="float"):
        super().__init__()
        self.hiddenSize, self.filterSize, self.reluDropout = hidden_size, filter_size, relu_dropout
        _dense_param(self, "filter", filter_size, hidden_size, True)
        _dense_param(self, "output", hidden_size, filter_size, True)

    def updateOutput(self, x):
        if (_native_dense_ok(x) and self.hiddenSize % 8 == 0 and self.filterSize % 8 == 0
                and x.shape[-1] == self.hiddenSize):
            return self._nat_forward(x)
        self._nat = None
        return super().updateOutput(x)

    def _nat_forward(self, x):
        from ... import ops
        from ...ops import native_ops as NO
        bf = torch.bfloat16
        x2 = x.reshape(-1, self.hiddenSize).to(bf).contiguous()
        h = NO.linear_forward(x2, self.cw("filterWeight", bf), self.filterBias, act=1)  # GEMM+bias+ReLU
        p = 1.0 - self.reluDropout
        hd, mask = h, None
        if self.train and p > 0:
            if p >= 1:
                hd = torch.zeros_like(h)
            else:
                hd, mask = ops.dropout_forward(h, p)
        y = NO.linear_forward(hd, self.cw("outputWeight", bf), self.outputBias)
        self._nat = (x2, h, hd, mask, p, x.shape, x.dtype) if self.train else None
        self._gi_done = False
        return y.view(*x.shape[:-1], self.hiddenSize)

    def _nat_backward(self, gradOutput, need_input):
        from ... import ops
        from ...ops import native_ops as NO
        x2, h, hd, mask, p, shape, xdt = self._nat
        self._nat = None
        bf, s = torch.bfloat16, self.scale_w
        gy = gradOutput.reshape(-1, self.hiddenSize).to(bf).contiguous()
        dhd = NO.linear_backward(gy, hd, self.cw("outputWeight", bf), True, self.outputGradWeight,
                                 self.outputGradBias, s)
        if mask is not None:
            dhd = ops.dropout_backward(dhd, mask, p)
        elif self.train and p >= 1:
            dhd = torch.zeros_like(dhd)
        dh = NO.relu_backward(dhd, h)
        dx = NO.linear_backward(dh, x2, self.cw("filterWeight", bf), need_input, self.filterGradWeight,
                                self.filterGradBias, s)
        self._gi_done = True
        return None if dx is None else dx.view(shape).to(xdt)

    def updateGradInput(self, input, gradOutput):
        if getattr(self, "_nat", None) is not None:
            return self._nat_backward(gradOutput, True)
        return super().updateGradInput(input, gradOutput)

    def accGradParameters(self, input, gradOutput):
        if getattr(self, "_gi_done", False):
            self._gi_done = False
            return
        if getattr(self, "_nat", None) is not None:
            self._nat_backward(gradOutput, False)
            self._gi_done = False
            return
        super().accGradParameters(input, gradOutput)

    def _forward(self, x):
        w1, b1 = self.P("filterWeight"), self.P("filterBias")
        h = F.relu(F.linear(x.to(w1.dtype), w1, b1.to(w1.dtype)))
        h = _drop(h, self.reluDropout, self.train)
        w2, b2 = self.P("outputWeight"), self.P("outputBias")
        return F.linear(h, w2, b2.to(w2.dtype))


def position_signal(length, channels, min_timescale=1.0, max_timescale=1.0e4, device=None):
    """``TransformerOperation.getPositionEncode``: [sin | cos] of position·inv_timescale."""
    n = channels // 2
    log_inc = math.log(max_timescale / min_timescale) / max(n - 1, 1)
    inv = min_timescale * torch.exp(torch.arange(n, dtype=torch.float32, device=device) * -log_inc)
    t = torch.arange(length, dtype=torch.float32, device=device).unsqueeze(1) * inv.unsqueeze(0)
    out = torch.zeros(length, channels, device=device)
    out[:, :n] = torch.sin(t)
    out[:, n:2 * n] = torch.cos(t)
    return out


def lower_triangle_bias(length, device=None):
    """(1, 1, L, L) with −1e9 above the diagonal (``attentionBiasLowerTriangle``)."""
    m = torch.triu(torch.full((length, length), _MASK, device=device), diagonal=1).reshape(1, 1, length, length)
    m._bigdl_causal = True  # the native attention applies this mask in-kernel (and skips masked tiles)
    return m


class PositionEncode(TensorModule):
    """Position signal (L, C) of a (B, L, C) input (no gradient to the input)."""

    def updateOutput(self, input):
        return position_signal(input.shape[1], input.shape[2], device=input.device).to(input.dtype)

    def updateGradInput(self, input, gradOutput):
        return torch.zeros_like(input)


class PositionEncodeWithShift(TensorModule):
    """Shift the sequence right by one step, then add the position signal."""

    def updateOutput(self, input):
        out = torch.zeros_like(input)
        out[:, 1:] = input[:, :-1]
        return out + position_signal(input.shape[1], input.shape[2], device=input.device).to(input.dtype)

    def updateGradInput(self, input, gradOutput):
        g = torch.zeros_like(gradOutput)
        g[:, :-1] = gradOutput[:, 1:]
        return g


class PaddingMask(TensorModule):
    """(B, L) ids → (B, 1, 1, L) bias with −1e9 at padding (id == 0) positions."""

    def updateOutput(self, input):
        return ((input == 0).to(torch.float32) * _MASK).unsqueeze(1).unsqueeze(1)

    def updateGradInput(self, input, gradOutput):
        return torch.zeros_like(input, dtype=torch.float32)


class SelfAttentionMask(TensorModule):
    """(B, L, ...) → (1, 1, L, L) causal bias."""

    def updateOutput(self, input):
        return lower_triangle_bias(input.shape[1], device=input.device)

    def updateGradInput(self, input, gradOutput):
        return torch.zeros_like(input)


class SplitTensor(TensorModule):
    """Split dimension ``dim`` (1-based) into ``n`` equal chunks → Table."""

    def __init__(self, dim, n, bigdl_type="float"):
        super().__init__()
        self.dim, self.n = dim, n

    def updateOutput(self, input):
        return T(*torch.chunk(input, self.n, self.dim - 1))

    def updateGradInput(self, input, gradOutput):
        return torch.cat([gradOutput[i + 1] for i in range(self.n)], self.dim - 1)


class Transformer(AbstractModule):
    """``DL/nn/Transformer.scala``.  ``transformer_type`` "LanguageModel" (input ids (B, L) →
    (B, L, H) hidden states) or "Translation" (training input T(src, tgt) → (B, Lt, H) or logits
    with ``with_share_weights_linear``; inference input src ids → T(decoded ids, scores) via
    ``beam_search``)."""

    def __init__(self, vocab_size, hidden_size, num_heads, filter_size, num_hidden_layers, embedding_dropout,
                 attention_dropout, ffn_dropout, padding_value=0.0, with_share_weights_linear=False,
                 transformer_type="LanguageModel", beam_search=None, bigdl_type="float"):
        super().__init__()
        from ..containers import Sequential
        from ..graph import Graph, Input
        from .embedding import LookupTable
        from .math_ops import MulConstant
        from .linear import Linear
        from .recurrent import TimeDistributed
        self.vocabSize, self.hiddenSize, self.numHeads = vocab_size, hidden_size, num_heads
        self.filterSize, self.numHiddenlayers = filter_size, num_hidden_layers
        self.embeddingDropout, self.attentionDropout, self.ffnDropout = embedding_dropout, attention_dropout, ffn_dropout
        self.paddingValue = padding_value
        self.withShareWeightsLinear = with_share_weights_linear
        self.transformerType = transformer_type
        self.beamSearch = beam_search
        self.embedding = LookupTable(vocab_size, hidden_size, padding_value=padding_value, mask_zero=True)
        self.embedding.set_name("embedding")
        emb_seq = Sequential().add(self.embedding).add(MulConstant(math.sqrt(hidden_size)))
        self.linearSharedWeights = TimeDistributed(Linear(hidden_size, vocab_size, with_bias=False))
        if transformer_type == "LanguageModel":
            inp = Input()
            e = emb_seq(inp)
            dec_in = _Dropout(embedding_dropout)(PositionEncodeWithShift()(e))
            bias = SelfAttentionMask()(e)
            out = self._block(dec_in, bias, None, None, "decode")
            self.model = Graph(inp, out)
        elif transformer_type == "Translation":
            self.encoderStack = self._stack(encoder=True)
            self.decoderStack = self._stack(encoder=False)
            src, tgt = Input(), Input()
            from .table_ops import JoinTable, SelectTable, CAddTable
            mask = PaddingMask()(src)
            joined = JoinTable(1, -1)(src, tgt)
            emb = emb_seq(joined)
            split = SplitTensor(1, 2)(emb)
            emb_in, emb_out = SelectTable(1)(split), SelectTable(2)(split)
            enc_out = self._encode(emb_in, mask)
            dec_in = _Dropout(embedding_dropout)(PositionEncodeWithShift()(emb_out))
            dec_bias = SelfAttentionMask()(emb_out)
            out = self.decoderStack(dec_in, dec_bias, enc_out, mask)
            self.model = Graph([src, tgt], out)
            self._emb_seq = emb_seq
            if beam_search is not None:
                beam_search.setLogitFn(self.symbols)
        else:
            raise ValueError(f"Only support LanguageModel and Translation transformer type, got {transformer_type}")

    # -- construction helpers ------------------------------------------------------------
    def _encode(self, emb, mask):
        from .table_ops import CAddTable
        pos = PositionEncode()(emb)
        x = _Dropout(self.embeddingDropout)(CAddTable()(emb, pos))
        return self.encoderStack(x, mask)

    def _stack(self, encoder):
        from ..graph import Graph, Input
        if encoder:
            x, b = Input(), Input()
            return Graph([x, b], self._block(x, b, None, None, "encoder"))
        x, b, eo, eb = Input(), Input(), Input(), Input()
        return Graph([x, b, eo, eb], self._block(x, b, eo, eb, "decoder"))

    def _sub(self, layer, x, inputs, name, suffix):
        from .normalization import LayerNormalization
        from .table_ops import CAddTable
        norm = LayerNormalization(self.hiddenSize).set_name(name + "/norm")(x)
        args = [norm if a is None else a for a in inputs]
        y = layer.set_name(name + "/" + suffix)(*args)
        return CAddTable()(x, _Dropout(self.embeddingDropout).set_name(name + "/dropout")(y))

    def _block(self, x, self_bias, enc_out, enc_bias, kind):
        from .normalization import LayerNormalization
        for i in range(self.numHiddenlayers):
            att = Attention(self.hiddenSize, self.numHeads, self.attentionDropout)
            x = self._sub(att, x, [None, None, self_bias], f"{kind}_self_attention_{i}", "self_attention")
            if enc_out is not None and enc_bias is not None:
                att2 = Attention(self.hiddenSize, self.numHeads, self.attentionDropout)
                x = self._sub(att2, x, [None, enc_out, enc_bias], f"{kind}_encdec_attention_{i}", "encdec_attention")
            ffn = FeedForwardNetwork(self.hiddenSize, self.filterSize, self.ffnDropout)
            x = self._sub(ffn, x, [None], f"{kind}_ffn_{i}", "ffn")
        return LayerNormalization(self.hiddenSize)(x)

    def children(self):
        ch = [self.model]
        if self.withShareWeightsLinear:
            ch.append(self.linearSharedWeights)
        return ch

    def _param_entries(self):
        return self.model._param_entries()

    def parameters(self):
        return self.model.parameters()

    def _set_arena_recursive(self, arena):
        self._arena = arena
        self.model._set_arena_recursive(arena)

    def zeroGradParameters(self):
        self.model.zeroGradParameters()

    def _share(self):
        lin = self.linearSharedWeights.layer
        with torch.no_grad():
            lin.weight.copy_(self.embedding.weight)

    # -- forward / backward --------------------------------------------------------------
    def updateOutput(self, input):
        if self.transformerType == "Translation" and isinstance(input, torch.Tensor):
            if self.train:
                raise RuntimeError("Input for Transformer should be tensor when doing translation prediction")
            return self._translate(input)
        out = self.model.forward(input)
        if self.withShareWeightsLinear:
            self._share()
            out = self.linearSharedWeights.forward(out)
        return out

    def updateGradInput(self, input, gradOutput):
        g = gradOutput
        if self.withShareWeightsLinear:
            g = self.linearSharedWeights.updateGradInput(self.model.output, gradOutput)
        return self.model.updateGradInput(input, g)

    def accGradParameters(self, input, gradOutput):
        g = gradOutput
        if self.withShareWeightsLinear:
            g = self.linearSharedWeights.gradInput
        self.model.accGradParameters(input, g)

    def backward(self, input, gradOutput):
        g = gradOutput
        if self.withShareWeightsLinear:
            g = self.linearSharedWeights.updateGradInput(self.model.output, gradOutput)
        gi = self.model.backward(input, g)
        self.gradInput = gi
        for h in self._grad_ready_hooks:
            h(self)
        return gi

    # -- translation inference -----------------------------------------------------------
    def _translate(self, src):
        if self.beamSearch is None:
            raise RuntimeError("Translation inference needs a SequenceBeamSearch")
        with torch.no_grad():
            mask = PaddingMask().forward(src)
            emb = self._emb_seq.forward(src)
            x = emb + position_signal(emb.shape[1], emb.shape[2], device=emb.device).to(emb.dtype)
            enc = self.encoderStack.forward(T(x, mask))
            res = self.beamSearch.forward(T(enc, mask))
        ids = res[1][:, 0]
        scores = res[2][:, 0]
        return T(ids[:, 1:], scores)

    def symbols(self, ids, i, max_decode_length, encoder_outputs, enc_bias, cache_value):
        """Logits for step ``i`` of incremental decoding (``Transformer.symbols``)."""
        cache = Table()
        for m in range(1, self.numHiddenlayers + 1):
            if cache_value.contains(f"layer_{m}_k"):
                cache[f"decoder_self_attention_{m - 1}/self_attention_k"] = cache_value[f"layer_{m}_k"]
                cache[f"decoder_self_attention_{m - 1}/self_attention_v"] = cache_value[f"layer_{m}_v"]
        sig = position_signal(max_decode_length + 1, self.hiddenSize, device=ids.device)
        dec_in = self._emb_seq.forward(ids[:, i:i + 1])
        dec_in = dec_in + sig[i].to(dec_in.dtype)
        self_bias = lower_triangle_bias(max_decode_length, device=ids.device)[:, :, i:i + 1, :i + 1]
        out = self.decoderStack.forward(T(dec_in, T(self_bias, cache), encoder_outputs, enc_bias))
        self._share()
        logits = self.linearSharedWeights.forward(out)
        for m in range(1, self.numHiddenlayers + 1):
            if cache_value.contains(f"layer_{m}_k"):
                cache_value[f"layer_{m}_k"] = cache[f"decoder_self_attention_{m - 1}/self_attention_k"]
                cache_value[f"layer_{m}_v"] = cache[f"decoder_self_attention_{m - 1}/self_attention_v"]
        return logits.squeeze(1), cache_value


class _Dropout(TensorModule):
    """``Dropout(1 - rate)`` as built inside the reference transformer layers."""

    def __init__(self, rate, bigdl_type="float"):
        super().__init__()
        self.rate = rate
        self._mask = None

    def updateOutput(self, input):
        p = 1.0 - self.rate
        if not self.train or p <= 0:
            self._mask = None
            return input
        keep = 1.0 - p
        self._mask = (torch.rand_like(input, dtype=torch.float32) < keep).to(input.dtype) / max(keep, 1e-12)
        return input * self._mask

    def updateGradInput(self, input, gradOutput):
        return gradOutput if self._mask is None else gradOutput * self._mask


class SequenceBeamSearch(AbstractModule):
    """Beam search over a logit function (``SequenceBeamSearch.scala``), vectorised on device.

    ``forward(T(encoder_outputs (B, L, H), attention_bias))`` → ``T(seq (B, beam, len+1),
    scores (B, beam))``.  The logit function is ``fn(ids (B·beam, i+1), i, max_len, enc, bias,
    cache Table) -> (logits (B·beam, V), cache)``."""

    def __init__(self, vocab_size, beam_size, alpha, max_decode_length, eos_id, padding_value, num_hidden_layers,
                 hidden_size, bigdl_type="float"):
        super().__init__()
        self.vocabSize, self.beamSize, self.alpha = vocab_size, beam_size, alpha
        self.maxDecodeLength, self.eosID, self.paddingValue = max_decode_length, eos_id, padding_value
        self.numHiddenLayers, self.hiddenSize = num_hidden_layers, hidden_size
        self._fn = None
        #: decode with preallocated in-place KV caches (:class:`DecodeCache`); False = tensor caches
        self.inPlaceCache = True

    INF = -1e7

    def setLogitFn(self, fn):
        self._fn = fn
        return self

    def _len_norm(self, length):
        return (5.0 + length / 6.0) ** self.alpha

    @staticmethod
    def _gather(t, idx):
        """t (B, K, ...) gathered along dim 1 by idx (B, K')."""
        shape = idx.shape + t.shape[2:]
        ix = idx.reshape(idx.shape + (1,) * (t.dim() - 2)).expand(shape)
        return torch.gather(t, 1, ix)

    def _cache_map(self, cache, fn):
        out = Table()
        for k, v in cache.items():
            out[k] = fn(v) if isinstance(v, torch.Tensor) and v.numel() > 0 else v
        return out

    def updateOutput(self, input):
        if self._fn is None:
            raise RuntimeError("SequenceBeamSearch: call setLogitFn first")
        enc, bias = input[1], input[2]
        B, K, V = enc.shape[0], self.beamSize, self.vocabSize
        dev = enc.device
        alive_seq = torch.full((B, K, 1), float(self.paddingValue), device=dev)
        alive_lp = torch.full((B, K), self.INF, device=dev)
        alive_lp[:, 0] = 0
        enc_b = enc.unsqueeze(1).expand(B, K, *enc.shape[1:]).contiguous()
        bias_b = bias.unsqueeze(1).expand(B, K, *bias.shape[1:]).contiguous()
        cache = Table()
        for j in range(1, self.numHiddenLayers + 1):
            if self.inPlaceCache:
                # one preallocated in-place KV cache per decoder layer (both Table entries)
                dc = DecodeCache(B * K, self.maxDecodeLength + 1, self.hiddenSize, dev)
                cache[f"layer_{j}_k"] = dc
                cache[f"layer_{j}_v"] = dc
            else:  # the reference's tensor cache ([new; cache] concatenation every step)
                cache[f"layer_{j}_k"] = torch.empty(0, device=dev)
                cache[f"layer_{j}_v"] = torch.empty(0, device=dev)
        fin_seq = torch.zeros_like(alive_seq)
        fin_scores = torch.full((B, K), self.INF, device=dev)
        fin_flags = torch.zeros(B, K, dtype=torch.bool, device=dev)
        flat = lambda t: t.reshape((B * t.shape[1],) + tuple(t.shape[2:]))  # noqa: E731
        i = 0
        while self._continue(i, alive_lp, fin_scores, fin_flags):
            # grow alive
            fcache = self._cache_map(cache, flat)
            logits, ncache = self._fn(flat(alive_seq).long(), i, self.maxDecodeLength, flat(enc_b), flat(bias_b),
                                      fcache)
            logits = logits.float().reshape(B, K, V)
            lp = torch.log_softmax(logits, -1) + alive_lp.unsqueeze(2)
            top_lp, top_idx = lp.reshape(B, K * V).topk(2 * K, -1)
            beam_idx = torch.div(top_idx, V, rounding_mode="floor")
            top_ids = (top_idx % V + 1).float()
            top_seq = torch.cat([self._gather(alive_seq, beam_idx), top_ids.unsqueeze(2)], 2)
            ncache = self._cache_map(ncache, lambda v: self._gather(v.reshape((B, K) + tuple(v.shape[1:])), beam_idx))
            enc2 = self._gather(enc_b, beam_idx)
            bias2 = self._gather(bias_b, beam_idx)
            finished_now = top_ids == self.eosID
            # new alive state
            nlp = top_lp + finished_now.float() * self.INF
            _, keep = nlp.topk(K, -1)
            # surviving beams of the in-place caches: row (b, k) ← alive row (b, beam_idx[b, keep[b, k]])
            dcs = {id(v): v for v in ncache.values() if isinstance(v, DecodeCache)}
            if dcs:
                sel = beam_idx.gather(1, keep)
                rows = (torch.arange(B, device=dev).unsqueeze(1) * K + sel).reshape(-1)
                for dc in dcs.values():
                    dc.reorder(rows)
            alive_seq = self._gather(top_seq, keep)
            alive_lp = self._gather(nlp, keep)
            enc_b = self._gather(enc2, keep)
            bias_b = self._gather(bias2, keep)
            cache = self._cache_map(ncache, lambda v: self._gather(v, keep))
            # new finished state
            fin_seq = torch.cat([fin_seq, torch.full((B, K, 1), float(self.paddingValue), device=dev)], 2)
            scores = top_lp / self._len_norm(i + 1) + (1.0 - finished_now.float()) * self.INF
            all_seq = torch.cat([fin_seq, top_seq], 1)
            all_scores = torch.cat([fin_scores, scores], 1)
            all_flags = torch.cat([fin_flags, finished_now], 1)
            _, keep = all_scores.topk(K, -1)
            fin_seq = self._gather(all_seq, keep)
            fin_scores = self._gather(all_scores, keep)
            fin_flags = self._gather(all_flags, keep)
            i += 1
        any_fin = fin_flags.any(1)
        seq = torch.where(any_fin.reshape(B, 1, 1), fin_seq, alive_seq)
        scores = torch.where(any_fin.reshape(B, 1), fin_scores, alive_lp)
        return T(seq, scores)

    def _continue(self, i, alive_lp, fin_scores, fin_flags):
        if i >= self.maxDecodeLength:
            return False
        best_alive = alive_lp[:, 0] / self._len_norm(self.maxDecodeLength)
        lowest_fin = (fin_scores * fin_flags.float()).min(1).values
        lowest_fin = lowest_fin + (1.0 - fin_flags.any(1).float()) * self.INF
        return not bool(torch.all(lowest_fin > best_alive))

    def updateGradInput(self, input, gradOutput):
        raise RuntimeError("SequenceBeamSearch is inference only")
