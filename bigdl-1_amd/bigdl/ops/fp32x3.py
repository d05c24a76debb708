"""fp32 compute mode on the bf16 MFMA kernels ("bf16x3", ``csrc/precision.hip``).

The reference trains in fp32 (MKL sgemm / MKL-DNN fp32 primitives: ``DL/nn/SpatialConvolution.scala:253-362``,
``DL/nn/Linear.scala:108-158``).  On CDNA4 an fp32 MFMA runs at 1/16 of the bf16 rate, so with
``bigdl.compute.dtype=fp32`` the convolutions and Linear layers on a GPU split every fp32 operand
into ``hi = bf16(v)`` and ``lo = bf16(v - hi)`` and evaluate ``a_hi·b_hi + a_hi·b_lo + a_lo·b_hi``
with fp32 accumulation (the dropped ``a_lo·b_lo`` term is ≤ 2^-16 relative per product, ~100× below
bf16 rounding and below TF32) — on the SAME tuned kernels as the bf16 path, the three products
being one GEMM over a 3× longer reduction:

* conv forward / data gradient: parts concatenated along the input channels — activations
  ``[hi | hi | lo]``, filters ``[hi | lo | hi]`` — into the implicit-GEMM conv with an fp32 epilogue
  (``ConvParams::y32``); strided data gradients run on a zero lattice of dY (stride-1 conv of the
  flipped filter);
* conv weight gradient: three launches of the split-K wgrad kernel (fp32 accumulation) over channel
  slices of the side-by-side splits — (x_hi, dY_hi), (x_hi, dY_lo), (x_lo, dY_hi) — reusing the
  data gradient's split of dY for stride-1 convs;
* Linear: the same concatenation along K into the MFMA GEMM with an fp32 C.

With ``bigdl.fp32.direct`` (default) convolutions whose reduction channels are a multiple of 32 skip
the materialised splits altogether: ``csrc/conv_x3.hip`` stages the raw fp32 activations / gradients
by LDS-DMA and splits each MFMA fragment while reading it (pre-split 32-channel [hi | lo] weight
chunks on the other side), and the weight gradient runs ONE launch of the fp32-operand wgrad kernel
(split between its global load and LDS store) — so the BatchNorm passes around them write fp32 only.

Every entry returns ``NotImplemented`` for a case it does not cover (grouped conv, fused BN
prologues) and the caller falls back to the torch op.  ``bigdl.fp32.native=false`` turns the path
off (torch / MIOpen fp32 everywhere).
"""
from __future__ import annotations

import ctypes as C
import weakref

import torch

from .native import ptr, check, stream_ptr
from . import native as N
from ..utils import config

_bf16 = torch.bfloat16
_f32 = torch.float32
_cl = torch.channels_last

#: part codes: bit q set → part q holds the lo half
HHL = 0b100  # [hi | hi | lo]  (the "A" side)
HLH = 0b010  # [hi | lo | hi]  (the "B" side)


def enabled(t) -> bool:
    return (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == _f32 and N.has("conv2d_forward")
            and bool(config.get_property("bigdl.fp32.native")))


def _r(n, m):
    return (n + m - 1) // m * m


def _s():
    return C.c_void_p(stream_ptr())


def split(rows2d: torch.Tensor, cp: int, code: int, stacked: bool, out: torch.Tensor = None) -> torch.Tensor:
    """fp32 [rows][C] (unit column stride) → bf16 parts, each ``cp`` wide (zero-padded): side by
    side ``[rows][3·cp]`` or stacked ``[3·rows][cp]``.  ``out`` (optional) receives them (it may
    have more rows than written, e.g. zero rows padding a GEMM operand)."""
    rows, c = rows2d.shape
    if rows2d.stride(1) != 1 or rows2d.dtype != _f32:
        rows2d = rows2d.float().contiguous()
    shape = (3 * rows, cp) if stacked else (rows, 3 * cp)
    if out is None:
        out = torch.empty(shape, dtype=_bf16, device=rows2d.device)
    check(N.lib().bigdl_split_bf16x3(ptr(rows2d), C.c_longlong(rows), C.c_int(c), C.c_longlong(rows2d.stride(0)),
                                     C.c_int(cp), ptr(out), C.c_int(code), C.c_int(1 if stacked else 0), _s()),
          "split_bf16x3")
    return out


def split2(rows2d: torch.Tensor, cp: int) -> torch.Tensor:
    """fp32 [rows][C] → bf16 ``[rows][2·cp]`` = [hi | lo] (zero-padded to cp each): the conv
    kernels read it as the three logical parts [hi | hi | lo] (``ConvParams::cdup``), so the duplicated
    hi part is never stored; the weight-gradient launches take its hi / lo halves as channel slices."""
    rows, c = rows2d.shape
    if rows2d.stride(1) != 1 or rows2d.dtype != _f32:
        rows2d = rows2d.float().contiguous()
    out = torch.empty((rows, 2 * cp), dtype=_bf16, device=rows2d.device)
    check(N.lib().bigdl_split_bf16x2(ptr(rows2d), C.c_longlong(rows), C.c_int(c), C.c_longlong(rows2d.stride(0)),
                                     C.c_int(cp), ptr(out), _s()), "split_bf16x2")
    return out


def _two_part() -> bool:
    return bool(config.get_property("bigdl.fp32.twoPart"))


# Splits written by the PRODUCER of an activation (the fp32 BN apply pass emits the [hi | lo] operand of
# the conv that consumes its output, forward and backward), keyed by the tensor's memory and checked
# against a weak reference to it (alive ⇒ the memory is not reused) and its version counter (shared by
# views: an in-place write invalidates the entry).
_SPLITS: dict = {}


def split_buffer(rows, c, device):
    """A [rows][2·c] bf16 buffer for a producer-side split, or None when the path is off (or not
    needed: with the direct kernels a consumer of C % 32 channels reads the fp32 tensor itself)."""
    if c % 8 or not _two_part() or not config.get_property("bigdl.fp32.producerSplit"):
        return None
    if c % 32 == 0 and _direct():
        return None
    return torch.empty((rows, 2 * c), dtype=_bf16, device=device)


def note_split(t, sp, bits=None):
    """Register producer-side by-products of ``t``: its [hi | lo] split and/or its ReLU mask bits."""
    if t is None or (sp is None and bits is None):
        return
    key = (t.data_ptr(), tuple(t.shape), tuple(t.stride()))
    _SPLITS[key] = (weakref.ref(t, lambda _r, k=key: _SPLITS.pop(k, None)), t._version, sp, bits)


def _entry(t):
    if t is None or not isinstance(t, torch.Tensor):
        return None
    key = (t.data_ptr(), tuple(t.shape), tuple(t.stride()))
    e = _SPLITS.get(key)
    if e is None:
        return None
    if e[0]() is None or t._version != e[1]:
        _SPLITS.pop(key, None)
        return None
    return e


def _producer_split(t, cp):
    if t is None or t.dim() != 4 or t.shape[1] != cp:
        return None
    e = _entry(t)
    return None if e is None else e[2]


def producer_bits(t):
    """The ReLU mask bits the fp32 BN forward wrote for its output ``t`` (None if absent)."""
    e = _entry(t)
    return None if e is None else e[3]


def _direct() -> bool:
    return bool(config.get_property("bigdl.fp32.direct"))


def _x3_has() -> bool:
    return hasattr(N.lib(), "bigdl_conv_x3") and hasattr(N.lib(), "bigdl_conv_wgrad_f32")


def _al(t) -> bool:
    return t is None or t.data_ptr() % 16 == 0


def _cl_f32(t) -> bool:
    return t.dtype == _f32 and t.dim() == 4 and t.is_contiguous(memory_format=_cl) and t.data_ptr() % 16 == 0


def chunk_split(w_rows: torch.Tensor) -> torch.Tensor:
    """fp32 [rows][n] (n % 32 == 0) → the conv_x3 weight operand: bf16 [rows][n / 32][64], each
    32-index chunk as [hi | lo] (one 128-B LDS row per k-tile)."""
    v = w_rows.reshape(-1, 32)
    if not v.is_contiguous():
        v = v.contiguous()
    return split2(v, 32)


# ---- weight operands of a whole step in one launch (csrc/weight_x3.hip k_wx3_multi) ----------------
# Every filter-derived operand (forward chunks, flipped / transposed dgrad chunks per parity class, the
# s2d stem filter, Linear [hi | lo | hi] rows) is cached per (weight, form).  An entry is valid while
# its weight tensor is alive, its version counter unchanged (torch in-place writes) and it is not
# marked dirty by a native update of the memory it derives from (:func:`mark_dirty`, called by the
# fused optimizer kernels and the DistriOptimizer's weight gathers).  The first access to a dirty
# entry refreshes EVERY dirty entry in one launch, so a training step pays one launch after its update
# instead of ≈120 split / flip / gather launches on the forward and backward critical paths.
_WP: dict = {}          # key → entry dict
_WP_TABLES: dict = {}   # tuple(entry ids) → (device table, total blocks, keep-alive)
_WX_REC = [0]


def _wx_rec_size():
    if not _WX_REC[0]:
        _WX_REC[0] = int(N.lib().bigdl_wx3_job_size())
    return _WX_REC[0]


def _wx_job(buf, i, e, first):
    kind, dims, strides, cls = e["job"]
    K_, C_, R_, S_ = dims
    ia, la = C.c_int * 32, C.c_longlong * 4
    ros, sos, rm, sm, offs = [1] * 4, [1] * 4, [0] * 32, [0] * 32, [0] * 4
    for q, (ro, so, rmap, smap, off) in enumerate(cls):
        ros[q], sos[q], offs[q] = ro, so, off
        rm[q * 8:q * 8 + ro] = rmap
        sm[q * 8:q * 8 + so] = smap
    nb = C.c_longlong(0)
    check(N.lib().bigdl_wx3_job(C.byref(buf, i * _wx_rec_size()), C.c_void_p(e["src"]), ptr(e["out"]), kind, K_, C_,
                                R_, S_,
                                *(C.c_longlong(v) for v in strides), max(1, len(cls)), ia(*ros), ia(*sos), ia(*rm),
                                ia(*sm), la(*offs), C.c_longlong(first), C.byref(nb)), "wx3_job")
    return nb.value


def _wx_run_one(e):
    buf = (C.c_ubyte * _wx_rec_size())()
    _wx_job(buf, 0, e, 0)
    check(N.lib().bigdl_wx3_one(buf, _s()), "wx3_one")


def _wx_refresh_dirty():
    ents = [e for e in _WP.values() if e["dirty"] and e["ref"]() is not None]
    if not ents:
        return
    key = tuple(id(e) for e in ents)
    tab = _WP_TABLES.get(key)
    if tab is None:
        rec = _wx_rec_size()
        buf = (C.c_ubyte * (rec * len(ents)))()
        first = 0
        for i, e in enumerate(ents):
            first += _wx_job(buf, i, e, first)
        host = torch.frombuffer(bytearray(bytes(buf)), dtype=torch.uint8)
        dev = torch.empty(host.numel() + 16, dtype=torch.uint8, device=ents[0]["out"].device)
        off = (-dev.data_ptr()) % 16
        table = dev[off:off + host.numel()]
        table.copy_(host)
        if len(_WP_TABLES) > 64:
            _WP_TABLES.clear()
        tab = _WP_TABLES[key] = (table, first, ents, dev)
    table, total, _e, _keep = tab
    check(N.lib().bigdl_wx3_multi(ptr(table), C.c_int(len(ents)), C.c_longlong(total), _s()), "wx3_multi")
    for e in ents:
        e["dirty"] = False
        e["ver"] = e["ref"]()._version


def mark_dirty(t) -> None:
    """The memory of ``t`` (an fp32 weight buffer or a slice of one) was rewritten by a kernel torch
    does not see (fused optimizer update, weight all-gather): derived operands over it go stale."""
    from ..nn import abstractnn
    abstractnn._MUTATION[0] += 1
    if not _WP or not isinstance(t, torch.Tensor) or not t.is_cuda:
        return
    lo = t.data_ptr()
    hi = lo + t.numel() * t.element_size()
    for e in _WP.values():
        if e["lo"] < hi and lo < e["hi"]:
            e["dirty"] = True


def _wprep(w, form):
    """The bf16 operand of fp32 weight ``w`` in ``form``:
    ("fwd",) → conv_x3 chunks of the KRSC rows; ("s2d",) → the stem's s2d filter chunks; ("c4",) → the
    4-channel stem filter chunks (8 taps × 4 channels per 32-index chunk);
    ("dg", classes) → [view per class] of the flipped, transposed sub-filters, classes = tuple of
    (rmap, smap) tap lists; ("rows3", rows, cp, transposed) → [rows][3·cp] = [hi | lo | hi] of w (or wᵀ)."""
    if not (w.is_cuda and hasattr(N.lib(), "bigdl_wx3_multi")):
        return NotImplemented
    wd = w.detach()
    converted = wd.dtype != _f32
    if converted:
        wd = wd.float()
    root = w._base if w._base is not None else w  # the layer's weight / the parameter arena: stable
    key = (wd.data_ptr(), tuple(wd.shape), tuple(wd.stride()), form)
    capturing = torch.cuda.is_current_stream_capturing()
    e = None if (converted or capturing) else _WP.get(key)
    if e is not None:
        if e["ref"]() is root:
            if e["dirty"] or e["ver"] != w._version:
                e["dirty"] = True
                _wx_refresh_dirty()
            return e["views"]
        _WP.pop(key, None)
    kind = form[0]
    if kind in ("fwd", "s2d", "dg", "c4"):
        k_, c_, r_, s_ = wd.shape
    if kind == "fwd":
        if (r_ * s_ * c_) % 32:
            return NotImplemented
        out = torch.empty(2 * wd.numel(), dtype=_bf16, device=wd.device)
        job = (0, (k_, c_, r_, s_), wd.stride(), ())
        views = out.view(k_, (r_ * s_ * c_) // 32, 64)
    elif kind == "s2d":
        r2, s2 = (r_ + 1) // 2, (s_ + 1) // 2
        if 4 * c_ > 32:
            return NotImplemented
        out = torch.empty(k_ * r2 * s2 * 64, dtype=_bf16, device=wd.device)
        job = (2, (k_, c_, r_, s_), wd.stride(), ())
        views = out.view(k_, r2 * s2, 64)
    elif kind == "c4":
        if c_ > 4 or r_ * s_ > 64:
            return NotImplemented
        kt = (r_ * s_ + 7) // 8
        out = torch.empty(k_ * kt * 64, dtype=_bf16, device=wd.device)
        job = (4, (k_, c_, r_, s_), wd.stride(), ())
        views = out.view(k_, kt, 64)
    elif kind == "dg":
        classes = form[1]
        if k_ % 32 or not 1 <= len(classes) <= 4 or any(len(a) > 8 or len(b) > 8 for a, b in classes):
            return NotImplemented
        cls, off, sizes = [], 0, []
        for rmap, smap in classes:
            n = c_ * len(rmap) * len(smap) * k_ * 2
            cls.append((len(rmap), len(smap), list(rmap), list(smap), off))
            sizes.append(n)
            off += n
        out = torch.empty(off, dtype=_bf16, device=wd.device)
        views = [out[o:o + n].view(c_, n // (2 * c_) // 32, 64)
                 for (_a, _b, _c, _d, o), n in zip(cls, sizes)]
        job = (1, (k_, c_, r_, s_), wd.stride(), tuple(cls))
    elif kind == "rows3":
        rows, cp, tr = form[1], form[2], form[3]
        nr, nc = (wd.shape[1], wd.shape[0]) if tr else (wd.shape[0], wd.shape[1])
        sr, sc = (wd.stride(1), wd.stride(0)) if tr else (wd.stride(0), wd.stride(1))
        if rows < nr or cp % 8 or cp < nc:
            return NotImplemented
        out = torch.empty((rows, 3 * cp), dtype=_bf16, device=wd.device)
        job = (3, (nr, nc, rows, cp), (sr, sc, 0, 0), ())
        views = out
    else:
        raise ValueError(form)
    lo = wd.data_ptr()
    span = 1 + sum((d - 1) * abs(st) for d, st in zip(wd.shape, wd.stride()))
    # the entry keeps no reference to the weight memory (a weak reference to its owner instead), so a
    # freed model releases it; refreshes only ever run over entries whose owner is alive
    e = {"src": lo, "out": out, "views": views, "job": job, "ref": weakref.ref(root), "ver": w._version,
         "dirty": True, "lo": lo, "hi": lo + 4 * span}
    if converted or capturing:
        _wx_run_one(e)  # a converted copy or a HIP-graph capture: recompute per call, no cache
        return views
    dead = [k for k, v in _WP.items() if v["ref"]() is None]
    for k in dead:
        _WP.pop(k, None)
    if dead:
        _WP_TABLES.clear()
    _WP[key] = e
    _wx_refresh_dirty()
    return views


def _x3(x, w2, y, nb, h, w, c, k, r, s, p, q, stride, pad, dil, bias=None, res=None, relu=False, stats=None, rep=0,
        shift=None, bnx=None, mean=None, bits=None, bsc=None, bsh=None, scatter=None, res_strided=None, tile=None,
        persist=0, pro=None):
    """One conv_x3 launch (csrc/conv_x3.hip); ``scatter`` = (osh, osw, ooh, oow, oH, oW) of a
    sub-pixel dgrad, ``res_strided`` = (res_sh, res_sw, res_H, res_W) of a compact residual; ``pro``
    (fp32 [2·C] scale | shift): ``x`` is the input of a training BN + ReLU and the conv reads
    relu(x·scale + shift) — the deferred BN output (bigdl.fp32.bnPrologue)."""
    osh, osw, ooh, oow, oh_, ow_ = scatter if scatter is not None else (1, 1, 0, 0, p, q)
    rsh, rsw, rh, rw = res_strided if res_strided is not None else (0, 0, 0, 0)

    def launch(t, st):
        if pro is not None:
            check(N.lib().bigdl_conv_x3_pro(ptr(x), ptr(w2), ptr(pro), ptr(bias), ptr(res), ptr(y), ptr(st), rep,
                                            ptr(shift), ptr(bnx), ptr(mean), ptr(bits), ptr(bsc), ptr(bsh), nb, h, w,
                                            c, k, r, s, p, q, stride[0], stride[1], pad[0], pad[1], dil[0], dil[1],
                                            int(bool(relu)), k, t[0], t[1], osh, osw, ooh, oow, oh_, ow_, _s()),
                  "conv_x3_pro")
            return
        check(N.lib().bigdl_conv_x3(ptr(x), ptr(w2), ptr(bias), ptr(res), ptr(y), ptr(st), rep, ptr(shift), ptr(bnx),
                                    ptr(mean), ptr(bits), ptr(bsc), ptr(bsh), nb, h, w, c, k, r, s, p, q, stride[0],
                                    stride[1], pad[0], pad[1], dil[0], dil[1], int(bool(relu)), k, t[0], t[1], osh,
                                    osw, ooh, oow, oh_, ow_, rsh, rsw, rh, rw, persist, _s()), "conv_x3")
    if tile is not None:
        launch(tile, stats)
        return
    # the kernel-selection table (training / inference compile phase): candidates per launch geometry
    from .native_ops import _tiled_launch, _stat_target
    key = ("x3", nb, h, w, c, k, r, s, p, q, tuple(stride), tuple(pad), scatter is not None, stats is not None,
           bnx is not None) + (("pro",) if pro is not None else ())

    def fn(t):
        t = (0, 0) if len(t) != 2 else t  # (0, 0, 0): no entry → the launcher's heuristic
        # re-timed after the step: the BN already consumed (and cleared) its replicated sums
        launch(t, None if stats is None else _stat_target(stats, True))
    _tiled_launch(key, fn)


def _x3_geom_ok(c, k, r, s, pad):
    return c % 32 == 0 and k % 8 == 0 and (r * s <= 64 or (r == 1 and s == 1 and tuple(pad) == (0, 0)))


def _w_fwd(w4):
    """The forward filter as conv_x3 chunks: KRSC rows of R·S·C (cached per weight update)."""
    v = _wprep(w4, ("fwd",))
    if v is not NotImplemented:
        return v
    k = w4.shape[0]
    return chunk_split(w4.detach().float().permute(0, 2, 3, 1).reshape(k, -1))


def _w_dgrad(w4, classes):
    """[per class] the flipped, transposed sub-filter chunks of the data gradient: class = (rmap, smap),
    W'[c][i][j][k] = W[k][c][rmap[i]][smap[j]] as rows of C (cached per weight update)."""
    form = ("dg", tuple((tuple(a), tuple(b)) for a, b in classes))
    v = _wprep(w4, form)
    if v is not NotImplemented:
        return v
    wf = w4.detach().float()
    return [chunk_split(wf[:, :, list(a)][:, :, :, list(b)].permute(1, 2, 3, 0).reshape(wf.shape[1], -1))
            for a, b in classes]


def _c4_ok(c, k, r, s, dilation):
    """The C4 stem path (conv_x3.hip MODE 2 forward, conv_wgrad.hip C4 F32 weight gradient) applies."""
    from ..utils import config
    return (c <= 4 and k % 8 == 0 and r * s <= 64 and tuple(dilation) == (1, 1) and _direct() and _x3_has()
            and hasattr(N.lib(), "bigdl_pad4_f32") and bool(config.get_property("bigdl.fp32.stemC4")))


def _stem_ok(c, k, stride, dilation, r=7, s=7):
    if _c4_ok(c, k, r, s, dilation):
        return True
    return (tuple(stride) == (2, 2) and tuple(dilation) == (1, 1) and 4 * c <= 32 and c % 32 != 0 and k % 8 == 0
            and _direct() and _x3_has() and hasattr(N.lib(), "bigdl_s2d_f32"))


def _pad4(x):
    """A ≤ 4-channel fp32 image (any strides) → NHWC [N][H][W][4] fp32, channels ≥ C zero."""
    nb, c, h, w = x.shape
    out = torch.empty((nb, 4, h, w), dtype=_f32, device=x.device, memory_format=_cl)
    xs = x.float()
    check(N.lib().bigdl_pad4_f32(ptr(xs), *(C.c_longlong(v) for v in xs.stride()), nb, c, h, w, ptr(out), _s()),
          "pad4_f32")
    return out


def _s2d(x, pad, r, s, p, q):
    """The space-to-depth image of a stride-2 conv input (csrc/precision.hip k_s2d_f32): fp32
    channels-last [N][32][H2][W2] with channel c·4 + bh·2 + bw = xpad[c][2·h2 + bh][2·w2 + bw]."""
    nb, c, h, w = x.shape
    h2, w2 = p + (r + 1) // 2 - 1, q + (s + 1) // 2 - 1
    out = torch.empty((nb, 32, h2, w2), dtype=_f32, device=x.device, memory_format=_cl)
    xs = x.float()
    check(N.lib().bigdl_s2d_f32(ptr(xs), C.c_longlong(xs.stride(0)), C.c_longlong(xs.stride(1)),
                                C.c_longlong(xs.stride(2)), C.c_longlong(xs.stride(3)), nb, c, h, w, pad[0], pad[1],
                                h2, w2, 32, ptr(out), _s()), "s2d_f32")
    return out


def _stem_weights(w4):
    """[K][C][R][S] → the s2d filter [K][⌈R/2⌉][⌈S/2⌉][32] (KRSC, channel c·4 + bh·2 + bw = tap (2a + bh,
    2a' + bw)), zero-padded taps / channels."""
    k, c, r, s = w4.shape
    r2, s2 = (r + 1) // 2, (s + 1) // 2
    wp = torch.zeros((k, c, 2 * r2, 2 * s2), dtype=_f32, device=w4.device)
    wp[:, :, :r, :s] = w4.detach().float()
    w6 = wp.reshape(k, c, r2, 2, s2, 2).permute(0, 2, 4, 1, 3, 5).reshape(k, r2, s2, 4 * c)
    out = torch.zeros((k, r2, s2, 32), dtype=_f32, device=w4.device)
    out[..., :4 * c] = w6
    return out


def _stem_forward(x, w4, b, stride, pad, relu, stats, rep, shift, slot):
    nb, c, h, w = x.shape
    k, _, r, s = w4.shape
    if _c4_ok(c, k, r, s, (1, 1)):
        p, q = _out_hw(h, w, r, s, stride, pad, (1, 1))
        if p <= 0 or q <= 0:
            return NotImplemented
        xs = _pad4(x)
        if slot is not None:
            slot[0] = (("c4",) + _slot_key(x, 4, True)[1:], xs)
        y = torch.empty((nb, k, p, q), dtype=_f32, device=x.device, memory_format=_cl)
        bias = b.detach().float().reshape(-1).contiguous() if b is not None else None
        w2 = _wprep(w4, ("c4",))
        if w2 is NotImplemented:
            return NotImplemented
        _x3(xs, w2, y, nb, h, w, 4, k, r, s, p, q, tuple(stride), tuple(pad), (1, 1), bias=bias, relu=relu,
            stats=stats, rep=rep, shift=shift)
        return y
    p, q = _out_hw(h, w, r, s, (2, 2), pad, (1, 1))
    if p <= 0 or q <= 0:
        return NotImplemented
    r2, s2 = (r + 1) // 2, (s + 1) // 2
    xs = _s2d(x, pad, r, s, p, q)
    if slot is not None:
        slot[0] = (("s2d",) + _slot_key(x, 32, True)[1:], xs)
    y = torch.empty((nb, k, p, q), dtype=_f32, device=x.device, memory_format=_cl)
    bias = b.detach().float().reshape(-1).contiguous() if b is not None else None
    w2 = _wprep(w4, ("s2d",))
    if w2 is NotImplemented:
        w2 = chunk_split(_stem_weights(w4).reshape(k, -1))
    _x3(xs, w2, y, nb, xs.shape[2], xs.shape[3], 32, k, r2, s2, p, q,
        (1, 1), (0, 0), (1, 1), bias=bias, relu=relu, stats=stats, rep=rep, shift=shift)
    return y


def _stem_wgrad(x, gy, gw_acc, scale, stride, pad, slot):
    """Weight gradient of the stem.  C4 path: the fp32 C4 wgrad over the 4-channel copy of the input
    into a persistent [K][R][S][4] buffer, folded onto the master's taps (and cleared) by one launch.
    s2d path: the fp32 wgrad of the 4×4 stride-1 conv over the s2d image, folded back onto the R×S×C
    taps."""
    nb, c, h, w = x.shape
    k, _, r, s = gw_acc.shape
    p, q = gy.shape[2], gy.shape[3]
    if _c4_ok(c, k, r, s, (1, 1)) and hasattr(N.lib(), "bigdl_c4_wgrad_fold") and gw_acc.dtype == _f32:
        held = slot[0] if slot is not None else None
        key = ("c4",) + _slot_key(x, 4, True)[1:]
        if isinstance(held, tuple) and len(held) == 2 and held[0] == key:
            xs = held[1]
            slot[0] = None
        else:
            xs = _pad4(x)
        bkey = ("c4", gw_acc.data_ptr(), k, r, s, gw_acc.device)
        g4 = _S2D_ACC.get(bkey)
        if g4 is None:
            g4 = _S2D_ACC[bkey] = torch.zeros((k, r, s, 4), dtype=_f32, device=x.device)
        check(N.lib().bigdl_conv_wgrad_f32(ptr(xs), ptr(gy), ptr(g4), C.c_float(1.0), nb, h, w, 4, k, r, s, p, q,
                                           stride[0], stride[1], pad[0], pad[1], 1, 1, 0, _s()), "conv_wgrad_f32(c4)")
        check(N.lib().bigdl_c4_wgrad_fold(ptr(g4), ptr(gw_acc), k, c, r, s, *(C.c_longlong(v) for v in gw_acc.stride()),
                                          C.c_float(float(scale)), _s()), "c4_wgrad_fold")
        return
    r2, s2 = (r + 1) // 2, (s + 1) // 2
    held = slot[0] if slot is not None else None
    key = ("s2d",) + _slot_key(x, 32, True)[1:]
    if isinstance(held, tuple) and len(held) == 2 and held[0] == key:
        xs = held[1]
        slot[0] = None
    else:
        xs = _s2d(x, pad, r, s, p, q)
    fold = hasattr(N.lib(), "bigdl_s2d_wgrad_fold") and gw_acc.dtype == _f32
    bkey = (gw_acc.data_ptr(), k, r2, s2, gw_acc.device)
    gw2 = _S2D_ACC.get(bkey) if fold else None
    if gw2 is None:
        # persistent accumulation buffer (zeroed once; the fold kernel clears what it reads)
        gw2 = torch.zeros((k, r2, s2, 32), dtype=_f32, device=x.device)
        if fold:
            _S2D_ACC[bkey] = gw2
    check(N.lib().bigdl_conv_wgrad_f32(ptr(xs), ptr(gy), ptr(gw2), C.c_float(1.0), nb, xs.shape[2], xs.shape[3], 32, k,
                                       r2, s2, p, q, 1, 1, 0, 0, 1, 1, 0, _s()), "conv_wgrad_f32(s2d)")
    if fold:
        check(N.lib().bigdl_s2d_wgrad_fold(ptr(gw2), ptr(gw_acc), k, c, r, s, *(C.c_longlong(v) for v in gw_acc.stride()),
                                           C.c_float(float(scale)), _s()), "s2d_wgrad_fold")
        return
    g6 = gw2[..., :4 * c].reshape(k, r2, s2, c, 2, 2).permute(0, 3, 1, 4, 2, 5).reshape(k, c, 2 * r2, 2 * s2)
    gw_acc.add_(g6[:, :, :r, :s], alpha=scale)


_S2D_ACC: dict = {}


def pro_ok(x, coef) -> bool:
    """A deferred BN + ReLU output (input ``x``, fp32 [scale | shift] ``coef``) can be consumed by the
    direct kernels' operand prologues (conv_x3 PRO, conv_wgrad F32 PRO)."""
    c = x.shape[1] if x.dim() == 4 else 0
    return (x.dim() == 4 and _cl_f32(x) and c % 32 == 0 and c <= 512 and isinstance(coef, torch.Tensor)
            and coef.dtype == _f32 and coef.numel() == 2 * c and coef.is_contiguous() and coef.data_ptr() % 16 == 0
            and _direct() and _x3_has() and hasattr(N.lib(), "bigdl_conv_x3_pro")
            and hasattr(N.lib(), "bigdl_conv_wgrad_f32_pro"))


def _direct_forward(x, w4, b, stride, pad, dilation, relu, stats=None, rep=0, shift=None, slot=None, pro=None):
    nb, c, h, w = x.shape
    k, _, r, s = w4.shape
    if pro is None and _stem_ok(c, k, stride, dilation, r, s) and x.dtype == _f32:
        return _stem_forward(x, w4, b, stride, pad, relu, stats, rep, shift, slot)
    if not (_direct() and _x3_has() and _x3_geom_ok(c, k, r, s, pad) and _cl_f32(x)):
        return NotImplemented
    if pro is not None and (not pro_ok(x, pro) or tuple(dilation) != (1, 1)):
        return NotImplemented
    p, q = _out_hw(h, w, r, s, stride, pad, dilation)
    if p <= 0 or q <= 0 or not _fits(nb * h * w * c * 4, k * r * s * c * 4):
        return NotImplemented
    y = torch.empty((nb, k, p, q), dtype=_f32, device=x.device, memory_format=_cl)
    bias = b.detach().float().reshape(-1).contiguous() if b is not None else None
    _x3(x, _w_fwd(w4), y, nb, h, w, c, k, r, s, p, q, stride, pad, dilation, bias=bias, relu=relu, stats=stats,
        rep=rep, shift=shift, pro=pro)
    return y


def _act_split(rows2d, cp, two, src=None):
    if two:
        sp = _producer_split(src, cp)
        return sp if sp is not None else split2(rows2d, cp)
    return split(rows2d, cp, HHL, False)


def _conv_f32out2(x2, w3, bias, y, nb, h, w, cp, k, r, s, p, q, stride, pad, dil, relu, ldy, res=None):
    """fp32-output conv of the two-part activation split (logical C = 3·cp)."""
    check(N.lib().bigdl_conv_fwd_f32out2(ptr(x2), ptr(w3), ptr(bias), ptr(res), ptr(y), nb, h, w, 3 * cp, cp, k, r, s,
                                         p, q, stride[0], stride[1], pad[0], pad[1], dil[0], dil[1], int(bool(relu)),
                                         ldy, _s()), "conv_fwd_f32out2")


def _nhwc_rows(x: torch.Tensor) -> torch.Tensor:
    """[N][C][H][W] fp32 → its channels-last storage as a [N·H·W][C] matrix."""
    xc = x.contiguous(memory_format=_cl)
    return xc.permute(0, 2, 3, 1).reshape(-1, x.shape[1])


def _conv_f32out(x3, w3, bias, y, nb, h, w, c3, k, r, s, p, q, stride, pad, dil, relu, ldy, res=None):
    if res is not None:  # fp32 residual summed in the epilogue (same [M][ldy] layout as y)
        check(N.lib().bigdl_conv_fwd_f32out_res(ptr(x3), ptr(w3), ptr(bias), ptr(res), ptr(y), nb, h, w, c3, k, r, s,
                                                p, q, stride[0], stride[1], pad[0], pad[1], dil[0], dil[1],
                                                int(bool(relu)), ldy, _s()), "conv_fwd_f32out_res")
        return
    check(N.lib().bigdl_conv_fwd_f32out(ptr(x3), ptr(w3), ptr(bias), ptr(y), nb, h, w, c3, k, r, s, p, q, stride[0],
                                        stride[1], pad[0], pad[1], dil[0], dil[1], int(bool(relu)), ldy, _s()),
          "conv_fwd_f32out")


def _out_hw(h, w, r, s, stride, pad, dil):
    return ((h + 2 * pad[0] - dil[0] * (r - 1) - 1) // stride[0] + 1,
            (w + 2 * pad[1] - dil[1] * (s - 1) - 1) // stride[1] + 1)


#: bytes one conv operand may span (32-bit buffer offsets in the conv kernels)
_OPERAND_LIMIT = 0x7fffffff


def _fits(*nbytes) -> bool:
    return all(b < 0x80000000 for b in nbytes)  # 32-bit buffer offsets in the conv kernels


def _slot_key(x, cp, two):
    return ("bf16x3", x.data_ptr(), x._version, tuple(x.shape), tuple(x.stride()), cp, two)


def conv_forward(x, w4, b, stride, pad, dilation=(1, 1), groups=1, relu=False, slot=None, pro=None):
    """fp32 NCHW-logical conv (any memory format in, channels-last fp32 out).  ``slot`` (the layer's
    one-entry holder, passed while training): keeps the input split for the weight gradient of the
    same input, which then skips its own split of x.  ``pro``: x is a deferred BN + ReLU output's
    input (see :func:`_x3`); NotImplemented when the direct kernels cannot take it."""
    if groups != 1 or x.dim() != 4 or w4.dim() != 4 or w4.shape[1] != x.shape[1]:
        return NotImplemented
    y = _direct_forward(x, w4, b, stride, pad, dilation, relu, slot=slot, pro=pro)
    if y is not NotImplemented or pro is not None:
        return y
    nb, c, h, w = x.shape
    k, _, r, s = w4.shape
    p, q = _out_hw(h, w, r, s, stride, pad, dilation)
    cp, kq = _r(c, 8), _r(k, 4)
    if p <= 0 or q <= 0 or not _fits(nb * h * w * 3 * cp * 2, kq * r * s * 3 * cp * 2):
        return NotImplemented
    two = _two_part()
    x3 = _act_split(_nhwc_rows(x), cp, two, x)
    if slot is not None:
        slot[0] = (_slot_key(x, cp, two), x3)
    wk = w4.detach().float().permute(0, 2, 3, 1).reshape(k * r * s, c)
    w3 = torch.zeros((kq * r * s, 3 * cp), dtype=_bf16, device=x.device) if kq != k else None
    w3 = split(wk, cp, HLH, False, out=w3)
    bias = None
    if b is not None:
        bias = torch.zeros(kq, dtype=_f32, device=x.device)
        bias[:k] = b.detach().float().reshape(-1)
    y = torch.empty((nb, kq, p, q), dtype=_f32, device=x.device, memory_format=_cl)
    if two:
        _conv_f32out2(x3, w3, bias, y, nb, h, w, cp, kq, r, s, p, q, stride, pad, dilation, relu, kq)
    else:
        _conv_f32out(x3, w3, bias, y, nb, h, w, 3 * cp, kq, r, s, p, q, stride, pad, dilation, relu, kq)
    if kq != k:
        y = y[:, :k].contiguous(memory_format=_cl)
    return y


def conv_forward_stats(x, w4, stride, pad, dilation, sums, shift, slot=None, pro=None):
    """fp32 conv (no bias / ReLU) whose epilogue also ADDS the following BN's statistics
    Σ(y − shift), Σ(y − shift)² into the BN's replicated buffer ``sums = (buf [2][R][K], R)``: returns
    ``(y, buf, R)`` for ``batchnorm_forward_train_partials`` (which finalizes from the R rows and clears
    them), or NotImplemented."""
    if (x.dim() != 4 or w4.dim() != 4 or w4.shape[1] != x.shape[1] or not _two_part() or not isinstance(sums, tuple)
            or not config.get_property("bigdl.fp32.convStats")):
        return NotImplemented
    nb, c, h, w = x.shape
    k, _, r, s = w4.shape
    buf, rep = sums
    if (k % 8 or shift is None or shift.dtype != _f32 or shift.numel() != k or not shift.is_contiguous()
            or buf.dtype != _f32 or buf.numel() != 2 * rep * k or not 1 <= rep <= 512):
        return NotImplemented
    y = _direct_forward(x, w4, None, stride, pad, dilation, False, stats=buf, rep=rep, shift=shift, slot=slot,
                        pro=pro)
    if y is not NotImplemented:
        return y, buf, rep
    if pro is not None:
        return NotImplemented
    p, q = _out_hw(h, w, r, s, stride, pad, dilation)
    cp = _r(c, 8)
    if p <= 0 or q <= 0 or not _fits(nb * h * w * 2 * cp * 2, k * r * s * 3 * cp * 2):
        return NotImplemented
    x3 = _act_split(_nhwc_rows(x), cp, True, x)
    if slot is not None:
        slot[0] = (_slot_key(x, cp, True), x3)
    w3 = split(w4.detach().float().permute(0, 2, 3, 1).reshape(k * r * s, c), cp, HLH, False)
    y = torch.empty((nb, k, p, q), dtype=_f32, device=x.device, memory_format=_cl)
    check(N.lib().bigdl_conv_fwd_f32out2_stats(ptr(x3), ptr(w3), ptr(y), ptr(buf), rep, ptr(shift), nb, h, w, 3 * cp,
                                               cp, k, r, s, p, q, stride[0], stride[1], pad[0], pad[1], dilation[0],
                                               dilation[1], _s()), "conv_fwd_f32out2_stats")
    return y, buf, rep


def _bnbwd_args(bn_fuse, nb, c, h, w, res):
    """The fp32 BN-backward statistics a data gradient can add in its epilogue (conv.py bn_fuse):
    (buf, R, bn input, mean, bits, scale, shift) or None."""
    if bn_fuse is None or not config.get_property("bigdl.fp32.convStats") or c % 8:
        return None
    sums, bx, mean = bn_fuse.get("sums"), bn_fuse.get("x"), bn_fuse.get("mean")
    if not isinstance(sums, tuple) or not isinstance(bx, torch.Tensor) or not isinstance(mean, torch.Tensor):
        return None
    buf, rep = sums
    if (buf.dtype != _f32 or buf.numel() != 2 * rep * c or not 1 <= rep <= 512 or bx.dtype != _f32
            or tuple(bx.shape) != (nb, c, h, w) or not bx.is_contiguous(memory_format=_cl) or bx.data_ptr() % 16
            or mean.dtype != _f32 or mean.numel() != c):
        return None
    sc, sh, bits = bn_fuse.get("scale"), bn_fuse.get("shift"), None
    if "mask" in bn_fuse:  # a block tail: the forward's ReLU mask bits of its output
        bits = producer_bits(bn_fuse["mask"])
        if bits is None or res is None:
            return None
        sc = sh = None
    elif not (isinstance(sc, torch.Tensor) and isinstance(sh, torch.Tensor) and res is None):
        return None
    return buf, rep, bx, mean, bits, sc, sh


_PARITY: dict = {}


def _parity(h, w, r, s, stride, pad):
    key = (h, w, r, s, tuple(stride), tuple(pad))
    cl = _PARITY.get(key)
    if cl is None:
        from .native_ops import _parity_classes
        cl = _PARITY[key] = _parity_classes(h, w, r, s, stride[0], stride[1], pad[0], pad[1])
    return cl


def _direct_dgrad(gy, w4, x_shape, stride, pad, dilation, residual, bn_fuse, lazy):
    """fp32 data gradient on conv_x3: a stride-1 conv of dY with the flipped, transposed filter
    (C·R·S rows of K); strided convs by sub-pixel decomposition (one scatter launch per parity class
    that receives taps).  Returns gi, a StridedGrad (``lazy`` 1×1 stride-s), or NotImplemented."""
    from .reference import StridedGrad
    nb, c, h, w = x_shape
    k, _, r, s = w4.shape
    p, q = gy.shape[2], gy.shape[3]
    if tuple(dilation) != (1, 1) or k % 32 or c % 8 or not _cl_f32(gy):
        return NotImplemented
    if not _fits(nb * p * q * k * 4, c * r * s * k * 4, nb * h * w * c * 4):
        return NotImplemented
    res_strided = None
    if isinstance(residual, StridedGrad):
        rt = residual.t
        if not (rt.dtype == _f32 and _cl_f32(rt) and rt.shape[0] == nb and rt.shape[1] == c
                and tuple(residual.shape) == (nb, c, h, w)):
            residual = residual.dense()
        else:
            res_strided = (residual.stride[0], residual.stride[1], rt.shape[2], rt.shape[3])
            residual = rt
    if residual is not None and res_strided is None and not (residual.dtype == _f32 and _cl_f32(residual)
                                                             and tuple(residual.shape) == (nb, c, h, w)):
        return NotImplemented
    bnb = _bnbwd_args(bn_fuse, nb, c, h, w, residual) if bn_fuse is not None else None
    if bn_fuse is not None and bnb is None:
        bn_fuse = None
    if tuple(stride) == (1, 1):
        pd = (r - 1 - pad[0], s - 1 - pad[1])
        if pd[0] < 0 or pd[1] < 0 or not _x3_geom_ok(k, c, r, s, pd) or (h, w) != (p + 2 * pd[0] - r + 1,
                                                                                 q + 2 * pd[1] - s + 1):
            return NotImplemented
        wt = _w_dgrad(w4, [(tuple(range(r - 1, -1, -1)), tuple(range(s - 1, -1, -1)))])[0]  # [C][R][S][K]
        gi = torch.empty((nb, c, h, w), dtype=_f32, device=gy.device, memory_format=_cl)
        if bnb is not None:
            buf, rep, bx, mean, bits, bsc, bsh = bnb
            _x3(gy, wt, gi, nb, p, q, k, c, r, s, h, w, (1, 1), pd, (1, 1), res=residual, stats=buf,
                rep=rep, bnx=bx, mean=mean, bits=bits, bsc=bsc, bsh=bsh, res_strided=res_strided)
            bn_fuse["partial"], bn_fuse["G"] = buf, rep
        else:
            _x3(gy, wt, gi, nb, p, q, k, c, r, s, h, w, (1, 1), pd, (1, 1), res=residual,
                res_strided=res_strided)
        return gi
    if res_strided is not None:
        return NotImplemented
    classes = _parity(h, w, r, s, stride, pad)
    live = [cl for cl in classes if cl[2] and cl[3]]
    if not live or any(not _x3_geom_ok(k, c, len(cl[2]), len(cl[3]), (len(cl[2]) - 1 - cl[6], len(cl[3]) - 1 - cl[7]))
                       for cl in live):
        return NotImplemented
    covered = len(live) == len(classes) and sum(cl[4] * cl[5] for cl in live) == h * w
    if bnb is not None and not covered:  # tap-less pixels would miss the BN-backward sums
        return NotImplemented
    subs = _w_dgrad(w4, [(tuple(rs[::-1]), tuple(ss[::-1])) for (a, b, rs, ss, *_r) in live])
    if lazy and residual is None and r == 1 and s == 1 and tuple(pad) == (0, 0) and len(live) == 1:
        (a, b, rs, ss, ho, wo, ea, eb) = live[0]
        tmp = torch.empty((nb, c, ho, wo), dtype=_f32, device=gy.device, memory_format=_cl)
        _x3(gy, subs[0], tmp, nb, p, q, k, c, 1, 1, ho, wo, (1, 1), (0, 0), (1, 1))
        return StridedGrad(tmp, tuple(stride), (nb, c, h, w))
    gi = torch.empty((nb, c, h, w), dtype=_f32, device=gy.device, memory_format=_cl)
    if not covered:
        if residual is not None:
            gi.copy_(residual)
        else:
            gi.zero_()
    # every parity class adds its pixels' share of the BN-backward sums (disjoint pixel sets)
    bn_kw = {}
    if bnb is not None:
        buf, rep, bx, mean, bits, bsc, bsh = bnb
        bn_kw = dict(stats=buf, rep=rep, bnx=bx, mean=mean, bits=bits, bsc=bsc, bsh=bsh)
    for (a, b, rs, ss, ho, wo, ea, eb), sub in zip(live, subs):
        ra, sb = len(rs), len(ss)
        _x3(gy, sub, gi, nb, p, q, k, c, ra, sb, ho, wo, (1, 1), (ra - 1 - ea, sb - 1 - eb), (1, 1),
            res=residual, scatter=(stride[0], stride[1], a, b, h, w), **bn_kw)
    if bnb is not None:
        bn_fuse["partial"], bn_fuse["G"] = bnb[0], bnb[1]
    return gi


def _direct_wgrad_ok(x, gy, gw_acc) -> bool:
    nb, c, h, w = x.shape
    k = gw_acc.shape[0]
    p, q = gy.shape[2], gy.shape[3]
    return (_direct() and _x3_has() and c % 8 == 0 and k % 8 == 0 and _cl_f32(x) and _cl_f32(gy)
            and gw_acc.dtype == _f32 and gw_acc.permute(0, 2, 3, 1).is_contiguous()
            and _fits(nb * h * w * c * 4, nb * p * q * k * 4))


def bias_grad_acc(gy, gb_acc, scale):
    """gb += scale · Σ_{n,h,w} dY (the conv bias gradient) on the fp32 column-sum kernel; torch's
    reduction only for a layout the kernel does not take."""
    from .native_ops import colsum_acc
    k = gy.shape[1]
    if (gy.dim() == 4 and _cl_f32(gy) and gb_acc.dtype == _f32 and gb_acc.is_contiguous()
            and colsum_acc(gy.permute(0, 2, 3, 1).reshape(-1, k), gb_acc.view(-1), scale) is not NotImplemented):
        return
    gb_acc.add_(gy.sum((0, 2, 3)).reshape(gb_acc.shape), alpha=scale)


def _direct_wgrad(x, gy, gw_acc, scale, stride, pad, dilation, pro=None):
    nb, c, h, w = x.shape
    k, _, r, s = gw_acc.shape
    p, q = gy.shape[2], gy.shape[3]
    if not _direct_wgrad_ok(x, gy, gw_acc) or (pro is not None and not pro_ok(x, pro)):
        return NotImplemented
    def fn(t):
        # t = (splits,): 0 = the launcher's heuristic (≈512 blocks), < 0 = -target block count
        sp = t[0] if len(t) == 1 else 0
        if pro is not None:
            check(N.lib().bigdl_conv_wgrad_f32_pro(ptr(x), ptr(pro), ptr(gy), ptr(gw_acc), C.c_float(float(scale)), nb,
                                                   h, w, c, k, r, s, p, q, stride[0], stride[1], pad[0], pad[1],
                                                   dilation[0], dilation[1], sp, _s()), "conv_wgrad_f32_pro")
            return
        check(N.lib().bigdl_conv_wgrad_f32(ptr(x), ptr(gy), ptr(gw_acc), C.c_float(float(scale)), nb, h, w, c, k, r,
                                           s, p, q, stride[0], stride[1], pad[0], pad[1], dilation[0], dilation[1],
                                           sp, _s()), "conv_wgrad_f32")
    from .native_ops import _tiled_launch
    _tiled_launch(("wg32", nb, h, w, c, k, r, s, p, q, tuple(stride), tuple(pad))
                  + (("pro",) if pro is not None else ()), fn)
    return None


def conv_backward(gy, x, w4, stride, pad, dilation=(1, 1), groups=1, need_input=True, gw_acc=None, gb_acc=None,
                  scale=1.0, residual=None, slot=None, bn_fuse=None, lazy_strided=False, pro=None):
    """Data gradient (fp32, channels-last) and fp32 weight / bias gradient accumulation.  ``bn_fuse``
    (conv.py: the BN + ReLU whose output this conv consumed): the data gradient's epilogue stores the
    ReLU-masked gradient and adds that BN's backward statistics into its replicated buffer, reported
    back as ``bn_fuse["partial"], bn_fuse["G"]``.  ``residual`` may be a StridedGrad (summed as a
    compact strided residual by the direct kernels); ``lazy_strided``: a 1×1 stride-s conv may return
    its input gradient as a StridedGrad."""
    if groups != 1 or x.dim() != 4 or gy.dim() != 4 or gy.dtype != _f32:
        return NotImplemented
    if pro is not None:
        # x is a deferred BN + ReLU output's input: only the weight gradient reads x (through the F32
        # prologue); the data gradient never does
        if not (_direct() and _x3_has() and _cl_f32(gy) and pro_ok(x, pro)):
            return NotImplemented
        if gw_acc is not None and scale != 0 and not _direct_wgrad_ok(x, gy, gw_acc):
            return NotImplemented
    if (pro is None and not need_input and gw_acc is not None
            and _stem_ok(x.shape[1], w4.shape[0], stride, dilation, w4.shape[2], w4.shape[3])
            and _cl_f32(gy) and x.dtype == _f32 and gw_acc.dtype == _f32):
        if scale != 0:
            from .native_ops import _wgrad_side_stream
            side = _wgrad_side_stream(gy)
            if side is not None:
                with torch.cuda.stream(side):
                    _stem_wgrad(x, gy, gw_acc, scale, stride, pad, slot)
                    if gb_acc is not None:
                        bias_grad_acc(gy, gb_acc, scale)
                for t in (x, gy):
                    t.record_stream(side)
            else:
                _stem_wgrad(x, gy, gw_acc, scale, stride, pad, slot)
                if gb_acc is not None:
                    bias_grad_acc(gy, gb_acc, scale)
        return None
    if _direct() and _x3_has() and _cl_f32(gy) and x.dtype == _f32:
        # each half independently on the direct kernels when its shape allows, else on the split path.
        # The one-launch fp32 weight gradient is forked onto the wgrad side stream BEFORE the data
        # gradient (as the bf16 path does, native_ops.conv2d_backward), so it runs beside the
        # backward-data chain; the optimizer joins the side stream before the update.
        wg_done = False
        if gw_acc is not None and scale != 0 and _direct_wgrad_ok(x, gy, gw_acc):
            from .native_ops import _wgrad_side_stream
            side = _wgrad_side_stream(gy)
            if side is not None:
                with torch.cuda.stream(side):
                    _direct_wgrad(x, gy, gw_acc, scale, stride, pad, dilation, pro=pro)
                    if gb_acc is not None:
                        bias_grad_acc(gy, gb_acc, scale)
                for t in (x, gy) + ((pro,) if pro is not None else ()):
                    t.record_stream(side)
                wg_done = True
        gi = None
        if need_input:
            gi = _direct_dgrad(gy, w4, tuple(x.shape), stride, pad, dilation, residual, bn_fuse, lazy_strided)
            if gi is NotImplemented:
                if pro is not None:
                    # (the split path's dgrad never reads x: it only needs x's shape)
                    gi = _split_backward(gy, x, w4, stride, pad, dilation, True, None, scale, None, residual,
                                         bn_fuse)
                else:
                    gi = _split_backward(gy, x, w4, stride, pad, dilation, True, None, scale, slot, residual, bn_fuse)
                if gi is NotImplemented:
                    return NotImplemented
        if gw_acc is not None and scale != 0 and not wg_done:
            if _direct_wgrad(x, gy, gw_acc, scale, stride, pad, dilation, pro=pro) is NotImplemented:
                if pro is not None:
                    raise RuntimeError("fp32 BN prologue: the weight gradient lost its direct kernel mid-call")
                r = _split_backward(gy, x, w4, stride, pad, dilation, False, gw_acc, scale, slot)
                if r is NotImplemented:
                    return NotImplemented
            if gb_acc is not None:
                bias_grad_acc(gy, gb_acc, scale)
        elif gb_acc is not None and scale != 0 and not wg_done:
            bias_grad_acc(gy, gb_acc, scale)
        return gi
    return _split_backward_full(gy, x, w4, stride, pad, dilation, need_input, gw_acc, gb_acc, scale, residual, slot,
                                bn_fuse)



def _split_backward(gy, x, w4, stride, pad, dilation, need_input, gw_acc, scale, slot, residual=None, bn_fuse=None):
    return _split_backward_full(gy, x, w4, stride, pad, dilation, need_input, gw_acc, None, scale, residual, slot,
                                bn_fuse)


def _split_backward_full(gy, x, w4, stride, pad, dilation, need_input, gw_acc, gb_acc, scale, residual, slot,
                         bn_fuse):
    """The split-operand backward (materialised [hi | lo] splits of dY and x)."""
    from .reference import StridedGrad
    if isinstance(residual, StridedGrad):
        residual = residual.dense()
    nb, c, h, w = x.shape
    k, _, r, s = w4.shape
    p, q = gy.shape[2], gy.shape[3]
    kp, cq, cp = _r(k, 8), _r(c, 4), _r(c, 8)
    gi = None
    two = _two_part()
    g3 = None
    if need_input:
        hl, wl = h + 2 * pad[0] - dilation[0] * (r - 1), w + 2 * pad[1] - dilation[1] * (s - 1)
        pd = (dilation[0] * (r - 1) - pad[0], dilation[1] * (s - 1) - pad[1])
        npart = 2 if two else 3
        if pd[0] < 0 or pd[1] < 0 or not _fits(hl * wl * npart * kp * 2, cq * r * s * 3 * kp * 2):
            return NotImplemented
        strided = tuple(stride) != (1, 1)
        if not strided and (hl, wl) != (p, q):
            return NotImplemented
        # images per launch: the dY operand must stay below the kernels' 2 GiB buffer offsets (the
        # 224² stem's lattice at batch 256 does not), so large batches run in image chunks
        nbc = min(nb, _OPERAND_LIMIT // (hl * wl * npart * kp * 2))
        if nbc < nb and cq <= 4:
            # the RGB stem at ImageNet batch sizes: a 4-channel data gradient leaves the MFMA tiles almost
            # idle and the lattice + splits cost more than torch's fp32 kernel (measured 1.8 vs 0.9 ms/step
            # for data + weight gradient, profiles/r4_fp32_profile.txt), so that one conv stays on torch
            return NotImplemented
        wt = w4.detach().float().flip(2, 3).permute(1, 2, 3, 0).reshape(c * r * s, k)  # [C][R][S][K]
        wt3 = torch.zeros((cq * r * s, 3 * kp), dtype=_bf16, device=x.device) if cq != c else None
        wt3 = split(wt, kp, HLH, False, out=wt3)
        gi = torch.empty((nb, cq, h, w), dtype=_f32, device=x.device, memory_format=_cl)
        # the shortcut's gradient summed in the epilogue (one pass fewer than a separate add)
        fuse_res = (residual is not None and cq == c and residual.dtype == _f32 and tuple(residual.shape) == (nb, c, h, w)
                    and residual.is_contiguous(memory_format=_cl) and residual.data_ptr() % 16 == 0)
        whole = _producer_split(gy, kp) if (two and not strided) else None
        bnb = _bnbwd_args(bn_fuse, nb, c, h, w, residual if fuse_res else None) if (two and nbc == nb
                                                                                    and cq == c) else None
        for i0 in range(0, nb, nbc):
            i1 = min(nb, i0 + nbc)
            gyc = gy if (i0, i1) == (0, nb) else gy[i0:i1]
            if strided:  # dY on the stride lattice (zeros between), then a stride-1 conv
                src = torch.empty((i1 - i0, k, hl, wl), dtype=_f32, device=gy.device, memory_format=_cl).zero_()
                src[:, :, ::stride[0], ::stride[1]] = gyc
            else:
                src = gyc
            if whole is not None:
                g3c = whole[i0 * p * q:i1 * p * q]
            else:
                g3c = _act_split(_nhwc_rows(src), kp, two, src)
            gic = gi if (i0, i1) == (0, nb) else gi[i0:i1]
            resc = (residual if (i0, i1) == (0, nb) else residual[i0:i1]) if fuse_res else None
            if bnb is not None:
                buf, rep, bx, mean, bits, bsc, bsh = bnb
                check(N.lib().bigdl_conv_fwd_f32out2_bnbwd(
                    ptr(g3c), ptr(wt3), ptr(resc), ptr(gic), ptr(buf), rep, ptr(bx), ptr(mean), ptr(bits), ptr(bsc),
                    ptr(bsh), i1 - i0, hl, wl, 3 * kp, kp, cq, r, s, h, w, 1, 1, pd[0], pd[1], dilation[0],
                    dilation[1], _s()), "conv_fwd_f32out2_bnbwd")
                bn_fuse["partial"], bn_fuse["G"] = buf, rep
            elif two:
                _conv_f32out2(g3c, wt3, None, gic, i1 - i0, hl, wl, kp, cq, r, s, h, w, (1, 1), pd, dilation, False,
                              cq, res=resc)
            else:
                _conv_f32out(g3c, wt3, None, gic, i1 - i0, hl, wl, 3 * kp, cq, r, s, h, w, (1, 1), pd, dilation,
                             False, cq, res=resc)
            if (i0, i1) == (0, nb) and not strided:
                g3 = g3c  # the wgrad reuses the whole dY split
        if cq != c:
            gi = gi[:, :c].contiguous(memory_format=_cl)
        if residual is not None and not fuse_res:
            gi.add_(residual)
    if gw_acc is not None and scale != 0:
        # three launches over the side-by-side parts — (x_hi, dY_hi), (x_hi, dY_lo), (x_lo, dY_hi) —
        # each a channel slice (pixel stride 2·Cp / 2·Kp of the [hi | lo] splits, 3·Cp / 3·Kp of the
        # three-part ones); a stride-1 conv reuses the data gradient's split of dY
        npart = 2 if two else 3
        if not _fits(nb * h * w * npart * cp * 2, nb * p * q * npart * kp * 2):
            return NotImplemented
        held = slot[0] if slot is not None else None
        if isinstance(held, tuple) and len(held) == 2 and held[0] == _slot_key(x, cp, two):
            x3 = held[1]  # the forward's split of this same input
            slot[0] = None
        else:
            x3 = _act_split(_nhwc_rows(x), cp, two, x)
        gy3 = g3 if g3 is not None else _act_split(_nhwc_rows(gy), kp, two, gy)
        direct = cp == c and kp == k and gw_acc.dtype == _f32 and gw_acc.permute(0, 2, 3, 1).is_contiguous()
        target = gw_acc.permute(0, 2, 3, 1) if direct else torch.zeros((kp, r, s, cp), dtype=_f32, device=x.device)
        sc = C.c_float(float(scale) if direct else 1.0)
        lo = npart - 1  # the lo part's index in the stored split
        for xq, gq in ((0, 0), (0, lo), (lo, 0)):
            check(N.lib().bigdl_conv_wgrad_grouped(C.c_void_p(x3.data_ptr() + 2 * xq * cp),
                                                   C.c_void_p(gy3.data_ptr() + 2 * gq * kp), ptr(target), sc, nb, h,
                                                   w, npart * cp, cp, npart * kp, kp, 1, r, s, p, q, stride[0], stride[1],
                                                   pad[0], pad[1], dilation[0], dilation[1], _s()),
                  "conv_wgrad(bf16x3)")
        if not direct:
            gw_acc.add_(target[:k, :, :, :c].permute(0, 3, 1, 2), alpha=scale)
    if gb_acc is not None and scale != 0:
        bias_grad_acc(gy, gb_acc, scale)
    return gi


def _gemm_f32(a3, b3, m, n4, bias=None, act=0):
    from .native_ops import gemm
    out = torch.empty((m, n4), dtype=_f32, device=a3.device)
    return gemm(a3, b3, bias, act=act, out=out)


def linear_forward(x, w, b, act=0):
    """y = act(x·Wᵀ + b), fp32 in / out."""
    if x.dim() != 2 or w.dim() != 2 or x.shape[1] != w.shape[1] or x.shape[0] == 0:
        return NotImplemented
    m, k = x.shape
    n = w.shape[0]
    k8, n4 = _r(k, 8), _r(n, 4)
    a3 = split(x, k8, HHL, False)
    b3 = _wprep(w, ("rows3", n4, k8, False))
    if b3 is NotImplemented:
        b3 = split(w.detach().float(), k8, HLH, False,
                   out=torch.zeros((n4, 3 * k8), dtype=_bf16, device=x.device) if n4 != n else None)
    bias = None
    if b is not None:
        bias = b.detach().reshape(-1)
        if n4 != n or bias.dtype != _f32 or not bias.is_contiguous() or bias.data_ptr() % 16:  # float4 epilogue reads
            bias = torch.zeros(n4, dtype=_f32, device=x.device)
            bias[:n] = b.detach().float().reshape(-1)
    y = _gemm_f32(a3, b3, m, n4, bias, act)
    if y is NotImplemented:
        return NotImplemented
    return y if n4 == n else y[:, :n].contiguous()


def linear_backward(gy, x, w, need_input=True, gw_acc=None, gb_acc=None, scale=1.0):
    if gy.dim() != 2 or x.dim() != 2 or w.dim() != 2 or gy.dtype != _f32:
        return NotImplemented
    m, n = gy.shape
    k = x.shape[1]
    n8, k4, k8 = _r(n, 8), _r(k, 4), _r(k, 8)
    gi = None
    two = _two_part()
    if need_input:
        g3 = split(gy, n8, HHL, False)
        wt3 = _wprep(w, ("rows3", k4, n8, True))
        if wt3 is NotImplemented:
            wt3 = split(w.detach().float().t(), n8, HLH, False,
                        out=torch.zeros((k4, 3 * n8), dtype=_bf16, device=gy.device) if k4 != k else None)
        gi = _gemm_f32(g3, wt3, m, k4)
        if gi is NotImplemented:
            return NotImplemented
        if k4 != k:
            gi = gi[:, :k].contiguous()
    if gw_acc is not None and scale != 0:
        from .native_ops import wgrad_rows
        g3 = split(gy, n8, HLH, True)   # [3M][N8] = [hi; lo; hi]
        x3 = split(x, k8, HHL, True)    # [3M][K8] = [hi; hi; lo]
        direct = n8 == n and k8 == k and gw_acc.dtype == _f32 and gw_acc.is_contiguous()
        tgt = gw_acc if direct else torch.zeros((n8, k8), dtype=_f32, device=gy.device)
        if wgrad_rows(g3, x3, tgt, scale if direct else 1.0) is NotImplemented:
            return NotImplemented
        if not direct:
            gw_acc.add_(tgt[:n, :k].reshape(gw_acc.shape), alpha=scale)
    if gb_acc is not None and scale != 0:
        from .native_ops import colsum_acc
        if not (gb_acc.dtype == _f32 and gb_acc.is_contiguous()
                and colsum_acc(gy, gb_acc.view(-1), scale) is not NotImplemented):
            gb_acc.add_(gy.sum(0).reshape(gb_acc.shape), alpha=scale)
    return gi
