"""int8 inference layers (``DL/nn/quantized/{Linear,SpatialConvolution,SpatialDilatedConvolution}.scala``).

Weights are quantised once, per output channel (``Quantization.quantize`` on the 2-D
``(out, in·kh·kw)`` view).  At run time every GEMM row of the input — an FC input row, or a conv
im2col window, BigQuant's "per-window" quantisation — gets its own scale; the product runs on the
int8 MFMA GEMM (``ops.gemm_i8``) with the dequantisation (row scale × channel scale + bias) fused
into its epilogue.  Backward is not supported (inference only), as in the reference.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ...utils import acc_float

from ... import ops
from ..abstractnn import TensorModule


def _kp(k: int) -> int:
    return (k + 63) // 64 * 64


def calibrated_scale(m):
    """The static activation scale clip / 127 of a float module's calibrated input, or None when the
    module was never calibrated.  ``bigdl.int8.calibration``: "max" clips at the largest max|x| over
    the calibration batches (``MklInt8Convertible``'s rule); "p99.9" / "p99.99" / "p99.999" at that
    percentile of |x| (the largest over the batches) — saturating the few outliers buys the bulk of a
    heavy-tailed ReLU activation finer steps."""
    from ...utils import config
    from ..int8_convertible import PERCENTILES
    st = m.__dict__.get("_int8_state")
    if not st or not st.get("in") or st.get("inMask", 0) != 0:
        return None
    amax = max(float(v[0]) for v in st["in"] if v)
    rule = str(config.get_property("bigdl.int8.calibration"))
    if rule.startswith("p") and st.get("in_pct"):
        try:
            i = PERCENTILES.index(float(rule[1:]))
        except ValueError:
            i = None
        if i is not None:
            clip = max(float(v[i]) for v in st["in_pct"])
            if clip > 0:
                amax = min(amax, clip)
    return amax / 127.0 if amax > 0 else None


def dequant(x):
    """An int8 activation tagged ``_qscale`` (and ``_qzero`` for the offset unsigned code) back to
    bf16 (the layer after a chain end that cannot consume int8)."""
    return ((x.float() + getattr(x, "_qzero", 0)) * x._qscale).to(torch.bfloat16)


def _retag(y, x):
    """Carry the quantisation tags of ``x`` over to a view ``y`` of it."""
    for k in ("_qscale", "_qzero", "_qtail"):
        v = getattr(x, k, None)
        if v is not None:
            setattr(y, k, v)
    return y


class _QuantizedBase(TensorModule):
    SCALA_PACKAGE = "com.intel.analytics.bigdl.nn.quantized"
    #: calibrated input scale (static quantisation; None = per-image dynamic scales)
    static_scale = None
    #: set by the quantizer when the next layer of the chain is a quantised conv with a static
    #: scale: this layer writes int8 requantised with it ...
    _out_qscale = None
    #: ... and applies the ReLU that follows it in the epilogue
    _relu_fused = False
    #: the ReLU'd int8 output uses the unsigned code (offset −128, ``_out_qscale`` = clip / 255)
    _out_u8 = False

    def _quantize_weight(self, w2d: torch.Tensor):
        q, s = ops.reference.quant_rows(w2d.detach().float().cpu())
        self.register_buffer("qweight", q)
        self.register_buffer("weight_scale", s.float())

    def _gemm(self, rows: torch.Tensor, out_dtype):
        qa, sa = ops.quant_rows(rows.contiguous(), self.qweight.shape[1])
        return ops.gemm_i8(qa, sa, self.qweight, self.weight_scale, self.bias_f, out_dtype=out_dtype)

    def updateGradInput(self, input, gradOutput):
        raise NotImplementedError(f"Doesn't updateGradInput for quantized model ({type(self).__name__})")

    def accGradParameters(self, input, gradOutput):
        pass

    def parameters(self):
        return None

    @property
    def bias_f(self):
        return getattr(self, "qbias", None)


class Linear(_QuantizedBase):
    def __init__(self, input_size: int, output_size: int, with_bias: bool = True):
        super().__init__()
        self.inputSize, self.outputSize, self.withBias = input_size, output_size, with_bias
        self.register_buffer("qweight", torch.zeros(output_size, _kp(input_size), dtype=torch.int8))
        self.register_buffer("weight_scale", torch.zeros(output_size))
        if with_bias:
            self.register_buffer("qbias", torch.zeros(output_size))

    @staticmethod
    def from_float(m) -> "Linear":
        q = Linear(m.inputSize, m.outputSize, m.bias is not None)
        q._quantize_weight(m.weight)
        if m.bias is not None:
            q.qbias = m.bias.detach().float().clone().cpu()
        q.static_scale = calibrated_scale(m)
        q.set_name(m.get_name())
        return q.to(m.weight.device)

    def _u8_bias(self, sx, dev):
        """The bias with the offset term of an unsigned (offset −128) int8 input of scale ``sx``:
        128·sx·sw[n]·Σ_k w[n][k] (padding columns are 0), cached per (device, scale)."""
        key = (dev, sx)
        t = getattr(self, "_lin_u8", None)
        if t is None or t[0] != key:
            w = self.qweight.to(dev).to(torch.int32).sum(-1).double()
            b = self.bias_f.to(dev).double() if self.bias_f is not None else torch.zeros_like(w)
            t = self._lin_u8 = (key, (b + 128.0 * w * float(sx) * self.weight_scale.to(dev).double()).float())
        return t[1]

    def _native_static(self, x):
        """Calibrated int8 path (the reference's int8 FC, quantized/Linear.scala, with MKL-DNN's static
        scales): an int8 input from the chain (tagged ``_qscale``) is used as is, an fp32 / bf16 input is
        quantised with the calibrated scale in one pass; split-K int8 GEMM with bias, ReLU and — when
        the next layer is a quantised Linear — the requantised int8 output in its epilogue."""
        from ...ops import native_ops as NO
        if not (x.is_cuda and x.dim() == 2 and ops.native_has("gemm_i8")):
            return NotImplemented
        M, K = x.shape
        kp = self.qweight.shape[1]
        dev = x.device
        if x.dtype == torch.int8:
            sx = getattr(x, "_qscale", None)
            if sx is None:
                return NotImplemented
            z = getattr(x, "_qzero", 0)
            qa = x.contiguous()
        elif self.static_scale is not None and x.dtype in (torch.float32, torch.bfloat16):
            sx, z = self.static_scale, 0
            qa = NO.quant_static(x.contiguous(), sx)
            if qa is NotImplemented:
                return NotImplemented
        else:
            return NotImplemented
        if kp != K:
            qa = torch.nn.functional.pad(qa, (0, kp - K))  # weight padding columns are 0
        qw = self.qweight if self.qweight.device == dev else self.qweight.to(dev)
        bias = self._u8_bias(sx, dev) if z else (self.bias_f.to(dev) if self.bias_f is not None else None)
        return NO.gemm_i8_static(qa, sx, qw, self.weight_scale.to(dev), bias, out_dtype=torch.bfloat16,
                                 relu=self._relu_fused, out_scale=self._out_qscale, out_u8=self._out_u8)

    def updateOutput(self, input):
        x2 = input if input.dim() == 2 else input.reshape(1, -1)
        if x2.dtype == torch.int8 and x2 is not input:
            _retag(x2, input)
        y = self._native_static(x2)
        if y is not NotImplemented:
            return y if input.dim() == 2 else _retag(y.reshape(-1), y)
        if input.dtype == torch.int8:
            input = dequant(input)
        x = input if input.dim() == 2 else input.reshape(1, -1)
        out_dt = x.dtype if x.is_floating_point() and x.dtype in (torch.float32, torch.bfloat16) else torch.float32
        y = self._gemm(x, out_dt)
        return y if input.dim() == 2 else y.reshape(-1)

    def __repr__(self):
        return f"quantized.Linear[{self.get_name()}]({self.inputSize} -> {self.outputSize})"


class SpatialConvolution(_QuantizedBase):
    def __init__(self, n_input_plane, n_output_plane, kernel_w, kernel_h, stride_w=1, stride_h=1, pad_w=0, pad_h=0,
                 n_group=1, dilation_w=1, dilation_h=1, with_bias=True):
        super().__init__()
        self.nInputPlane, self.nOutputPlane = n_input_plane, n_output_plane
        self.kernelW, self.kernelH, self.strideW, self.strideH = kernel_w, kernel_h, stride_w, stride_h
        self.padW, self.padH, self.nGroup = pad_w, pad_h, n_group
        self.dilationW, self.dilationH = dilation_w, dilation_h
        self.withBias = with_bias
        kg = n_input_plane // n_group * kernel_h * kernel_w
        self.register_buffer("qweight", torch.zeros(n_output_plane, _kp(kg), dtype=torch.int8))
        self.register_buffer("weight_scale", torch.zeros(n_output_plane))
        if with_bias:
            self.register_buffer("qbias", torch.zeros(n_output_plane))

    @staticmethod
    def from_float(m) -> "SpatialConvolution":
        q = SpatialConvolution(m.nInputPlane, m.nOutputPlane, m.kernelW, m.kernelH, m.strideW, m.strideH, m.padW,
                               m.padH, m.nGroup, getattr(m, "dilationW", 1), getattr(m, "dilationH", 1), m.withBias)
        w = m.weight  # (g, out/g, in/g, kh, kw)
        q._quantize_weight(w.reshape(m.nOutputPlane, -1))
        fb = m.__dict__.get("_folded_bias")  # a BatchNorm folded in by the quantizer
        if fb is not None:
            q.withBias = True
            q.qbias = fb.detach().float().clone().cpu()
        elif m.withBias:
            q.qbias = m.bias.detach().float().clone().cpu()
        q.format = getattr(m, "format", "NCHW")
        q.static_scale = calibrated_scale(m)
        oa = m.__dict__.get("_folded_out_amax")
        q.static_out_scale = oa / 127.0 if oa else None
        q.set_name(m.get_name())
        return q.to(w.device)

    def _i8_prep(self, x, C):
        from ...ops import native_ops as NO
        prep = getattr(self, "_i8w", None)
        if prep is None or prep[0].device != x.device:
            wq, ldw = NO.conv_i8_weight(self.qweight.to(x.device), self.nOutputPlane, C, self.kernelH, self.kernelW)
            prep = self._i8w = (wq, ldw, self.weight_scale.to(x.device).float().contiguous(),
                                self.bias_f.to(x.device).float().contiguous() if self.bias_f is not None else None)
        return prep

    def _u8_bias(self, x, prep, C):
        """The bias with the offset term of an unsigned (offset) int8 input, cached per (device,
        input scale)."""
        from ...ops import native_ops as NO
        if not getattr(x, "_qzero", 0):
            return None
        key = (x.device, x._qscale)
        t = getattr(self, "_i8u8", None)
        if t is None or t[0] != key:
            t = self._i8u8 = (key, NO.conv_i8_u8_bias(prep[0], prep[1], self.nOutputPlane, self.kernelH, self.kernelW,
                                                      C, x._qscale, prep[2], prep[3]))
        return t[1]

    def _out_hw(self, x, pads):
        pt, pb, pl, pr = pads
        H, W = x.shape[2], x.shape[3]
        P = (H + pt + pb - self.dilationH * (self.kernelH - 1) - 1) // self.strideH + 1
        Q = (W + pl + pr - self.dilationW * (self.kernelW - 1) - 1) // self.strideW + 1
        return P, Q

    def _pair_ok(self, x, pads, residual=None):
        """A 64-channel 1×1 stride-1 conv on an int8 chain input: run as the GEMM of pixel PAIRS
        ([M/2][128] codes · block-diagonal [[W, 0], [0, W]]), whose output rows [M/2][2K] are exactly
        the NHWC [M][K] result — every staged activation byte is useful (the 64-channel k-tile of the
        plain form is half padding) and half as many tiles re-stage the weights."""
        N, C, H, W = x.shape
        return (x.dtype == torch.int8 and C == 64 and self.kernelH == 1 and self.kernelW == 1 and self.strideH == 1
                and self.strideW == 1 and tuple(pads) == (0, 0, 0, 0) and (N * H * W) % 2 == 0
                and self.nOutputPlane % 16 == 0 and self.__dict__.get("_cat_join") is None
                and x.is_contiguous(memory_format=torch.channels_last)
                and (residual is None or residual.is_contiguous(memory_format=torch.channels_last)))

    def _pair_prep(self, x):
        from ...ops import native_ops as NO
        prep = self._i8_prep(x, 64)
        pp = self.__dict__.get("_i8pair")
        if pp is None or pp[0].device != x.device:
            K = self.nOutputPlane
            wq = prep[0].view(torch.int8).reshape(K, prep[1])  # [K][128]: 64 weights + 64 zero pad
            w2 = torch.zeros(2 * K, 128, dtype=torch.int8, device=x.device)
            w2[:K, :64] = wq[:, :64]
            w2[K:, 64:] = wq[:, :64]
            pp = self._i8pair = (w2.contiguous(), 128, torch.cat([prep[2], prep[2]]).contiguous(),
                                 torch.cat([prep[3], prep[3]]).contiguous() if prep[3] is not None else None)
        return pp

    @staticmethod
    def _as_pairs(t, C2):
        """[N][C][H][W] channels-last → the [1][2C][1][N·H·W/2] view of the same bytes (tags kept)."""
        N, C, H, W = t.shape
        m2 = N * H * W // 2
        v = torch.as_strided(t, (1, C2, 1, m2), (m2 * C2, 1, m2 * C2, C2))
        return _retag(v, t)

    def _native_pairs(self, x, residual=None, out_scale=None, out_u8=False, relu=None):
        from ...ops import native_ops as NO
        N, C, H, W = x.shape
        K = self.nOutputPlane
        w2, ldw, sw2, b2 = self._pair_prep(x)
        xp = self._as_pairs(x, 128)
        if getattr(x, "_qzero", 0):
            key = (x.device, x._qscale)
            t = self.__dict__.get("_i8pair_u8")
            if t is None or t[0] != key:
                t = self._i8pair_u8 = (key, NO.conv_i8_u8_bias(w2, ldw, 2 * K, 1, 1, 128, x._qscale, sw2, b2))
            ub = t[1]
        else:
            ub = None
        rp = self._as_pairs(residual, 2 * K) if residual is not None else None
        y = NO.conv2d_i8_forward_static(xp, w2, ldw, sw2, b2, 2 * K, 1, 1, (1, 1), (0, 0), (1, 1), (1, N * H * W // 2),
                                        relu=self._relu_fused if relu is None else relu, in_scale=self.static_scale,
                                        out_scale=out_scale, out_u8=out_u8, u8_bias=ub, residual=rp)
        if y is NotImplemented:
            return y
        out = torch.as_strided(y, (N, K, H, W), (H * W * K, 1, W * K, K))
        return _retag(out, y)

    def _native_static(self, x, pads):
        """Calibrated int8 path: int8 (or statically quantised) input, int8 output for the next
        quantised layer of the chain (bias + ReLU + requantisation in the epilogue) or bf16."""
        from ...ops import native_ops as NO
        pt, pb, pl, pr = pads
        if not (x.is_cuda and self.nGroup == 1 and self.nOutputPlane % 8 == 0 and pt == pb and pl == pr
                and ops.native_has("gemm_i8")):
            return NotImplemented
        if x.dtype != torch.int8 and self.static_scale is None:
            return NotImplemented
        if self._pair_ok(x, pads) and self._out_qscale is not None:
            y = self._native_pairs(x, out_scale=self._out_qscale, out_u8=self._out_u8)
            if y is not NotImplemented:
                return y
        C = x.shape[1]
        if NO.conv_i8_supported(C, self.kernelH, self.kernelW):
            prep = self._i8_prep(x, C)
            xin = x if x.dtype == torch.int8 else x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            out = None
            cj = self.__dict__.get("_cat_join")
            if cj is not None and self._out_qscale is not None:
                # zero-copy concat: write this conv's channel slice of the join's output
                join, off, ctot = cj
                P, Q = self._out_hw(x, pads)
                buf = join._i8_cat_buffer(x.shape[0], ctot, P, Q, x.device, self._out_u8)
                out = buf[:, off:off + self.nOutputPlane]
            y = NO.conv2d_i8_forward_static(xin, prep[0], prep[1], prep[2], prep[3], self.nOutputPlane,
                                            self.kernelH, self.kernelW, (self.strideH, self.strideW), (pt, pl),
                                            (self.dilationH, self.dilationW), self._out_hw(x, pads),
                                            relu=self._relu_fused, in_scale=self.static_scale,
                                            out_scale=self._out_qscale, out_u8=self._out_u8,
                                            u8_bias=self._u8_bias(x, prep, C), out=out)
            if y is NotImplemented and out is not None:
                y = NO.conv2d_i8_forward_static(xin, prep[0], prep[1], prep[2], prep[3], self.nOutputPlane,
                                                self.kernelH, self.kernelW, (self.strideH, self.strideW), (pt, pl),
                                                (self.dilationH, self.dilationW), self._out_hw(x, pads),
                                                relu=self._relu_fused, in_scale=self.static_scale,
                                                out_scale=self._out_qscale, out_u8=self._out_u8,
                                                u8_bias=self._u8_bias(x, prep, C))
            return y
        if x.dtype == torch.int8:
            return NotImplemented
        # a shape the int8 kernel does not tile (the C = 3 RGB stem): bf16 conv with the dequantised
        # int8 weights, then the static quantisation of its output for the chain
        wf = getattr(self, "_wdeq", None)
        if wf is None or wf.device != x.device:
            kg = C * self.kernelH * self.kernelW
            wf = (self.qweight[:, :kg].float() * self.weight_scale.float()[:, None]).reshape(
                self.nOutputPlane, C, self.kernelH, self.kernelW).to(device=x.device, dtype=torch.bfloat16)
            self._wdeq = wf
        b = self.bias_f.to(x.device).float() if self.bias_f is not None else None
        xb = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        if (self._out_qscale is not None and C <= 4 and self.dilationH == 1 and self.dilationW == 1
                and ops.native_has("conv2d_forward")):
            # quantised in the conv's epilogue: no bf16 activation, no separate quantisation pass
            yq = NO.conv2d_forward_q(xb, wf, b, (self.strideH, self.strideW), (pt, pl), self._relu_fused,
                                     self._out_qscale, u8=self._out_u8)
            if yq is not NotImplemented:
                return yq
        y = NO.conv2d_forward(xb, wf, b, (self.strideH, self.strideW), (pt, pl), (self.dilationH, self.dilationW), 1,
                              relu=self._relu_fused)
        if y is NotImplemented or self._out_qscale is None:
            return y
        return NO.quant_static(y, self._out_qscale, u8=self._out_u8)

    def forward_residual(self, x, res, out_scale=None, out_u8=False):
        """ReLU(conv(x) + res) with the sum and the ReLU in the int8 kernel's epilogue (a residual block
        tail), written as int8 for the next quantised layer when ``out_scale`` is given, else bf16;
        NotImplemented when the calibrated int8 kernel does not apply (the caller sums in torch)."""
        import torch
        from ...ops import native_ops as NO
        if getattr(self, "format", "NCHW") == "NHWC" or x.dim() != 4 or not x.is_cuda:
            return NotImplemented
        pt, pb, pl, pr = self._pads(x)
        C = x.shape[1]
        if not (self.nGroup == 1 and self.nOutputPlane % 16 == 0 and pt == pb and pl == pr and ops.native_has("gemm_i8")
                and NO.conv_i8_supported(C, self.kernelH, self.kernelW)):
            return NotImplemented
        if x.dtype != torch.int8 and self.static_scale is None:
            return NotImplemented
        if res.dtype != torch.int8 or getattr(res, "_qscale", None) is None:
            res = res.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        if self._pair_ok(x, (pt, pb, pl, pr), res) and out_scale is not None and res.dtype == torch.int8:
            y = self._native_pairs(x, residual=res, out_scale=out_scale,
                                   out_u8=bool(out_u8 and out_scale is not None), relu=True)
            if y is not NotImplemented:
                return y
        prep = self._i8_prep(x, C)
        xin = x if x.dtype == torch.int8 else x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        return NO.conv2d_i8_forward_static(xin, prep[0], prep[1], prep[2], prep[3], self.nOutputPlane, self.kernelH,
                                           self.kernelW, (self.strideH, self.strideW), (pt, pl),
                                           (self.dilationH, self.dilationW), self._out_hw(x, (pt, pb, pl, pr)),
                                           relu=True, in_scale=self.static_scale, out_scale=out_scale,
                                           out_u8=bool(out_u8 and out_scale is not None),
                                           u8_bias=self._u8_bias(x, prep, C), residual=res)

    def _pads(self, x):
        from ..layers.conv import same_padding
        if self.padW == -1 and self.padH == -1:
            return same_padding(x.shape[2], x.shape[3], self.strideH, self.strideW, self.kernelH, self.kernelW,
                                self.dilationH, self.dilationW)
        return self.padH, self.padH, self.padW, self.padW

    def _native_i8(self, x, pads):
        """The int8 implicit-GEMM kernel (ops/csrc/conv_i8.hip): per-image activation scales, the
        gather and the GEMM in one launch, dequantisation + bias in the epilogue."""
        from ...ops import native_ops as NO
        pt, pb, pl, pr = pads
        N, C, H, W = x.shape
        kh, kw = self.kernelH, self.kernelW
        if not (x.is_cuda and self.nGroup == 1 and NO.conv_i8_supported(C, kh, kw) and self.nOutputPlane % 8 == 0
                and ops.native_has("gemm_i8")):
            return NotImplemented
        P = (H + pt + pb - self.dilationH * (kh - 1) - 1) // self.strideH + 1
        Q = (W + pl + pr - self.dilationW * (kw - 1) - 1) // self.strideW + 1
        prep = getattr(self, "_i8w", None)
        if prep is None or prep[0].device != x.device:
            wq, ldw = NO.conv_i8_weight(self.qweight.to(x.device), self.nOutputPlane, C, kh, kw)
            prep = self._i8w = (wq, ldw, self.weight_scale.to(x.device).float().contiguous(),
                                self.bias_f.to(x.device).float().contiguous() if self.bias_f is not None else None)
        xb = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        return NO.conv2d_i8_forward(xb, prep[0], prep[1], prep[2], prep[3], self.nOutputPlane, kh, kw,
                                    (self.strideH, self.strideW), (pt, pl), (self.dilationH, self.dilationW), (P, Q))

    def updateOutput(self, input):
        x = input if input.dim() == 4 else input.unsqueeze(0)
        if getattr(self, "format", "NCHW") == "NHWC":
            x = x.permute(0, 3, 1, 2)
        pt, pb, pl, pr = self._pads(x)
        y = self._native_static(x, (pt, pb, pl, pr))
        if y is not NotImplemented:
            if getattr(self, "format", "NCHW") == "NHWC":
                y = _retag(y.permute(0, 2, 3, 1), y)
            return y if input.dim() == 4 else _retag(y.squeeze(0), y)
        if x.dtype == torch.int8:
            x = dequant(x)
        y = self._native_i8(x, (pt, pb, pl, pr))
        if y is not NotImplemented:
            if x.dtype == torch.float32:
                y = y.float()
            if self._relu_fused:
                y = torch.relu(y)
            if getattr(self, "format", "NCHW") == "NHWC":
                y = y.permute(0, 2, 3, 1)
            return y if input.dim() == 4 else y.squeeze(0)
        x = F.pad(x, (pl, pr, pt, pb)) if (pt or pb or pl or pr) else x
        N, C, H, W = x.shape
        kh, kw = self.kernelH, self.kernelW
        P = (H - self.dilationH * (kh - 1) - 1) // self.strideH + 1
        Q = (W - self.dilationW * (kw - 1) - 1) // self.strideW + 1
        out_dt = x.dtype if x.dtype in (torch.float32, torch.bfloat16) else torch.float32
        g = self.nGroup
        cg, kg = C // g, self.nOutputPlane // g
        # one activation scale per image (max|x| of the whole image / 127), as the reference's
        # ConvDataInit quantises each batch element's input (quantized/SpatialConvolution.scala:
        # 163-208) and as the int8 kernel does (ops/csrc/conv_i8.hip)
        amax = acc_float(x).abs().amax(dim=(1, 2, 3))
        inv = torch.where(amax > 0, 127.0 / amax, torch.zeros_like(amax)).repeat_interleave(P * Q)
        outs = []
        for gi in range(g):
            xs = x[:, gi * cg:(gi + 1) * cg]
            cols = F.unfold(xs, (kh, kw), dilation=(self.dilationH, self.dilationW),
                            stride=(self.strideH, self.strideW))  # [N, cg·kh·kw, L]
            rows = acc_float(cols.transpose(1, 2).reshape(N * P * Q, cg * kh * kw))
            kp = self.qweight.shape[1]
            qa = torch.zeros((N * P * Q, kp), dtype=torch.int8, device=x.device)
            qa[:, :cg * kh * kw] = torch.floor(rows * inv[:, None] + 0.5).clamp(-127, 127).to(torch.int8)
            sa = (amax / 127.0).repeat_interleave(P * Q)
            bias = self.bias_f[gi * kg:(gi + 1) * kg] if self.bias_f is not None else None
            y = ops.gemm_i8(qa, sa, self.qweight[gi * kg:(gi + 1) * kg].contiguous(),
                            self.weight_scale[gi * kg:(gi + 1) * kg].contiguous(), bias, out_dtype=out_dt)
            outs.append(y.reshape(N, P, Q, kg))
        y = torch.cat(outs, dim=3) if g > 1 else outs[0]
        y = y.permute(0, 3, 1, 2)  # NCHW logical, channels-last memory
        if self._relu_fused:
            y = torch.relu(y)
        if getattr(self, "format", "NCHW") == "NHWC":
            y = y.permute(0, 2, 3, 1)
        return y if input.dim() == 4 else y.squeeze(0)

    def __repr__(self):
        return (f"quantized.SpatialConvolution[{self.get_name()}]({self.nInputPlane} -> {self.nOutputPlane}, "
                f"{self.kernelW} x {self.kernelH}, {self.strideW}, {self.strideH}, {self.padW}, {self.padH})")


class SpatialDilatedConvolution(SpatialConvolution):
    @staticmethod
    def from_float(m) -> "SpatialDilatedConvolution":
        q = SpatialConvolution.from_float(m)
        q.__class__ = SpatialDilatedConvolution
        return q
