"""Convolution family.

* ``SpatialConvolution`` — ``DL/nn/SpatialConvolution.scala`` (weight 5-D
  ``(nGroup, out/g, in/g, kH, kW)`` at 93-98; ``padW=padH=-1`` = TensorFlow SAME padding via
  ``Utils.getSAMEOutSizeAndPadding``; default init U(±1/√(kW·kH·nIn)) at 150-154).
  The reference runs im2col + MKL GEMM per sample; here the whole batch is one NHWC implicit-GEMM
  launch on MFMA (``bigdl/ops/csrc/conv_igemm.hip``).  The weight is stored physically as
  ``(g, out/g, kH, kW, in/g)`` = KRSC so the kernel's B operand is K-contiguous; the logical
  tensor the user sees keeps BigDL's shape.
* ``SpatialShareConvolution`` (``:312``) — buffer sharing is the allocator's job on HIP; kept as a
  class for API/serialization compatibility.
* Dilated / Full(transposed) / Separable / ConvolutionMap / Temporal / Volumetric / LocallyConnected.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from ... import ops
from ...ops.reference import BNGrad, BNOut, StridedGrad, as_dense
from ...utils.engine import Engine
from ...utils import config
from ..abstractnn import AbstractModule, TensorModule, AutogradModule
from ..initialization_method import RandomUniform, Zeros, VariableFormats
from ...utils import acc_float


def same_padding(in_h, in_w, stride_h, stride_w, k_h, k_w, dil_h=1, dil_w=1):
    """``Utils.getSAMEOutSizeAndPadding``: returns (padTop, padBottom, padLeft, padRight, outH, outW)."""
    out_h = math.ceil(in_h / stride_h)
    out_w = math.ceil(in_w / stride_w)
    ekh = (k_h - 1) * dil_h + 1
    ekw = (k_w - 1) * dil_w + 1
    ph = max((out_h - 1) * stride_h + ekh - in_h, 0)
    pw = max((out_w - 1) * stride_w + ekw - in_w, 0)
    return ph // 2, ph - ph // 2, pw // 2, pw - pw // 2, out_h, out_w


def to_device_layout(x: torch.Tensor) -> torch.Tensor:
    """Device activations are NHWC (channels_last) in the compute dtype."""
    if x.is_cuda and x.dim() == 4:
        dt = Engine.compute_dtype()
        if (dt == torch.bfloat16 and x.dtype in (torch.float32, torch.bfloat16) and x.is_contiguous()
                and not x.is_contiguous(memory_format=torch.channels_last)):
            from ...ops import native as N
            if N.has("nchw_to_nhwc_bf16"):
                y = N.native_ops.nchw_to_nhwc_bf16(x)  # cast + relayout in one pass
                if y is not NotImplemented:
                    return y
        if x.dtype != dt and x.is_floating_point():
            x = x.to(dt)
        if not x.is_contiguous(memory_format=torch.channels_last):
            x = x.contiguous(memory_format=torch.channels_last)
    return x


class SpatialConvolution(TensorModule):
    def __init__(self, n_input_plane, n_output_plane, kernel_w, kernel_h, stride_w=1, stride_h=1, pad_w=0,
                 pad_h=0, n_group=1, propagate_back=True, wRegularizer=None, bRegularizer=None, init_weight=None,
                 init_bias=None, init_grad_weight=None, init_grad_bias=None, with_bias=True, data_format="NCHW",
                 bigdl_type="float"):
        super().__init__()
        if n_output_plane % n_group != 0 or n_input_plane % n_group != 0:
            raise ValueError(f"channels must be multiples of group: in {n_input_plane} out {n_output_plane} g {n_group}")
        if not ((pad_w >= 0 and pad_h >= 0) or (pad_w == -1 and pad_h == -1)):
            raise ValueError(f"Illegal padding configuration (padW: {pad_w}, padH: {pad_h})")
        self.nInputPlane, self.nOutputPlane = n_input_plane, n_output_plane
        self.kernelW, self.kernelH = kernel_w, kernel_h
        self.strideW, self.strideH = stride_w, stride_h
        self.padW, self.padH = pad_w, pad_h
        self.nGroup = n_group
        self.propagateBack = propagate_back
        self.withBias = with_bias
        self.format = data_format
        self.dilationW = self.dilationH = 1
        self.wRegularizer, self.bRegularizer = wRegularizer, bRegularizer
        g = n_group
        shape5 = (g, n_output_plane // g, n_input_plane // g, kernel_h, kernel_w)
        phys = (g, n_output_plane // g, kernel_h, kernel_w, n_input_plane // g)
        w = init_weight if init_weight is not None else torch.zeros(shape5)
        self.register_parameter("weight", torch.as_tensor(w, dtype=torch.float32).reshape(shape5), "gradWeight",
                                layout=(phys, (0, 1, 4, 2, 3)))
        if with_bias:
            b = init_bias if init_bias is not None else torch.zeros(n_output_plane)
            self.register_parameter("bias", torch.as_tensor(b, dtype=torch.float32).reshape(n_output_plane), "gradBias")
        else:
            self.bias = None
            self.gradBias = None
        self._has_init_w = init_weight is not None
        self._has_init_b = init_bias is not None
        stdv = 1.0 / math.sqrt(kernel_w * kernel_h * n_input_plane)
        self._init_weight_method = RandomUniform(-stdv, stdv)
        self._init_bias_method = RandomUniform(-stdv, stdv) if with_bias else Zeros()
        self.reset()

    def reset(self):
        if not self._has_init_w:
            self._init_weight_method.init(self.weight, VariableFormats.GP_OUT_IN_KW_KH)
        if self.withBias and not self._has_init_b:
            self._init_bias_method.init(self.bias, VariableFormats.ONE_D)
        self.zeroGradParameters()
        return self

    # -- geometry ----------------------------------------------------------------------------
    def _pads(self, x):
        H, W = x.shape[-2], x.shape[-1]
        if self.padW == -1 and self.padH == -1:
            pt, pb, pl, pr, _, _ = same_padding(H, W, self.strideH, self.strideW, self.kernelH, self.kernelW,
                                                self.dilationH, self.dilationW)
            return pt, pb, pl, pr
        return self.padH, self.padH, self.padW, self.padW

    def _w4(self, w):
        """(O, I/g, kH, kW) view of a logical 5-D weight without copying when it is KRSC."""
        g, og, ig, kh, kw = w.shape
        krsc = w.permute(0, 1, 3, 4, 2)
        if krsc.is_contiguous():
            return krsc.reshape(g * og, kh, kw, ig).permute(0, 3, 1, 2)
        return w.reshape(g * og, ig, kh, kw)

    def _prep(self, input):
        x = input
        batched = x.dim() == 4
        if not batched:
            x = x.unsqueeze(0)
        if self.format == "NHWC":
            x = x.permute(0, 3, 1, 2)
        if (self.nInputPlane <= 3 and self.nGroup == 1 and x.is_cuda and x.dim() == 4 and x.is_contiguous()
                and not x.is_contiguous(memory_format=torch.channels_last) and (self.dilationH, self.dilationW) == (1, 1)
                and Engine.compute_dtype() == torch.bfloat16 and x.dtype in (torch.float32, torch.bfloat16)):
            # the RGB input: cast + relayout + channel padding for the C4 stem kernel in one pass
            from ...ops import native as N
            y = N.native_ops.nchw_to_nhwc_padded(x, self._pad_slot_()) if N.has("conv2d_forward") else NotImplemented
            x = to_device_layout(x) if y is NotImplemented else y
        else:
            x = to_device_layout(x)
        pt, pb, pl, pr = self._pads(x)
        if pt != pb or pl != pr:
            x = F.pad(x, (pl, pr, pt, pb))
            pad = (0, 0)
        else:
            pad = (pt, pl)
        return x, pad, batched, (pt, pb, pl, pr)

    #: BN this conv's bias is folded into (set by bigdl.nn.fusion); the BN adds it implicitly and
    #: accumulates its gradient, so the conv skips both
    _bias_folded_into = None
    #: the following ReLU is applied in this conv's epilogue (bigdl.nn.fusion ``convrelu``; the ReLU
    #: module then only masks the gradient)
    _fused_relu = False
    #: channel slice of a concat output this conv writes straight into (set per forward by a
    #: zero-copy JoinTable/Concat plan); consumed once
    _out_target = None

    #: gradient added to this conv's gradInput in the dgrad epilogue (set by a fused residual
    #: ConcatTable for the first conv of a block: the branch/shortcut gradient sum)
    _grad_residual = None
    #: BN (+fused ReLU) whose output this conv consumes: the dgrad epilogue applies its ReLU mask
    #: and produces its backward reductions (set by bigdl.nn.fusion)
    _bn_bwd_target = None
    #: fused block-tail BNs (ReLU(BN(x) + shortcut)) whose output may be this conv's input: the
    #: dgrad epilogue then also applies that ReLU mask and produces the tail BN's reductions
    _tail_candidates = None
    #: this conv is a fused block's 1×1 strided shortcut: its input gradient may be returned as a
    #: StridedGrad (set by bigdl.nn.fusion; the block's first conv consumes it)
    _lazy_strided_ok = False

    def _pad_slot_(self):
        """One-entry holder for the channel-padded copy of a C % 8 input (RGB stem): made by the
        forward, reused by this layer's backward of the same input (ops.native_ops._pad_channels)."""
        s = self.__dict__.get("_pad_slot")
        if s is None:
            s = self.__dict__["_pad_slot"] = [None]
        return s

    def _tail_target(self, x):
        for bn in self._tail_candidates or ():
            y = bn.output
            if (isinstance(y, torch.Tensor) and y.data_ptr() == x.data_ptr() and y.shape == x.shape and bn.train
                    and getattr(bn, "_last_relu", False)
                    and bn._last_input is not None and bn._last_input.shape == x.shape):
                return bn
        return None

    def _stats_consumer(self, x):
        """The training BN that will consume this conv's output (fusion), if the epilogue can
        produce its statistics."""
        bn = self._bias_folded_into
        if bn is None or not bn.train or not x.is_cuda:
            return None
        if getattr(bn, "_sync", False) and not config.get_property("bigdl.bn.shiftedStats"):
            return None  # SyncBN sums partials across ranks: they need the common running-mean shift
        if self.format != "NCHW" or not config.get_property("bigdl.fusion.convstats"):
            return None
        return bn

    def _pro_input(self, input):
        """A deferred BN + ReLU output (fp32 bigdl.fp32.bnPrologue) this conv can take as is: (BN input,
        [scale | shift]) or None (the caller materialises it)."""
        if not (isinstance(input, BNOut) and input.relu and self.format == "NCHW" and self.nGroup == 1
                and input.dim() == 4 and input.is_cuda and self.padW >= 0 and self.padH >= 0):
            return None
        return input.x, input.coef

    def updateOutput(self, input):
        pro = self._pro_input(input)
        if pro is not None:
            y = self._pro_forward(pro[0], pro[1])
            if y is not NotImplemented:
                return y
        if isinstance(input, BNOut):
            input = input.dense()
        x, pad, batched, _ = self._prep(input)
        w4 = self._w4(self.cw("weight"))
        # fp32 master bias: the HIP epilogue adds fp32 (no per-call cast), the reference casts
        b = self.bias if (self.withBias and self._bias_folded_into is None) else None
        bn = self._stats_consumer(x) if batched else None
        y = NotImplemented
        if bn is not None and ops.native_has("conv2d_forward"):
            shift = bn._stat_shift() if config.get_property("bigdl.bn.shiftedStats") else None
            sums = bn._atomic_sums("fwd", self.nOutputPlane, x.device) if shift is not None else None
            r = ops.native_ops.conv2d_forward_stats(x, w4, b, (self.strideH, self.strideW), pad,
                                                (self.dilationH, self.dilationW), self.nGroup,
                                                pad_slot=self._pad_slot_(), shift=shift, sums=sums)
            if r is not NotImplemented:
                y, part, G = r
                bn._pending_stats = (y.data_ptr(), tuple(y.shape), part, G, shift)
        if y is NotImplemented:
            tgt, self._out_target = self._out_target, None
            if tgt is not None and (not batched or self.format != "NCHW"):
                tgt = None
            y = ops.conv2d_forward(x, w4, b, (self.strideH, self.strideW), pad, (self.dilationH, self.dilationW),
                                   self.nGroup, relu=self._fused_relu, out=tgt,
                                   pad_slot=self._pad_slot_() if (self.train or self.nInputPlane <= 3) else None)
        if self.format == "NHWC":
            y = y.permute(0, 2, 3, 1)
        return y if batched else y.squeeze(0)

    def _pro_forward(self, xb, coef):
        """Forward of a deferred BN + ReLU output (BN input ``xb``, ``coef`` = [scale | shift]) on the
        fp32 direct kernels' B-operand prologue (+ this conv's own BN statistics epilogue)."""
        if not ops.native_has("conv2d_forward"):
            return NotImplemented
        pt, pb, pl, pr = self._pads(xb)
        if pt != pb or pl != pr:
            return NotImplemented
        pad = (pt, pl)
        w4 = self._w4(self.cw("weight"))
        b = self.bias if (self.withBias and self._bias_folded_into is None) else None
        st, dl = (self.strideH, self.strideW), (self.dilationH, self.dilationW)
        bn = self._stats_consumer(xb)
        if bn is not None:
            shift = bn._stat_shift() if config.get_property("bigdl.bn.shiftedStats") else None
            sums = bn._atomic_sums("fwd", self.nOutputPlane, xb.device) if shift is not None else None
            r = ops.native_ops.conv2d_forward_stats(xb, w4, b, st, pad, dl, self.nGroup, shift=shift, sums=sums,
                                                    pro=coef) if sums is not None else NotImplemented
            if r is not NotImplemented:
                y, part, G = r
                bn._pending_stats = (y.data_ptr(), tuple(y.shape), part, G, shift)
                return y
            if sums is not None:
                bn._drop_sums((None, None, sums[0], sums[1]), 3)
        return ops.native_ops.conv2d_forward(xb, w4, b, st, pad, dl, self.nGroup, relu=self._fused_relu, pro=coef)

    def _backward(self, input, gradOutput, need_input, acc):
        pro = self._pro_input(input)
        if pro is not None:
            r = self._pro_backward(pro[0], pro[1], gradOutput, need_input, acc)
            if r is not NotImplemented:
                return r
        if isinstance(input, BNOut):
            input = input.dense()
        x, pad, batched, pads = self._prep(input)
        if isinstance(gradOutput, BNGrad):
            # a deferred BN input gradient: consumed in the backward prologues when this conv can
            # (ops.native_ops.bngrad_consumable), built as a tensor otherwise
            own = self.withBias and self._bias_folded_into is None and acc
            if not (batched and self.format == "NCHW" and not own and ops.native_has("conv2d_backward")
                    and ops.native_ops.bngrad_consumable(gradOutput, x, self._w4(self.cw("weight")),
                                                          (self.strideH, self.strideW), pad, self.nGroup)):
                gradOutput = gradOutput.dense()
        if isinstance(gradOutput, BNGrad):
            gy = gradOutput
        else:
            gy = gradOutput if batched else gradOutput.unsqueeze(0)
            if self.format == "NHWC":
                gy = gy.permute(0, 3, 1, 2)
            gy = to_device_layout(gy)
        w4 = self._w4(self.cw("weight"))
        gw = self._w4(self.gradWeight) if acc else None
        same_scale = self.scale_b == self.scale_w
        own_bias = self.withBias and self._bias_folded_into is None
        gb = self.gradBias if (acc and own_bias and same_scale) else None
        res = self._grad_residual if need_input else None
        self._grad_residual = None
        pt, pb, pl, pr = pads
        fuse_res = res is not None and pt == pb and pl == pr and self.format == "NCHW" and batched
        if isinstance(res, StridedGrad) and not (fuse_res and gy.is_cuda):
            res = res.dense()
        bn = self._bn_bwd_target
        bn_fuse = None
        if (bn is not None and need_input and res is None and pt == pb and pl == pr and self.format == "NCHW"
                and batched and gy.is_cuda and bn.train and bn._fused_relu
                and bn._coef is not None and bn._last_input is not None
                and config.get_property("bigdl.fusion.bnbwd")):
            C_ = bn._coef.numel() // 2
            bn_fuse = {"x": bn._last_input, "scale": bn._coef[:C_], "shift": bn._coef[C_:], "mean": bn.saveMean,
                       "sums": bn._atomic_sums("bwd", C_, bn.saveMean.device)}
        elif (fuse_res and self._tail_candidates and gy.is_cuda and config.get_property("bigdl.fusion.bnbwd")):
            bn = self._tail_target(x)
            if bn is not None:
                bn_fuse = {"x": bn._last_input, "mean": bn.saveMean, "mask": bn.output,
                           "bits": getattr(bn, "_relu_bits", None),
                           "sums": bn._atomic_sums("bwd", bn.saveMean.numel(), bn.saveMean.device)}
        # the shortcut conv of a fused ResNet block (1×1 stride 2) may hand its input gradient back
        # as a StridedGrad: the block's first conv sums it in its dgrad epilogue
        lazy = (need_input and self._lazy_strided_ok and res is None and bn_fuse is None and batched
                and self.format == "NCHW" and pt == pb and pl == pr and gy.is_cuda)
        if fuse_res and not isinstance(res, StridedGrad):
            res = to_device_layout(res)
        gi = ops.conv2d_backward(gy, x, w4, (self.strideH, self.strideW), pad, (self.dilationH, self.dilationW),
                                 self.nGroup, need_input, gw, gb, self.scale_w if acc else 0.0,
                                 residual=res if fuse_res else None, bn_fuse=bn_fuse,
                                 pad_slot=self._pad_slot_(), lazy_strided=lazy)
        if isinstance(gi, StridedGrad):
            return gi
        if bn_fuse is not None and "partial" in bn_fuse and gi is not None:
            bn._pending_grad = (gi.data_ptr(), bn_fuse["partial"], bn_fuse["G"])
        if acc and own_bias and not same_scale and self.scale_b != 0:
            self.gradBias.add_(acc_float(gy).sum((0, 2, 3)), alpha=self.scale_b)
        if need_input and gi is not None:
            pt, pb, pl, pr = pads
            if pt != pb or pl != pr:
                gi = gi[:, :, pt:gi.shape[2] - pb, pl:gi.shape[3] - pr]
            if self.format == "NHWC":
                gi = gi.permute(0, 2, 3, 1)
            if not batched:
                gi = gi.squeeze(0)
            if res is not None and not fuse_res:
                gi = gi + as_dense(res)
        return gi

    def _pro_backward(self, xb, coef, gradOutput, need_input, acc):
        """Backward of a conv whose input is a deferred BN + ReLU output: the weight gradient reads
        relu(xb·scale + shift) through the fp32 wgrad prologue; the data gradient's epilogue applies
        that BN's ReLU mask (recomputed from xb) and adds its backward statistics (bn_fuse)."""
        if not isinstance(gradOutput, torch.Tensor) or gradOutput.dim() != 4 or not gradOutput.is_cuda:
            return NotImplemented
        pt, pb, pl, pr = self._pads(xb)
        if pt != pb or pl != pr:
            return NotImplemented
        pad = (pt, pl)
        gy = to_device_layout(gradOutput)
        w4 = self._w4(self.cw("weight"))
        gw = self._w4(self.gradWeight) if acc else None
        own_bias = self.withBias and self._bias_folded_into is None
        same_scale = self.scale_b == self.scale_w
        gb = self.gradBias if (acc and own_bias and same_scale) else None
        if self._grad_residual is not None and need_input:
            return NotImplemented  # (a block head never consumes a deferred BN output)
        bn = self._bn_bwd_target
        bn_fuse = None
        if (need_input and bn is not None and bn.train and bn._coef is coef and bn._last_input is xb
                and config.get_property("bigdl.fusion.bnbwd")):
            C_ = coef.numel() // 2
            bn_fuse = {"x": xb, "scale": coef[:C_], "shift": coef[C_:], "mean": bn.saveMean,
                       "sums": bn._atomic_sums("bwd", C_, bn.saveMean.device)}
        elif need_input:
            return NotImplemented
        gi = ops.native_ops.conv2d_backward(gy, xb, w4, (self.strideH, self.strideW), pad,
                                            (self.dilationH, self.dilationW), self.nGroup, need_input, gw, gb,
                                            self.scale_w if acc else 0.0, bn_fuse=bn_fuse, pro=coef)
        if gi is NotImplemented:
            if bn_fuse is not None:
                bn._drop_sums((None, bn_fuse["sums"][0], bn_fuse["sums"][1]), 2)
            return NotImplemented
        if bn_fuse is not None and "partial" in bn_fuse and gi is not None:
            bn._pending_grad = (gi.data_ptr(), bn_fuse["partial"], bn_fuse["G"])
        # (otherwise gi is unmasked and the BN's own backward applies its ReLU mask from BNOut.dense())
        if acc and own_bias and not same_scale and self.scale_b != 0:
            self.gradBias.add_(acc_float(gy).sum((0, 2, 3)), alpha=self.scale_b)
        return gi

    #: False when this conv consumes the model input of a training run (set by
    #: bigdl.nn.fusion.mark_input_no_grad): the optimizer never reads that gradInput
    _input_grad_needed = True

    def updateGradInput(self, input, gradOutput):
        if not self._input_grad_needed and self.propagateBack:
            self._gi_done = False
            if self._grad_residual is None:
                return torch.empty(0, device=input.device, dtype=input.dtype)
        if not self.propagateBack:
            self._gi_done = False
            res, self._grad_residual = self._grad_residual, None
            if res is not None:
                return as_dense(res).clone()
            # the reference returns its (empty) gradInput untouched (SpatialConvolution.scala:364-366):
            # no zero-filled input-sized tensor
            return torch.empty(0, device=input.device, dtype=input.dtype) if isinstance(input, torch.Tensor) else None
        # compute gradInput and (fused) parameter gradients in one pass; accGradParameters then
        # only applies regularisers
        gi = self._backward(input, gradOutput, True, True)
        self._gi_done = True
        return gi

    def accGradParameters(self, input, gradOutput):
        if not getattr(self, "_gi_done", False):
            self._backward(input, gradOutput, False, True)
        self._gi_done = False
        if self.wRegularizer is not None and self.scale_w != 0:
            self.wRegularizer.accRegularization(self.weight, self.gradWeight, self.scale_w)
        if self.withBias and self.bRegularizer is not None and self.scale_b != 0:
            self.bRegularizer.accRegularization(self.bias, self.gradBias, self.scale_b)

    def backward(self, input, gradOutput):
        return super().backward(input, gradOutput)

    def __repr__(self):
        return (f"SpatialConvolution[{self.get_name()}]({self.nInputPlane} -> {self.nOutputPlane}, "
                f"{self.kernelW} x {self.kernelH}, {self.strideW}, {self.strideH}, {self.padW}, {self.padH})")


class FusedConvSum(AbstractModule):
    """Inference form of a residual block tail produced by the IR lowering: input
    ``Table(x, shortcut)`` → ``[ReLU](conv(x) + shortcut)``, the add and ReLU done in the conv
    epilogue (the reference's conv+sum MKL-DNN post-op, ``Fusion.fusionCAddTable``)."""

    def __init__(self, conv, relu=True):
        super().__init__()
        self.conv, self.relu = conv, relu
        self.set_name(conv.get_name() + "/sum")

    def children(self):
        return [self.conv]

    def updateOutput(self, input):
        c = self.conv
        x, pad, batched, _ = c._prep(input[1])
        r = input[2] if batched else input[2].unsqueeze(0)
        r = to_device_layout(r)
        b = c.bias if c.withBias else None
        y = ops.conv2d_forward(x, c._w4(c.cw("weight")), b, (c.strideH, c.strideW), pad, (c.dilationH, c.dilationW),
                               c.nGroup, relu=self.relu, res=r)
        return y if batched else y.squeeze(0)

    def updateGradInput(self, input, gradOutput):
        raise RuntimeError("FusedConvSum is an inference-only node")

    def __repr__(self):
        return f"FusedConvSum({self.conv!r}, relu={self.relu})"


class SpatialShareConvolution(SpatialConvolution):
    """Same math as SpatialConvolution; the reference shares im2col buffers between layers
    (``SpatialShareConvolution.scala:312``) — implicit GEMM needs no im2col buffer at all."""


class SpatialDilatedConvolution(SpatialConvolution):
    def __init__(self, n_input_plane, n_output_plane, kw, kh, dw=1, dh=1, pad_w=0, pad_h=0, dilation_w=1,
                 dilation_h=1, wRegularizer=None, bRegularizer=None, bigdl_type="float"):
        super().__init__(n_input_plane, n_output_plane, kw, kh, dw, dh, pad_w, pad_h, 1, True, wRegularizer,
                         bRegularizer)
        self.dilationW, self.dilationH = dilation_w, dilation_h


class SpatialFullConvolution(AutogradModule):
    """Transposed convolution (``SpatialFullConvolution.scala``); weight (g, in/g, out/g, kH, kW)."""

    def __init__(self, n_input_plane, n_output_plane, kw, kh, dw=1, dh=1, pad_w=0, pad_h=0, adj_w=0, adj_h=0,
                 n_group=1, no_bias=False, wRegularizer=None, bRegularizer=None, bigdl_type="float"):
        super().__init__()
        self.nInputPlane, self.nOutputPlane = n_input_plane, n_output_plane
        self.kW, self.kH, self.dW, self.dH = kw, kh, dw, dh
        self.padW, self.padH, self.adjW, self.adjH = pad_w, pad_h, adj_w, adj_h
        self.nGroup, self.noBias = n_group, no_bias
        self.wRegularizer, self.bRegularizer = wRegularizer, bRegularizer
        self.register_parameter("weight", torch.zeros(n_group, n_input_plane // n_group, n_output_plane // n_group, kh, kw))
        if not no_bias:
            self.register_parameter("bias", torch.zeros(n_output_plane))
        stdv = 1.0 / math.sqrt(kw * kh * n_input_plane)
        self._init_weight_method = RandomUniform(-stdv, stdv)
        self._init_bias_method = RandomUniform(-stdv, stdv)
        self.reset()

    def reset(self):
        self._init_weight_method.init(self.weight, VariableFormats.GP_IN_OUT_KW_KH)
        if not self.noBias:
            self._init_bias_method.init(self.bias, VariableFormats.ONE_D)
        return self

    def _forward(self, x):
        if isinstance(x, torch.Tensor):
            inp = x
            adj = (self.adjH, self.adjW)
        else:  # Table(input, sizeTensor) variant
            inp = x[1]
            target = x[2]
            oh = (inp.shape[-2] - 1) * self.dH - 2 * self.padH + self.kH
            ow = (inp.shape[-1] - 1) * self.dW - 2 * self.padW + self.kW
            adj = (target.shape[-2] - oh, target.shape[-1] - ow)
        batched = inp.dim() == 4
        if not batched:
            inp = inp.unsqueeze(0)
        w = self.P("weight")
        g = self.nGroup
        w4 = w.reshape(g * w.shape[1], w.shape[2], self.kH, self.kW)
        b = self.P("bias") if not self.noBias else None
        if inp.is_cuda and ops.native_has("conv2d_forward"):
            y = ops.native_ops.conv_transpose2d(to_device_layout(inp), w4, b, (self.dH, self.dW),
                                                (self.padH, self.padW), adj, g)
            if y is not NotImplemented:
                return y if batched else y.squeeze(0)
            ops.native.note_fallback("conv_transpose2d", "geometry", (inp, w4))
        y = F.conv_transpose2d(inp, w4.to(inp.dtype), None if b is None else b.to(inp.dtype), (self.dH, self.dW),
                               (self.padH, self.padW), adj, g)
        return y if batched else y.squeeze(0)


class SpatialSeparableConvolution(AutogradModule):
    """Depthwise (multiplier) + pointwise conv (``SpatialSeparableConvolution.scala``)."""

    def __init__(self, n_input_channel, n_output_channel, depth_multiplier, kernel_w, kernel_h, stride_w=1,
                 stride_h=1, pad_w=0, pad_h=0, with_bias=True, data_format="NCHW", w_regularizer=None,
                 b_regularizer=None, p_regularizer=None, bigdl_type="float"):
        super().__init__()
        self.nIn, self.nOut, self.mult = n_input_channel, n_output_channel, depth_multiplier
        self.kW, self.kH, self.sW, self.sH, self.pW, self.pH = kernel_w, kernel_h, stride_w, stride_h, pad_w, pad_h
        self.withBias, self.format = with_bias, data_format
        self.register_parameter("depthWeight", torch.zeros(n_input_channel * depth_multiplier, 1, kernel_h, kernel_w),
                                "depthGradWeight")
        self.register_parameter("pointWeight", torch.zeros(n_output_channel, n_input_channel * depth_multiplier, 1, 1),
                                "pointGradWeight")
        if with_bias:
            self.register_parameter("bias", torch.zeros(n_output_channel))
        self.reset()

    def reset(self):
        RandomUniform().init(self.depthWeight, VariableFormats.OUT_IN_KW_KH)
        RandomUniform().init(self.pointWeight, VariableFormats.OUT_IN_KW_KH)
        if self.withBias:
            Zeros().init(self.bias)
        return self

    def _forward(self, x):
        nhwc = self.format == "NHWC"
        if nhwc:
            x = x.permute(0, 3, 1, 2)
        pad = (self.pH, self.pW)
        if self.pW == -1:
            pt, pb, pl, pr, _, _ = same_padding(x.shape[2], x.shape[3], self.sH, self.sW, self.kH, self.kW)
            x = F.pad(x, (pl, pr, pt, pb))
            pad = (0, 0)
        bias = self.P("bias") if self.withBias else None
        if x.is_cuda and ops.native_has("conv2d_forward"):
            # depthwise stencil kernel + pointwise MFMA conv, both differentiable native ops
            xd = to_device_layout(x)
            y = ops.native_ops.conv2d_autograd(xd, self.P("depthWeight"), None, (self.sH, self.sW), pad, (1, 1),
                                               self.nIn)
            if y is not NotImplemented:
                y2 = ops.native_ops.conv2d_autograd(y, self.P("pointWeight"), bias, (1, 1), (0, 0))
                if y2 is not NotImplemented:
                    return y2.permute(0, 2, 3, 1) if nhwc else y2
            ops.native.note_fallback("separable_conv", "geometry", (xd,))
        y = F.conv2d(x, self.P("depthWeight").to(x.dtype), None, (self.sH, self.sW), pad, 1, self.nIn)
        y = F.conv2d(y, self.P("pointWeight").to(x.dtype), bias.to(x.dtype) if bias is not None else None)
        return y.permute(0, 2, 3, 1) if nhwc else y


class SpatialConvolutionMap(AutogradModule):
    """Convolution with an explicit input→output connection table (``SpatialConvolutionMap.scala``)."""

    def __init__(self, conn_table, kw, kh, dw=1, dh=1, pad_w=0, pad_h=0, wRegularizer=None, bRegularizer=None,
                 bigdl_type="float"):
        super().__init__()
        ct = torch.as_tensor(conn_table).long()
        self.connTable = ct
        self.kW, self.kH, self.dW, self.dH, self.padW, self.padH = kw, kh, dw, dh, pad_w, pad_h
        self.nInputPlane = int(ct[:, 0].max())
        self.nOutputPlane = int(ct[:, 1].max())
        self.register_parameter("weight", torch.zeros(ct.shape[0], kh, kw))
        self.register_parameter("bias", torch.zeros(self.nOutputPlane))
        self.reset()

    @staticmethod
    def full(nin, nout):
        return torch.tensor([[i + 1, o + 1] for o in range(nout) for i in range(nin)])

    @staticmethod
    def oneToOne(n):
        return torch.tensor([[i + 1, i + 1] for i in range(n)])

    @staticmethod
    def random(nin, nout, nto):
        rows = []
        for o in range(nout):
            perm = torch.randperm(nin)[:nto]
            rows += [[int(i) + 1, o + 1] for i in perm]
        return torch.tensor(rows)

    def reset(self):
        ninp = {}
        for i, o in self.connTable.tolist():
            ninp[o] = ninp.get(o, 0) + 1
        stdv = 1.0 / math.sqrt(self.kW * self.kH * max(ninp.values()))
        RandomUniform(-stdv, stdv).init(self.weight)
        RandomUniform(-stdv, stdv).init(self.bias)
        return self

    def _forward(self, x):
        batched = x.dim() == 4
        if not batched:
            x = x.unsqueeze(0)
        dense = torch.zeros(self.nOutputPlane, self.nInputPlane, self.kH, self.kW, dtype=x.dtype, device=x.device)
        w = self.P("weight").to(x.dtype)
        idx_o = self.connTable[:, 1].to(x.device) - 1
        idx_i = self.connTable[:, 0].to(x.device) - 1
        dense = dense.index_put((idx_o, idx_i), w, accumulate=True)
        y = F.conv2d(x, dense, self.P("bias").to(x.dtype), (self.dH, self.dW), (self.padH, self.padW))
        return y if batched else y.squeeze(0)


class TemporalConvolution(AutogradModule):
    """1-D conv over (batch, frames, features) (``TemporalConvolution.scala``): weight (out, in·kW)."""

    def __init__(self, input_frame_size, output_frame_size, kernel_w, stride_w=1, propagate_back=True,
                 weight_regularizer=None, bias_regularizer=None, init_weight=None, init_bias=None,
                 init_grad_weight=None, init_grad_bias=None, bigdl_type="float"):
        super().__init__()
        self.inputFrameSize, self.outputFrameSize = input_frame_size, output_frame_size
        self.kernelW, self.strideW = kernel_w, stride_w
        self.wRegularizer, self.bRegularizer = weight_regularizer, bias_regularizer
        self.register_parameter("weight", torch.zeros(output_frame_size, input_frame_size * kernel_w))
        self.register_parameter("bias", torch.zeros(output_frame_size))
        stdv = 1.0 / math.sqrt(kernel_w * input_frame_size)
        if init_weight is not None:
            self.weight.copy_(torch.as_tensor(init_weight).reshape(self.weight.shape))
        else:
            RandomUniform(-stdv, stdv).init(self.weight)
        if init_bias is not None:
            self.bias.copy_(torch.as_tensor(init_bias).reshape(self.bias.shape))
        else:
            RandomUniform(-stdv, stdv).init(self.bias)

    def _forward(self, x):
        batched = x.dim() == 3
        if not batched:
            x = x.unsqueeze(0)
        if x.is_cuda and ops.native_has("conv2d_forward") and Engine.compute_dtype() == torch.bfloat16:
            # (N, T, C) frames are the NHWC image (N, C, 1, T): the 2-D native conv with a 1×kW filter
            # runs on the same memory (weight (out, kW·in) → [out][in][1][kW])
            xb = x.to(torch.bfloat16).contiguous()
            x4 = xb.permute(0, 2, 1).unsqueeze(2)
            if x4.is_contiguous(memory_format=torch.channels_last):
                w4 = self.P("weight").view(self.outputFrameSize, self.kernelW, self.inputFrameSize) \
                    .permute(0, 2, 1).unsqueeze(2)
                y = ops.native_ops.conv2d_autograd(x4, w4, self.P("bias"), (1, self.strideW), (0, 0))
                if y is not NotImplemented:
                    y = y.squeeze(2).permute(0, 2, 1)
                    return y if batched else y.squeeze(0)
            ops.native.note_fallback("temporal_conv", "geometry", (x,))
        w = self.P("weight").to(x.dtype).view(self.outputFrameSize, self.kernelW, self.inputFrameSize).permute(0, 2, 1)
        y = F.conv1d(x.transpose(1, 2), w, self.P("bias").to(x.dtype), self.strideW).transpose(1, 2)
        return y if batched else y.squeeze(0)


class VolumetricConvolution(AutogradModule):
    """3-D conv (``VolumetricConvolution.scala``): weight (out, in, kT, kH, kW)."""

    def __init__(self, n_input_plane, n_output_plane, k_t, k_w, k_h, d_t=1, d_w=1, d_h=1, pad_t=0, pad_w=0,
                 pad_h=0, with_bias=True, wRegularizer=None, bRegularizer=None, bigdl_type="float"):
        super().__init__()
        self.nInputPlane, self.nOutputPlane = n_input_plane, n_output_plane
        self.k = (k_t, k_h, k_w)
        self.d = (d_t, d_h, d_w)
        self.p = (pad_t, pad_h, pad_w)
        self.withBias = with_bias
        self.wRegularizer, self.bRegularizer = wRegularizer, bRegularizer
        self.register_parameter("weight", torch.zeros(n_output_plane, n_input_plane, k_t, k_h, k_w))
        if with_bias:
            self.register_parameter("bias", torch.zeros(n_output_plane))
        stdv = 1.0 / math.sqrt(k_t * k_w * k_h * n_input_plane)
        RandomUniform(-stdv, stdv).init(self.weight)
        if with_bias:
            RandomUniform(-stdv, stdv).init(self.bias)

    def _forward(self, x):
        batched = x.dim() == 5
        if not batched:
            x = x.unsqueeze(0)
        pad = self.p
        pads = None
        if self.p[1] == -1:
            pads = []
            for dim, k, s in zip(x.shape[2:], self.k, self.d):
                o = math.ceil(dim / s)
                tot = max((o - 1) * s + k - dim, 0)
                pads.append((tot // 2, tot - tot // 2))
        if x.is_cuda and ops.native_has("conv2d_forward") and Engine.compute_dtype() == torch.bfloat16:
            # implicit-GEMM 3-D conv (conv_igemm.hip D3): SAME padding is the leading pad + output size
            lead = tuple(p_[0] for p_ in pads) if pads else pad
            outd = tuple(math.ceil(dim / s) for dim, s in zip(x.shape[2:], self.d)) if pads else None
            y = ops.native_ops.conv3d_autograd(x, self.P("weight"), self.P("bias") if self.withBias else None,
                                               self.d, lead, (1, 1, 1), outd)
            if y is not NotImplemented:
                return y if batched else y.squeeze(0)
            ops.native.note_fallback("volumetric_conv", "geometry", (x,))
        if pads:
            x = F.pad(x, (pads[2][0], pads[2][1], pads[1][0], pads[1][1], pads[0][0], pads[0][1]))
            pad = (0, 0, 0)
        y = F.conv3d(x, self.P("weight").to(x.dtype), self.P("bias").to(x.dtype) if self.withBias else None, self.d,
                     pad)
        return y if batched else y.squeeze(0)


class VolumetricFullConvolution(AutogradModule):
    def __init__(self, n_input_plane, n_output_plane, kt, kw, kh, dt=1, dw=1, dh=1, pad_t=0, pad_w=0, pad_h=0,
                 adj_t=0, adj_w=0, adj_h=0, n_group=1, no_bias=False, wRegularizer=None, bRegularizer=None,
                 bigdl_type="float"):
        super().__init__()
        self.k, self.d, self.p, self.adj = (kt, kh, kw), (dt, dh, dw), (pad_t, pad_h, pad_w), (adj_t, adj_h, adj_w)
        self.nGroup, self.noBias = n_group, no_bias
        self.register_parameter("weight", torch.zeros(n_group, n_input_plane // n_group, n_output_plane // n_group,
                                                      kt, kh, kw))
        if not no_bias:
            self.register_parameter("bias", torch.zeros(n_output_plane))
        stdv = 1.0 / math.sqrt(kt * kw * kh * n_input_plane)
        RandomUniform(-stdv, stdv).init(self.weight)
        if not no_bias:
            RandomUniform(-stdv, stdv).init(self.bias)

    def _forward(self, x):
        batched = x.dim() == 5
        if not batched:
            x = x.unsqueeze(0)
        w = self.P("weight")
        w5 = w.reshape(w.shape[0] * w.shape[1], w.shape[2], *self.k)
        y = F.conv_transpose3d(x, w5.to(x.dtype), None if self.noBias else self.P("bias").to(x.dtype), self.d,
                               self.p, self.adj, self.nGroup)
        return y if batched else y.squeeze(0)


class LocallyConnected2D(AutogradModule):
    """Unshared-weight 2-D conv (``LocallyConnected2D.scala``)."""

    def __init__(self, n_input_plane, input_width, input_height, n_output_plane, kernel_w, kernel_h, stride_w=1,
                 stride_h=1, pad_w=0, pad_h=0, propagate_back=True, wRegularizer=None, bRegularizer=None,
                 init_weight=None, init_bias=None, init_grad_weight=None, init_grad_bias=None, with_bias=True,
                 data_format="NCHW", bigdl_type="float"):
        super().__init__()
        self.nIn, self.nOut = n_input_plane, n_output_plane
        self.kW, self.kH, self.sW, self.sH, self.pW, self.pH = kernel_w, kernel_h, stride_w, stride_h, pad_w, pad_h
        self.oH = (input_height + 2 * pad_h - kernel_h) // stride_h + 1
        self.oW = (input_width + 2 * pad_w - kernel_w) // stride_w + 1
        self.withBias, self.format = with_bias, data_format
        L = self.oH * self.oW
        self.register_parameter("weight", torch.zeros(L, n_output_plane, n_input_plane * kernel_h * kernel_w))
        if with_bias:
            self.register_parameter("bias", torch.zeros(L, n_output_plane))
        stdv = 1.0 / math.sqrt(kernel_w * kernel_h * n_input_plane)
        RandomUniform(-stdv, stdv).init(self.weight)
        if with_bias:
            RandomUniform(-stdv, stdv).init(self.bias)

    def _forward(self, x):
        nhwc = self.format == "NHWC"
        if nhwc:
            x = x.permute(0, 3, 1, 2)
        batched = x.dim() == 4
        if not batched:
            x = x.unsqueeze(0)
        cols = F.unfold(x, (self.kH, self.kW), padding=(self.pH, self.pW), stride=(self.sH, self.sW))  # N, CKK, L
        y = torch.einsum("ncl,loc->nol", cols, self.P("weight").to(x.dtype))
        if self.withBias:
            y = y + self.P("bias").to(x.dtype).t().unsqueeze(0)
        y = y.reshape(x.shape[0], self.nOut, self.oH, self.oW)
        if not batched:
            y = y.squeeze(0)
        return y.permute(0, 2, 3, 1) if nhwc else y


class LocallyConnected1D(AutogradModule):
    def __init__(self, n_input_frame, input_frame_size, output_frame_size, kernel_w, stride_w=1,
                 propagate_back=True, weight_regularizer=None, bias_regularizer=None, init_weight=None,
                 init_bias=None, init_grad_weight=None, init_grad_bias=None, bigdl_type="float"):
        super().__init__()
        self.nFrame, self.inSize, self.outSize, self.kW, self.sW = n_input_frame, input_frame_size, output_frame_size, kernel_w, stride_w
        self.nOutFrame = (n_input_frame - kernel_w) // stride_w + 1
        self.register_parameter("weight", torch.zeros(self.nOutFrame, output_frame_size, input_frame_size * kernel_w))
        self.register_parameter("bias", torch.zeros(self.nOutFrame, output_frame_size))
        stdv = 1.0 / math.sqrt(kernel_w * input_frame_size)
        RandomUniform(-stdv, stdv).init(self.weight)
        RandomUniform(-stdv, stdv).init(self.bias)

    def _forward(self, x):
        batched = x.dim() == 3
        if not batched:
            x = x.unsqueeze(0)
        win = x.unfold(1, self.kW, self.sW)  # N, L, F, kW
        win = win.permute(0, 1, 3, 2).reshape(x.shape[0], self.nOutFrame, -1)
        y = torch.einsum("nlc,loc->nlo", win, self.P("weight").to(x.dtype)) + self.P("bias").to(x.dtype)
        return y if batched else y.squeeze(0)
