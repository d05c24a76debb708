"""Pooling and resampling.

``SpatialMaxPooling`` (``DL/nn/SpatialMaxPooling.scala:91-246`` via ``NNPrimitive.maxPooling*``;
``ceil()`` = Caffe ceil mode), ``SpatialAveragePooling`` (``SpatialAveragePooling.scala:115-700``:
count_include_pad, ceil, global pooling, ``divide``).  Device path: NHWC vectorised kernels that
save the argmax offset within the window.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from ... import ops
from ..abstractnn import TensorModule, AutogradModule
from .conv import to_device_layout, same_padding
from ...utils import acc_float


def _pool_pad(x, kh, kw, dh, dw, ph, pw):
    if ph == -1 and pw == -1:
        pt, pb, pl, pr, _, _ = same_padding(x.shape[-2], x.shape[-1], dh, dw, kh, kw)
        return pt, pb, pl, pr
    return ph, ph, pw, pw


class SpatialMaxPooling(TensorModule):
    def __init__(self, kw, kh, dw=None, dh=None, pad_w=0, pad_h=0, to_ceil=False, format="NCHW",
                 bigdl_type="float"):
        super().__init__()
        self.kW, self.kH = kw, kh
        self.dW = dw if dw is not None else kw
        self.dH = dh if dh is not None else kh
        self.padW, self.padH = pad_w, pad_h
        self.ceilMode = to_ceil
        self.format = format

    def ceil(self):
        self.ceilMode = True
        return self

    def floor(self):
        self.ceilMode = False
        return self

    def _prep(self, input):
        x = input
        if self.format == "NHWC":
            x = x.permute(0, 3, 1, 2) if x.dim() == 4 else x.permute(2, 0, 1)
        batched = x.dim() == 4
        if not batched:
            x = x.unsqueeze(0)
        x = to_device_layout(x)
        pt, pb, pl, pr = _pool_pad(x, self.kH, self.kW, self.dH, self.dW, self.padH, self.padW)
        if pt != pb or pl != pr:
            x = F.pad(x, (pl, pr, pt, pb), value=float("-inf"))
            pad = (0, 0)
        else:
            pad = (pt, pl)
        return x, pad, batched, (pt, pb, pl, pr)

    def _post(self, y, batched):
        if not batched:
            y = y.squeeze(0)
        if self.format == "NHWC":
            y = y.permute(0, 2, 3, 1) if y.dim() == 4 else y.permute(1, 2, 0)
        return y

    def _int8_forward(self, input):
        """Max pooling of an int8 activation of a quantised chain (NHWC int8 kernel; the scale carries
        over) — None when it does not apply."""
        from ...ops import native_ops as NO
        if not (input.is_cuda and input.dim() == 4 and self.format == "NCHW" and not self.train):
            return None
        pt, pb, pl, pr = _pool_pad(input, self.kH, self.kW, self.dH, self.dW, self.padH, self.padW)
        if pt != pb or pl != pr:
            return None
        H, W = input.shape[2], input.shape[3]
        P = NO._pool_out(H, self.kH, self.dH, pt, self.ceilMode)
        Q = NO._pool_out(W, self.kW, self.dW, pl, self.ceilMode)
        y = NO.maxpool_i8(input, self.kH, self.kW, self.dH, self.dW, pt, pl, P, Q)
        return None if y is NotImplemented else y

    def updateOutput(self, input):
        if input.dtype == torch.int8 and getattr(input, "_qscale", None) is not None:
            y = self._int8_forward(input)
            if y is not None:
                return y
            from ..quantized.layers import dequant
            input = dequant(input)
        x, pad, batched, _ = self._prep(input)
        # evaluate mode: no argmax (no backward follows; updateGradInput recomputes it if one does)
        y, idx = ops.maxpool2d_forward(x, (self.kH, self.kW), (self.dH, self.dW), pad, self.ceilMode,
                                       need_indices=bool(self.train))
        self._indices = idx
        return self._post(y, batched)

    def updateGradInput(self, input, gradOutput):
        x, pad, batched, pads = self._prep(input)
        gy = gradOutput
        if self.format == "NHWC":
            gy = gy.permute(0, 3, 1, 2) if gy.dim() == 4 else gy.permute(2, 0, 1)
        if not batched:
            gy = gy.unsqueeze(0)
        gy = to_device_layout(gy)
        if self._indices is None:  # forward ran in evaluate mode: recompute the argmax
            _, self._indices = ops.maxpool2d_forward(x, (self.kH, self.kW), (self.dH, self.dW), pad, self.ceilMode)
        gi = ops.maxpool2d_backward(gy, x, self._indices, (self.kH, self.kW), (self.dH, self.dW), pad, self.ceilMode)
        pt, pb, pl, pr = pads
        if pt != pb or pl != pr:
            gi = gi[:, :, pt:gi.shape[2] - pb, pl:gi.shape[3] - pr]
        return self._post(gi, batched)

    def __repr__(self):
        return f"SpatialMaxPooling[{self.get_name()}]({self.kW}, {self.kH}, {self.dW}, {self.dH}, {self.padW}, {self.padH})"


class SpatialAveragePooling(TensorModule):
    def __init__(self, kw, kh, dw=1, dh=1, pad_w=0, pad_h=0, global_pooling=False, ceil_mode=False,
                 count_include_pad=True, divide=True, format="NCHW", bigdl_type="float"):
        super().__init__()
        self.kW, self.kH, self.dW, self.dH = kw, kh, dw, dh
        self.padW, self.padH = pad_w, pad_h
        self.globalPooling = global_pooling
        self.ceilMode = ceil_mode
        self.countIncludePad = count_include_pad
        self.divide = divide
        self.format = format

    def ceil(self):
        self.ceilMode = True
        return self

    def floor(self):
        self.ceilMode = False
        return self

    def _geom(self, x):
        if self.globalPooling:
            return (x.shape[-2], x.shape[-1]), (1, 1), (0, 0)
        return (self.kH, self.kW), (self.dH, self.dW), None

    def _prep(self, input):
        x = input
        if self.format == "NHWC":
            x = x.permute(0, 3, 1, 2) if x.dim() == 4 else x.permute(2, 0, 1)
        batched = x.dim() == 4
        if not batched:
            x = x.unsqueeze(0)
        x = to_device_layout(x)
        k, s, p = self._geom(x)
        pads = (0, 0, 0, 0)
        if p is None:
            pt, pb, pl, pr = _pool_pad(x, k[0], k[1], s[0], s[1], self.padH, self.padW)
            pads = (pt, pb, pl, pr)
            if pt != pb or pl != pr:
                x = F.pad(x, (pl, pr, pt, pb))
                p = (0, 0)
            else:
                p = (pt, pl)
        divisor = None if self.divide else 1
        return x, k, s, p, batched, pads, divisor

    def _post(self, y, batched):
        if not batched:
            y = y.squeeze(0)
        if self.format == "NHWC":
            y = y.permute(0, 2, 3, 1) if y.dim() == 4 else y.permute(1, 2, 0)
        return y

    def updateOutput(self, input):
        x, k, s, p, batched, _, divisor = self._prep(input)
        y = ops.avgpool2d_forward(x, k, s, p, self.ceilMode, self.countIncludePad, divisor)
        return self._post(y, batched)

    def updateGradInput(self, input, gradOutput):
        x, k, s, p, batched, pads, divisor = self._prep(input)
        gy = gradOutput
        if self.format == "NHWC":
            gy = gy.permute(0, 3, 1, 2) if gy.dim() == 4 else gy.permute(2, 0, 1)
        if not batched:
            gy = gy.unsqueeze(0)
        gy = to_device_layout(gy)
        gi = ops.avgpool2d_backward(gy, x, k, s, p, self.ceilMode, self.countIncludePad, divisor)
        pt, pb, pl, pr = pads
        if pt != pb or pl != pr:
            gi = gi[:, :, pt:gi.shape[2] - pb, pl:gi.shape[3] - pr]
        return self._post(gi, batched)


class TemporalMaxPooling(AutogradModule):
    def __init__(self, k_w, d_w=-1, bigdl_type="float"):
        super().__init__()
        self.kW, self.dW = k_w, (d_w if d_w != -1 else k_w)

    def _forward(self, x):
        batched = x.dim() == 3
        if not batched:
            x = x.unsqueeze(0)
        y = F.max_pool1d(x.transpose(1, 2), self.kW, self.dW).transpose(1, 2)
        return y if batched else y.squeeze(0)


class VolumetricMaxPooling(AutogradModule):
    def __init__(self, k_t, k_w, k_h, d_t, d_w, d_h, pad_t=0, pad_w=0, pad_h=0, bigdl_type="float"):
        super().__init__()
        self.k, self.d, self.p = (k_t, k_h, k_w), (d_t, d_h, d_w), (pad_t, pad_h, pad_w)
        self.ceilMode = False

    def ceil(self):
        self.ceilMode = True
        return self

    def _forward(self, x):
        batched = x.dim() == 5
        if not batched:
            x = x.unsqueeze(0)
        y = NotImplemented
        if x.is_cuda and x.dtype == torch.bfloat16 and ops.native_has("pool3d"):
            y = ops.native_ops.pool3d(x.contiguous(memory_format=torch.channels_last_3d), 0, self.k, self.d, self.p,
                                      self.ceilMode)
        if y is NotImplemented:
            y = F.max_pool3d(x, self.k, self.d, self.p, ceil_mode=self.ceilMode)
        return y if batched else y.squeeze(0)


class VolumetricAveragePooling(AutogradModule):
    def __init__(self, k_t, k_w, k_h, d_t, d_w, d_h, pad_t=0, pad_w=0, pad_h=0, count_include_pad=True,
                 ceil_mode=False, bigdl_type="float"):
        super().__init__()
        self.k, self.d, self.p = (k_t, k_h, k_w), (d_t, d_h, d_w), (pad_t, pad_h, pad_w)
        self.countIncludePad, self.ceilMode = count_include_pad, ceil_mode

    def _forward(self, x):
        batched = x.dim() == 5
        if not batched:
            x = x.unsqueeze(0)
        y = NotImplemented
        if x.is_cuda and x.dtype == torch.bfloat16 and ops.native_has("pool3d"):
            y = ops.native_ops.pool3d(x.contiguous(memory_format=torch.channels_last_3d), 1, self.k, self.d, self.p,
                                      self.ceilMode, self.countIncludePad)
        if y is NotImplemented:
            y = F.avg_pool3d(x, self.k, self.d, self.p, self.ceilMode, self.countIncludePad)
        return y if batched else y.squeeze(0)


class RoiPooling(AutogradModule):
    """Max-pool each ROI (batch_idx, x1, y1, x2, y2) to (pooledH, pooledW) (``RoiPooling.scala``)."""

    def __init__(self, pooled_w, pooled_h, spatial_scale, bigdl_type="float"):
        super().__init__()
        self.pooledW, self.pooledH, self.spatialScale = pooled_w, pooled_h, spatial_scale

    def _forward(self, x):
        data, rois = x[1], x[2]
        outs = []
        H, W = data.shape[2], data.shape[3]
        for r in rois.tolist():
            b = int(r[0])
            x1, y1, x2, y2 = [int(round(v * self.spatialScale)) for v in r[1:5]]
            rh = max(y2 - y1 + 1, 1)
            rw = max(x2 - x1 + 1, 1)
            bh, bw = rh / self.pooledH, rw / self.pooledW
            cells = []
            for ph in range(self.pooledH):
                hs = min(max(int(math.floor(ph * bh)) + y1, 0), H)
                he = min(max(int(math.ceil((ph + 1) * bh)) + y1, 0), H)
                row = []
                for pw in range(self.pooledW):
                    ws = min(max(int(math.floor(pw * bw)) + x1, 0), W)
                    we = min(max(int(math.ceil((pw + 1) * bw)) + x1, 0), W)
                    if he <= hs or we <= ws:
                        row.append(torch.zeros(data.shape[1], dtype=data.dtype, device=data.device))
                    else:
                        row.append(data[b, :, hs:he, ws:we].amax(dim=(1, 2)))
                cells.append(torch.stack(row, -1))
            outs.append(torch.stack(cells, -2))
        return torch.stack(outs, 0)


def roi_align(data: torch.Tensor, rois: torch.Tensor, spatial_scale: float, out_h: int, out_w: int,
              sampling_ratio: int = 2, aligned: bool = True, chunk: int = 256) -> torch.Tensor:
    """Bilinear ROI align over NCHW ``data`` for ``rois [K, 5]`` (batch index, x1, y1, x2, y2),
    averaging ``sampling_ratio²`` samples per bin (``RoiAlign.scala``).  Gather-based and batched
    over ROIs (chunks of ``chunk`` to bound the K·S·C sample tensor); differentiable via autograd."""
    K = rois.shape[0]
    N, C, H, W = data.shape
    if K == 0:
        return data.new_zeros((0, C, out_h, out_w))
    if data.is_cuda:
        from ...ops import native as NO
        if NO.has("roi_align"):
            y = NO.native_ops.roi_align(data, rois, spatial_scale, out_h, out_w, sampling_ratio, aligned)
            if y is not NotImplemented:
                return y
            NO.note_fallback("roi_align", "shape/dtype", (data, rois))
    off = 0.5 if aligned else 0.0
    if sampling_ratio <= 0:
        # adaptive grid: ceil(roi_size / bins) samples per bin, per ROI — group ROIs sharing a grid
        r = acc_float(rois)
        rw = ((r[:, 3] - r[:, 1]) * spatial_scale).clamp_min(0.0 if aligned else 1.0)
        rh = ((r[:, 4] - r[:, 2]) * spatial_scale).clamp_min(0.0 if aligned else 1.0)
        gh = torch.ceil(rh / out_h).clamp_min(1).long()
        gw = torch.ceil(rw / out_w).clamp_min(1).long()
        out = data.new_zeros((K, C, out_h, out_w))
        for key in torch.unique(torch.stack([gh, gw], 1), dim=0).tolist():
            idx = torch.nonzero((gh == key[0]) & (gw == key[1])).flatten()
            out[idx] = _roi_align_grid(data, rois[idx], spatial_scale, out_h, out_w, key[0], key[1], off,
                                       aligned, chunk).to(data.dtype)
        return out
    sr = int(sampling_ratio)
    return _roi_align_grid(data, rois, spatial_scale, out_h, out_w, sr, sr, off, aligned, chunk).to(data.dtype)


def _roi_align_grid(data, rois, spatial_scale, out_h, out_w, srh, srw, off, aligned, chunk):
    K = rois.shape[0]
    N, C, H, W = data.shape
    d = data.permute(0, 2, 3, 1).float()  # N, H, W, C
    gy = (torch.arange(out_h * srh, device=data.device, dtype=torch.float32) + 0.5) / srh
    gx = (torch.arange(out_w * srw, device=data.device, dtype=torch.float32) + 0.5) / srw
    outs = []
    for s in range(0, K, chunk):
        r = acc_float(rois[s:s + chunk])
        k = r.shape[0]
        bi = r[:, 0].long()
        x1 = r[:, 1] * spatial_scale - off
        y1 = r[:, 2] * spatial_scale - off
        x2 = r[:, 3] * spatial_scale - off
        y2 = r[:, 4] * spatial_scale - off
        rw = (x2 - x1) if aligned else (x2 - x1).clamp_min(1.0)
        rh = (y2 - y1) if aligned else (y2 - y1).clamp_min(1.0)
        ys = y1[:, None] + gy[None, :] * (rh / out_h)[:, None]  # k, oh·sr
        xs = x1[:, None] + gx[None, :] * (rw / out_w)[:, None]
        Y = ys[:, :, None].expand(k, out_h * srh, out_w * srw)
        X = xs[:, None, :].expand(k, out_h * srh, out_w * srw)
        valid = (Y >= -1.0) & (Y <= H) & (X >= -1.0) & (X <= W)
        Y = Y.clamp(0, H - 1)
        X = X.clamp(0, W - 1)
        y0 = Y.floor().long()
        x0 = X.floor().long()
        y1i = (y0 + 1).clamp_max(H - 1)
        x1i = (x0 + 1).clamp_max(W - 1)
        ly, lx = Y - y0, X - x0
        hy, hx = 1 - ly, 1 - lx
        b = bi[:, None, None].expand_as(y0)
        v = (d[b, y0, x0] * (hy * hx)[..., None] + d[b, y0, x1i] * (hy * lx)[..., None] +
             d[b, y1i, x0] * (ly * hx)[..., None] + d[b, y1i, x1i] * (ly * lx)[..., None])
        v = v * valid[..., None]
        v = v.view(k, out_h, srh, out_w, srw, C).mean((2, 4))
        outs.append(v.permute(0, 3, 1, 2))
    return torch.cat(outs)


class RoiAlign(AutogradModule):
    """Bilinear ROI align (``RoiAlign.scala:45``): Table(data NCHW, rois (K, 4) on image 0 or (K, 5)
    with a leading batch index); ``aligned=False`` is the reference's sampling (no half-pixel shift,
    ROI sizes clamped to ≥1); ``samplingRatio ≤ 0`` picks ceil(roi/bin) samples per bin."""

    def __init__(self, spatial_scale, sampling_ratio, pooled_h, pooled_w, mode="avg", aligned=False,
                 bigdl_type="float"):
        super().__init__()
        self.spatialScale, self.samplingRatio = spatial_scale, sampling_ratio
        self.pooledH, self.pooledW, self.aligned = pooled_h, pooled_w, aligned

    def _forward(self, x):
        data, rois = x[1], x[2]
        if rois.shape[-1] == 4:
            rois = torch.cat([torch.zeros(rois.shape[0], 1, dtype=rois.dtype, device=rois.device), rois], 1)
        return roi_align(data, rois, self.spatialScale, self.pooledH, self.pooledW, self.samplingRatio, self.aligned)


class UpSampling1D(AutogradModule):
    def __init__(self, length, bigdl_type="float"):
        super().__init__()
        self.length = length

    def _forward(self, x):
        return x.repeat_interleave(self.length, dim=-2)


class UpSampling2D(AutogradModule):
    def __init__(self, size, data_format="nchw", bigdl_type="float"):
        super().__init__()
        self.size, self.format = list(size), data_format.lower()

    def _forward(self, x):
        hd, wd = (2, 3) if self.format == "nchw" else (1, 2)
        return x.repeat_interleave(self.size[0], dim=hd).repeat_interleave(self.size[1], dim=wd)


class UpSampling3D(AutogradModule):
    def __init__(self, size, bigdl_type="float"):
        super().__init__()
        self.size = list(size)

    def _forward(self, x):
        return x.repeat_interleave(self.size[0], 2).repeat_interleave(self.size[1], 3).repeat_interleave(self.size[2], 4)


class ResizeBilinear(AutogradModule):
    def __init__(self, output_height, output_width, align_corner=False, data_format="NCHW", bigdl_type="float"):
        super().__init__()
        self.oh, self.ow, self.alignCorners, self.format = output_height, output_width, align_corner, data_format

    def _forward(self, x):
        """TensorFlow-style sampling as the reference (``nn/ResizeBilinear.scala:266-284,406-412``:
        src = dst·in/out, no half-pixel offset) — not ``F.interpolate``'s half-pixel centres."""
        nhwc = self.format == "NHWC"
        if nhwc:
            x = x.permute(0, 3, 1, 2)
        y = NotImplemented
        if x.is_cuda and ops.native_has("resize_bilinear"):
            xd = x if x.dtype != torch.bfloat16 else x.contiguous(memory_format=torch.channels_last)
            y = ops.native_ops.resize_bilinear(xd, self.oh, self.ow, self.alignCorners)
        if y is NotImplemented:
            from ...ops.reference import resize_bilinear
            y = resize_bilinear(x, self.oh, self.ow, self.alignCorners)
        return y.permute(0, 2, 3, 1) if nhwc else y
