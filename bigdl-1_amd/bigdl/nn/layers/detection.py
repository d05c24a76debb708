"""Object-detection layers (Faster/Mask R-CNN and SSD): ``Anchor``, ``Nms``, ``Proposal``,
``RegionProposal``, ``PriorBox``, ``DetectionOutputSSD``, ``DetectionOutputFrcnn``, ``Pooler``,
``FPN``, ``BoxHead``, ``MaskHead`` (``DL/nn/{Anchor,Nms,Proposal,RegionProposal,PriorBox,
DetectionOutputSSD,DetectionOutputFrcnn,Pooler,FPN,BoxHead,MaskHead}.scala``) plus a vectorised
``roi_align``.

Design: everything runs on the tensors' device with batched torch ops (IoU matrices, top-k,
gather-based bilinear sampling) — no per-box host loops except NMS's inherently sequential greedy
scan, which walks a device-computed suppression bitmask on the host.  Post-processing layers are
inference-only (in training they pass their input through, as the reference does); the trainable
heads (FPN, BoxHead, MaskHead, RegionProposal's conv head) are ordinary modules.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F

from ...utils.table import Table
from ..abstractnn import AbstractModule, TensorModule
from ..containers import Sequential
from .conv import SpatialConvolution
from .activation import ReLU, SoftMax
from .linear import Linear
from .pooling import roi_align  # noqa: F401  (re-exported)


# ------------------------------------------------------------------------------------------------ anchors / nms
class Anchor:
    """Faster R-CNN anchors (``Anchor.scala``): ``ratios × scales`` basic anchors around a
    ``base_size``-pixel cell, shifted over a ``width × height`` feature map with stride
    ``feat_stride``; output ``[H·W·A, 4]`` ordered (y, x, anchor)."""

    def __init__(self, ratios: Sequence[float], scales: Sequence[float]):
        self.ratios = [float(r) for r in ratios]
        self.scales = [float(s) for s in scales]
        self.anchor_num = len(self.ratios) * len(self.scales)
        self._base = None
        self._base_size = None

    anchorNum = property(lambda self: self.anchor_num)

    @staticmethod
    def _whctr(a):
        w = a[2] - a[0] + 1
        h = a[3] - a[1] + 1
        return w, h, a[0] + 0.5 * (w - 1), a[1] + 0.5 * (h - 1)

    @staticmethod
    def _mk(ws, hs, xc, yc):
        return [[xc - (w / 2 - 0.5), yc - (h / 2 - 0.5), xc + (w / 2 - 0.5), yc + (h / 2 - 0.5)] for w, h in zip(ws, hs)]

    def basic_anchors(self, base_size: float = 16.0) -> torch.Tensor:
        base = [0.0, 0.0, base_size - 1, base_size - 1]
        w, h, xc, yc = self._whctr(base)
        area = w * h
        ws = [float(round(math.sqrt(area / r))) for r in self.ratios]
        hs = [float(round(wv * r)) for wv, r in zip(ws, self.ratios)]
        out = []
        for ra in self._mk(ws, hs, xc, yc):
            w2, h2, xc2, yc2 = self._whctr(ra)
            out += self._mk([s * w2 for s in self.scales], [s * h2 for s in self.scales], xc2, yc2)
        return torch.tensor(out, dtype=torch.float32)

    generateBasicAnchors = basic_anchors

    def generate_anchors(self, width: int, height: int, feat_stride: float = 16.0, device=None) -> torch.Tensor:
        if self._base is None or self._base_size != feat_stride:
            self._base = self.basic_anchors(feat_stride)
            self._base_size = feat_stride
        base = self._base.to(device) if device is not None else self._base
        sx = torch.arange(width, device=base.device, dtype=torch.float32) * feat_stride
        sy = torch.arange(height, device=base.device, dtype=torch.float32) * feat_stride
        yy, xx = torch.meshgrid(sy, sx, indexing="ij")
        shifts = torch.stack([xx, yy, xx, yy], -1).reshape(-1, 1, 4)
        return (shifts + base.view(1, -1, 4)).reshape(-1, 4)

    generateAnchors = generate_anchors


def box_iou(a: torch.Tensor, b: torch.Tensor, plus_one: float = 1.0) -> torch.Tensor:
    lt = torch.max(a[:, None, :2], b[None, :, :2])
    rb = torch.min(a[:, None, 2:], b[None, :, 2:])
    wh = (rb - lt + plus_one).clamp_min(0)
    inter = wh[..., 0] * wh[..., 1]
    aa = ((a[:, 2] - a[:, 0] + plus_one) * (a[:, 3] - a[:, 1] + plus_one))[:, None]
    ab = ((b[:, 2] - b[:, 0] + plus_one) * (b[:, 3] - b[:, 1] + plus_one))[None, :]
    return inter / (aa + ab - inter).clamp_min(1e-12)


def nms(boxes: torch.Tensor, scores: torch.Tensor, thresh: float, plus_one: float = 1.0,
        max_keep: int = -1) -> torch.Tensor:
    """Greedy non-maximum suppression; returns kept indices (0-based, descending score).
    IoU > thresh suppresses (``Nms.scala``).  The N×N overlap test runs on the device; the greedy
    scan walks the resulting bitmask on the host."""
    n = boxes.shape[0]
    if n == 0:
        return torch.zeros(0, dtype=torch.long, device=boxes.device)
    order = torch.argsort(scores, descending=True)
    b = boxes[order].float()
    if b.is_cuda:
        from ...ops import native as N
        if N.has("nms"):
            k = N.native_ops.nms(b, thresh, plus_one, max_keep)  # device bitmask + one-wave scan
            if k is not NotImplemented:
                return order[k]
            N.note_fallback("nms", "size", (b,))
    over = (box_iou(b, b, plus_one) > thresh).cpu().numpy()
    keep = []
    removed = np.zeros(n, dtype=bool)
    for i in range(n):
        if removed[i]:
            continue
        keep.append(i)
        if 0 < max_keep <= len(keep):
            break
        removed |= over[i]
    return order[torch.as_tensor(keep, dtype=torch.long, device=boxes.device)]


class Nms:
    """``Nms.scala`` API: ``nms(scores, boxes, thresh, indices, sorted)`` fills ``indices``
    (1-based positions into the inputs) and returns the kept count."""

    def nms(self, scores, boxes, thresh, indices=None, sorted=False, order_with_bbox=False):
        keep = nms(boxes, scores, thresh)
        if indices is not None:
            k = keep.cpu().numpy() + 1
            indices[:len(k)] = k
        return int(keep.numel())


def bbox_transform_inv(boxes: torch.Tensor, deltas: torch.Tensor, weights=(1.0, 1.0, 1.0, 1.0)) -> torch.Tensor:
    from ...transform.vision.image.label.roi import BboxUtil
    return BboxUtil.bbox_transform_inv(boxes, deltas, weights)


def clip_boxes(boxes: torch.Tensor, h: float, w: float) -> torch.Tensor:
    out = boxes.clone()
    out[:, 0::2] = out[:, 0::2].clamp(0, w - 1)
    out[:, 1::2] = out[:, 1::2].clamp(0, h - 1)
    return out


class _Composite(AbstractModule):
    """A module built from sub-modules that forward()s through a custom dataflow."""

    def children(self):
        return list(self.modules)

    def parameters(self):
        ws, gs = [], []
        for m in self.modules:
            p = m.parameters()
            if p is not None:
                ws += p[0]
                gs += p[1]
        return (ws, gs) if ws else None

    def _param_entries(self):
        out = []
        for m in self.modules:
            out += m._param_entries()
        return out

    def _set_arena_recursive(self, arena):
        self._arena = arena
        for m in self.modules:
            m._set_arena_recursive(arena)


# ------------------------------------------------------------------------------------------------ RPN
class Proposal(AbstractModule):
    """RPN proposals (``Proposal.scala``): input Table(scores [1, 2A, H, W], deltas [1, 4A, H, W],
    im_info [1, 4] = (h, w, scale_h, scale_w)) → rois [K, 5] (batch 0, x1, y1, x2, y2)."""

    def __init__(self, pre_nms_topn_test, post_nms_topn_test, ratios, scales, rpn_pre_nms_topn_train,
                 rpn_post_nms_topn_train, min_size=16, nms_thresh=0.7, feat_stride=16.0):
        super().__init__()
        self.preNmsTopNTest, self.postNmsTopNTest = pre_nms_topn_test, post_nms_topn_test
        self.rpnPreNmsTopNTrain, self.rpnPostNmsTopNTrain = rpn_pre_nms_topn_train, rpn_post_nms_topn_train
        self.ratios, self.scales = list(ratios), list(scales)
        self.anchor = Anchor(ratios, scales)
        self.minSize, self.nmsThresh, self.featStride = min_size, nms_thresh, feat_stride

    def updateOutput(self, input):
        score, deltas, im_info = input[1], input[2], input[3]
        A = self.anchor.anchor_num
        H, W = score.shape[2], score.shape[3]
        fg = score[0, A:2 * A].permute(1, 2, 0).reshape(-1).float()
        d = deltas[0].permute(1, 2, 0).reshape(-1, 4).float()
        anchors = self.anchor.generate_anchors(W, H, self.featStride, device=score.device)
        props = bbox_transform_inv(anchors, d)
        ih, iw = float(im_info[0, 0]), float(im_info[0, 1])
        props = clip_boxes(props, ih, iw)
        ms_h, ms_w = self.minSize * float(im_info[0, 2]), self.minSize * float(im_info[0, 3])
        keep = ((props[:, 2] - props[:, 0] + 1) >= ms_w) & ((props[:, 3] - props[:, 1] + 1) >= ms_h)
        props, fg = props[keep], fg[keep]
        pre = self.rpnPreNmsTopNTrain if self.train else self.preNmsTopNTest
        post = self.rpnPostNmsTopNTrain if self.train else self.postNmsTopNTest
        top = torch.topk(fg, min(pre, fg.numel())).indices
        props, fg = props[top], fg[top]
        k = nms(props, fg, self.nmsThresh)
        if post > 0:
            k = k[:post]
        rois = props[k]
        return torch.cat([rois.new_zeros(rois.shape[0], 1), rois], 1)

    def updateGradInput(self, input, gradOutput):
        return Table(*[torch.zeros_like(input[i]) for i in (1, 2, 3)])


class RegionProposal(_Composite):
    """FPN region proposal network (``RegionProposal.scala``): a shared 3×3 conv + ReLU head with
    objectness (A) and box-delta (4A) 1×1 convs per level, anchors per level
    (``anchorSizes[i]`` × ``aspectRatios`` at ``anchorStride[i]``), decoding, per-level top-k,
    NMS and a final top-k.  Input Table(features..., im_info); output rois [K, 4]."""

    def __init__(self, in_channels, anchor_sizes, aspect_ratios, anchor_stride, pre_nms_topn_test=1000,
                 post_nms_topn_test=1000, pre_nms_topn_train=2000, post_nms_topn_train=2000, nms_thread=0.7,
                 min_size=0):
        super().__init__()
        self.inChannels, self.anchorSizes = in_channels, list(anchor_sizes)
        self.aspectRatios, self.anchorStride = list(aspect_ratios), list(anchor_stride)
        self.preNmsTopNTest, self.postNmsTopNTest = pre_nms_topn_test, post_nms_topn_test
        self.preNmsTopNTrain, self.postNmsTopNTrain = pre_nms_topn_train, post_nms_topn_train
        self.nmsThread, self.minSize = nms_thread, min_size
        A = len(self.aspectRatios)
        self.conv = SpatialConvolution(in_channels, in_channels, 3, 3, 1, 1, 1, 1)
        self.cls = SpatialConvolution(in_channels, A, 1, 1)
        self.bbox = SpatialConvolution(in_channels, 4 * A, 1, 1)
        self.relu = ReLU()
        self.modules = [self.conv, self.cls, self.bbox, self.relu]

    def _anchors(self, i, H, W, dev):
        size = self.anchorSizes[i]
        stride = self.anchorStride[i]
        a = Anchor(self.aspectRatios, [size / stride])
        return a.generate_anchors(W, H, stride, device=dev)

    def updateOutput(self, input):
        feats = input[1]
        feats = [feats[i + 1] for i in range(len(feats))] if isinstance(feats, Table) else [feats]
        im = input[2].flatten()
        ih, iw = float(im[0]), float(im[1])
        pre = self.preNmsTopNTrain if self.train else self.preNmsTopNTest
        post = self.postNmsTopNTrain if self.train else self.postNmsTopNTest
        heads = []
        for i, f in enumerate(feats):
            t = self.relu.forward(self.conv.forward(f))
            heads.append((self.cls.forward(t).float(), self.bbox.forward(t).float()))
        out = Table()
        for b in range(feats[0].shape[0]):
            all_b, all_s = [], []
            for i, (obj_all, reg_all) in enumerate(heads):
                obj, reg = obj_all[b], reg_all[b]
                H, W = obj.shape[1], obj.shape[2]
                s = torch.sigmoid(obj.permute(1, 2, 0).reshape(-1))
                d = reg.view(-1, 4, H, W).permute(2, 3, 0, 1).reshape(-1, 4)
                anchors = self._anchors(i, H, W, obj.device)
                top = torch.topk(s, min(pre, s.numel())).indices
                boxes = clip_boxes(bbox_transform_inv(anchors[top], d[top]), ih, iw)
                s = s[top]
                keep = ((boxes[:, 2] - boxes[:, 0] + 1) >= self.minSize) & \
                       ((boxes[:, 3] - boxes[:, 1] + 1) >= self.minSize)
                boxes, s = boxes[keep], s[keep]
                k = nms(boxes, s, self.nmsThread)[:post]
                all_b.append(boxes[k])
                all_s.append(s[k])
            bx, sc = torch.cat(all_b), torch.cat(all_s)
            top = torch.topk(sc, min(post, sc.numel())).indices
            out.insert(bx[top])
        return out

    def updateGradInput(self, input, gradOutput):
        raise NotImplementedError("RegionProposal: proposal selection is inference-only (RegionProposal.scala)")


# ------------------------------------------------------------------------------------------------ SSD
class PriorBox(TensorModule):
    """SSD prior boxes (``PriorBox.scala``): output [1, 2, H·W·P·4] — normalised priors and their
    variances for a feature map of the input's spatial size."""

    def __init__(self, min_sizes, max_sizes=None, aspect_ratios=None, is_flip=True, is_clip=False, variances=None,
                 offset=0.5, img_h=0, img_w=0, img_size=0, step_h=0.0, step_w=0.0, step=0.0):
        super().__init__()
        self.minSizes = list(min_sizes)
        self.maxSizes = list(max_sizes) if max_sizes else []
        ars = [1.0]
        for a in (aspect_ratios or []):
            if all(abs(a - x) > 1e-6 for x in ars):
                ars.append(a)
                if is_flip:
                    ars.append(1.0 / a)
        self.aspectRatios = ars
        self.isClip = is_clip
        self.variances = list(variances) if variances else [0.1]
        self.offset = offset
        self.imgH, self.imgW = (img_size, img_size) if img_size else (img_h, img_w)
        self.stepH, self.stepW = (step, step) if step else (step_h, step_w)
        self.numPriors = len(self.aspectRatios) * len(self.minSizes) + len(self.maxSizes)

    def updateOutput(self, input):
        x = input[1] if isinstance(input, Table) else input
        H, W = x.shape[-2], x.shape[-1]
        img = input[2] if isinstance(input, Table) and len(input) > 1 else None
        ih = self.imgH or (img.shape[-2] if img is not None else H)
        iw = self.imgW or (img.shape[-1] if img is not None else W)
        sh = self.stepH or ih / H
        sw = self.stepW or iw / W
        boxes = []
        for h in range(H):
            for w in range(W):
                cx, cy = (w + self.offset) * sw, (h + self.offset) * sh
                for i, ms in enumerate(self.minSizes):
                    ms = float(int(ms))  # sizes are truncated to integers (PriorBox.scala:168)
                    boxes.append((cx, cy, ms, ms))
                    if self.maxSizes:
                        s = math.sqrt(ms * int(self.maxSizes[i]))
                        boxes.append((cx, cy, s, s))
                    for a in self.aspectRatios:
                        if abs(a - 1.0) < 1e-6:
                            continue
                        boxes.append((cx, cy, ms * math.sqrt(a), ms / math.sqrt(a)))
        b = torch.tensor(boxes, dtype=torch.float32)
        pri = torch.stack([(b[:, 0] - b[:, 2] / 2) / iw, (b[:, 1] - b[:, 3] / 2) / ih,
                           (b[:, 0] + b[:, 2] / 2) / iw, (b[:, 1] + b[:, 3] / 2) / ih], 1)
        if self.isClip:
            pri = pri.clamp(0, 1)
        var = torch.tensor(self.variances * (4 // len(self.variances)) if len(self.variances) < 4
                           else self.variances, dtype=torch.float32).repeat(pri.shape[0])
        return torch.stack([pri.reshape(-1), var]).unsqueeze(0).to(x.device)

    def updateGradInput(self, input, gradOutput):
        return torch.zeros_like(input) if isinstance(input, torch.Tensor) else \
            Table(*[torch.zeros_like(v) for v in input.values()])


class DetectionOutputSSD(AbstractModule):
    """SSD post-processing (``DetectionOutputSSD.scala``): Table(loc [B, P·4], conf [B, P·nC],
    priors [1, 2, P·4]) → [B, 1 + maxDet·6] rows (count, then label, score, x1, y1, x2, y2 …)."""

    def __init__(self, n_classes=21, share_location=True, bg_label=0, nms_thresh=0.45, nms_topk=400,
                 keep_top_k=200, conf_thresh=0.01, variance_encoded_in_target=False, conf_post_process=True):
        super().__init__()
        self.nClasses, self.shareLocation, self.bgLabel = n_classes, share_location, bg_label
        self.nmsThresh, self.nmsTopk, self.keepTopK = nms_thresh, nms_topk, keep_top_k
        self.confThresh, self.varianceEncodedInTarget = conf_thresh, variance_encoded_in_target
        self.confPostProcess = conf_post_process

    def updateOutput(self, input):
        if self.train:
            return input
        loc, conf, prior = input[1].float(), input[2].float(), input[3].float()
        B = loc.shape[0]
        P = prior.shape[-1] // 4
        pri = prior[0, 0].view(P, 4)
        var = prior[0, 1].view(P, 4)
        conf = conf.view(B, P, self.nClasses)
        if self.confPostProcess:
            conf = torch.softmax(conf, -1)
        loc = loc.view(B, P, 4)
        results = []
        for b in range(B):
            pw, ph = pri[:, 2] - pri[:, 0], pri[:, 3] - pri[:, 1]
            pcx, pcy = (pri[:, 0] + pri[:, 2]) / 2, (pri[:, 1] + pri[:, 3]) / 2
            v = var if not self.varianceEncodedInTarget else torch.ones_like(var)
            cx = v[:, 0] * loc[b, :, 0] * pw + pcx
            cy = v[:, 1] * loc[b, :, 1] * ph + pcy
            w = torch.exp(v[:, 2] * loc[b, :, 2]) * pw
            h = torch.exp(v[:, 3] * loc[b, :, 3]) * ph
            boxes = torch.stack([cx - w / 2, cy - h / 2, cx + w / 2, cy + h / 2], 1)
            dets = []
            for c in range(self.nClasses):
                if c == self.bgLabel:
                    continue
                sc = conf[b, :, c]
                m = sc > self.confThresh
                if not m.any():
                    continue
                bs, ss = boxes[m], sc[m]
                if ss.numel() > self.nmsTopk:
                    t = torch.topk(ss, self.nmsTopk).indices
                    bs, ss = bs[t], ss[t]
                k = nms(bs, ss, self.nmsThresh, plus_one=0.0)
                for i in k.tolist():
                    dets.append((float(ss[i]), c, bs[i]))
            dets.sort(key=lambda d: -d[0])
            if self.keepTopK > -1:
                dets = dets[:self.keepTopK]
            dets.sort(key=lambda d: d[1])
            results.append(dets)
        maxd = max((len(d) for d in results), default=0)
        out = torch.zeros(B, 1 + maxd * 6)
        for b, dets in enumerate(results):
            out[b, 0] = len(dets)
            for j, (s, c, bx) in enumerate(dets):
                out[b, 1 + 6 * j:1 + 6 * j + 6] = torch.tensor([c, s] + bx.tolist())
        return out

    def updateGradInput(self, input, gradOutput):
        return gradOutput


class DetectionOutputFrcnn(AbstractModule):
    """Faster R-CNN post-processing (``DetectionOutputFrcnn.scala``): Table(im_info, rois,
    bbox_pred [N, 4·nC], cls_prob [N, nC]) → [1 + K·6] (count, label, score, box …) per image."""

    def __init__(self, nms_thresh=0.3, n_classes=21, bbox_vote=False, max_per_image=100, thresh=0.05):
        super().__init__()
        self.nmsThresh, self.nClasses, self.bboxVote = nms_thresh, n_classes, bbox_vote
        self.maxPerImage, self.thresh = max_per_image, thresh

    def updateOutput(self, input):
        if self.train:
            return input
        im_info = input[1]
        rois = input[2][1] if isinstance(input[2], Table) else input[2]
        deltas, scores = input[3].float(), input[4].float()
        scale = float(im_info[0, 2])
        boxes = rois[:, 1:5].float() / scale
        pred = clip_boxes(bbox_transform_inv(boxes, deltas).view(-1, 4),
                          float(im_info[0, 0]) / scale, float(im_info[0, 1]) / float(im_info[0, 3])
                          ).view(deltas.shape)
        dets = []
        for c in range(1, self.nClasses):
            m = scores[:, c] > self.thresh
            if not m.any():
                continue
            bs = pred[m, 4 * c:4 * c + 4]
            ss = scores[m, c]
            k = nms(bs, ss, self.nmsThresh)
            for i in k.tolist():
                dets.append((float(ss[i]), c, bs[i]))
        dets.sort(key=lambda d: -d[0])
        if self.maxPerImage > 0:
            dets = dets[:self.maxPerImage]
        out = torch.zeros(1 + 6 * len(dets))
        out[0] = len(dets)
        for j, (s, c, b) in enumerate(dets):
            out[1 + 6 * j:7 + 6 * j] = torch.tensor([c, s] + b.tolist())
        return out

    def updateGradInput(self, input, gradOutput):
        return gradOutput


# ------------------------------------------------------------------------------------------------ FPN / heads
class Pooler(AbstractModule):
    """Multi-level ROI align (``Pooler.scala:33``): ROI k goes to level
    ``floor(4 + log2(sqrt(area_k) / 224 + 1e-6))`` clamped to the available levels (canonical scale
    224 at level 4), then ``RoiAlign`` (reference sampling) at that level's ``scale``.  Input
    Table(Table(feature maps), rois [K, 4] or Table(per-image rois)) → [ΣK, C, R, R]."""

    def __init__(self, resolution, scales, sampling_ratio):
        super().__init__()
        self.resolution, self.scales, self.samplingRatio = resolution, list(scales), sampling_ratio
        self.lvl_min = int(-math.log(self.scales[0]) / math.log(2.0))
        self.lvl_max = int(-math.log(self.scales[-1]) / math.log(2.0))

    def level_mapping(self, rois: torch.Tensor) -> torch.Tensor:
        r = rois.float()
        area = (r[:, 2] - r[:, 0] + 1) * (r[:, 3] - r[:, 1] + 1)
        lvl = torch.floor(4 + torch.log2(torch.sqrt(area) / 224 + 1e-6)).clamp(self.lvl_min, self.lvl_max)
        return (lvl - self.lvl_min).long()

    def updateOutput(self, input):
        feats = input[1]
        feats = [feats[i + 1] for i in range(len(feats))] if isinstance(feats, Table) else [feats]
        rb = input[2]
        per_image = [rb[i + 1] for i in range(len(rb))] if isinstance(rb, Table) else [rb]
        C, R = feats[0].shape[1], self.resolution
        outs = []
        for b, rois in enumerate(per_image):
            rois = rois[:, -4:]
            lvl = self.level_mapping(rois)
            out = feats[0].new_zeros((rois.shape[0], C, R, R))
            for i, (f, s) in enumerate(zip(feats, self.scales)):
                idx = torch.nonzero(lvl == i).flatten()
                if idx.numel():
                    r5 = torch.cat([rois.new_zeros(idx.numel(), 1), rois[idx]], 1)
                    out[idx] = roi_align(f[b:b + 1], r5, s, R, R, self.samplingRatio, aligned=False).to(out.dtype)
            outs.append(out)
        return torch.cat(outs)

    def updateGradInput(self, input, gradOutput):
        raise NotImplementedError("Pooler: backward not supported (Pooler.scala:160)")


class FPN(_Composite):
    """Feature pyramid (``FPN.scala:30``): lateral 1×1 convs, top-down nearest ×2 upsampling + add,
    3×3 output convs; optional P6 (max-pool of the top) or P6/P7 convs (``topBlocks``).  Input
    Table(C2..C5) → Table(P2..P5[, P6[, P7]])."""

    def __init__(self, in_channels, out_channels, top_blocks=0, in_channels_of_p6p7=0, out_channels_of_p6p7=0):
        super().__init__()
        self.inChannels, self.outChannels, self.topBlocks = list(in_channels), out_channels, top_blocks
        self.inChannelsOfP6P7, self.outChannelsOfP6P7 = in_channels_of_p6p7, out_channels_of_p6p7
        self.inner = [SpatialConvolution(c, out_channels, 1, 1) for c in self.inChannels]
        self.layer = [SpatialConvolution(out_channels, out_channels, 3, 3, 1, 1, 1, 1) for _ in self.inChannels]
        self.modules = self.inner + self.layer
        if top_blocks == 2:
            self.p6 = SpatialConvolution(in_channels_of_p6p7, out_channels_of_p6p7, 3, 3, 2, 2, 1, 1)
            self.p7 = SpatialConvolution(out_channels_of_p6p7, out_channels_of_p6p7, 3, 3, 2, 2, 1, 1)
            self.modules += [self.p6, self.p7]

    def updateOutput(self, input):
        n = len(self.inChannels)
        xs = [input[i + 1] for i in range(n)]
        last = self.inner[-1].forward(xs[-1])
        outs = [self.layer[-1].forward(last)]
        for i in range(n - 2, -1, -1):
            lat = self.inner[i].forward(xs[i])
            last = lat + last.repeat_interleave(2, dim=2).repeat_interleave(2, dim=3)  # UpSampling2D(2, 2)
            outs.insert(0, self.layer[i].forward(last))
        if self.topBlocks == 1:
            outs.append(outs[n - 1][:, :, ::2, ::2].contiguous())  # SpatialMaxPooling(1, 1, 2, 2)
        elif self.topBlocks == 2:
            src = outs[n - 1] if self.inChannelsOfP6P7 == self.outChannelsOfP6P7 else xs[-1]
            p6 = self.p6.forward(src)
            outs += [p6, self.p7.forward(torch.relu(p6))]
        return Table(*outs)

    def updateGradInput(self, input, gradOutput):
        raise NotImplementedError("FPN: backward not supported (FPN.scala)")


class BoxHead(_Composite):
    """Box head (``BoxHead.scala:30``): Pooler → FC(``outputSize``)+ReLU ×2 → class logits and
    per-class box deltas (weights 10, 10, 5, 5); in eval mode post-processed per image (softmax,
    decode, clip, per-class score threshold + NMS, top ``maxPerImage`` over classes).
    Input Table(features Table, proposals [K, 4] or Table(per-image), image_info [2+])
    → Table(box_features, Table(labels, Table(per-image boxes), scores))."""

    def __init__(self, in_channels, resolution, scales, sampling_ratio, score_thresh, nms_thresh, max_per_image,
                 output_size, num_classes):
        super().__init__()
        from ..initialization_method import Xavier, Zeros
        self.pooler = Pooler(resolution, scales, sampling_ratio)
        self.fc1 = Linear(in_channels * resolution * resolution, output_size).setInitMethod(Xavier(), Zeros())
        self.fc2 = Linear(output_size, output_size).setInitMethod(Xavier(), Zeros())
        self.cls = Linear(output_size, num_classes)
        self.bbox = Linear(output_size, num_classes * 4)
        with torch.no_grad():
            self.cls.weight.normal_(0, 0.01)
            self.cls.bias.zero_()
            self.bbox.weight.normal_(0, 0.001)
            self.bbox.bias.zero_()
        self.modules = [self.fc1, self.fc2, self.cls, self.bbox]
        self.scoreThresh, self.nmsThresh, self.maxPerImage, self.numClasses = score_thresh, nms_thresh, \
            max_per_image, num_classes

    def _post(self, probs, boxes):
        ob, ol, os_ = [], [], []
        for c in range(1, self.numClasses):
            m = probs[:, c] > self.scoreThresh
            if not m.any():
                continue
            bs, ss = boxes[m, 4 * c:4 * c + 4], probs[m, c]
            k = nms(bs, ss, self.nmsThresh)
            ob.append(bs[k])
            os_.append(ss[k])
            ol.append(torch.full((k.numel(),), float(c), device=bs.device))
        if not ob:
            e = boxes.new_zeros((0, 4))
            return e, e.new_zeros(0), e.new_zeros(0)
        b, l, s = torch.cat(ob), torch.cat(ol), torch.cat(os_)
        if self.maxPerImage > 0 and s.numel() > self.maxPerImage:
            thr = torch.topk(s, self.maxPerImage).values[-1]
            keep = s >= thr
            b, l, s = b[keep], l[keep], s[keep]
        return b, l, s

    def updateOutput(self, input):
        feats, props, info = input[1], input[2], input[3]
        x = self.pooler.forward(Table(feats, props)).flatten(1)
        x = torch.relu(self.fc2.forward(torch.relu(self.fc1.forward(x))))
        if self.train:
            return Table(x, Table(self.cls.forward(x), self.bbox.forward(x), props, info))
        logits, deltas = self.cls.forward(x).float(), self.bbox.forward(x).float()
        probs = torch.softmax(logits, -1)
        per_image = [props[i + 1] for i in range(len(props))] if isinstance(props, Table) else [props]
        cat = torch.cat([p[:, -4:].float() for p in per_image])
        boxes = bbox_transform_inv(cat, deltas, (10.0, 10.0, 5.0, 5.0))
        info = info.flatten()
        boxes = clip_boxes(boxes.view(-1, 4), float(info[0]), float(info[1])).view(boxes.shape)
        labels, bxs, scores, start = [], Table(), [], 0
        for p in per_image:
            n = p.shape[0]
            b, l, s = self._post(probs[start:start + n], boxes[start:start + n])
            start += n
            bxs.insert(b)
            labels.append(l)
            scores.append(s)
        return Table(x, Table(torch.cat(labels), bxs, torch.cat(scores)))


class MaskHead(_Composite):
    """Mask head (``MaskHead.scala:35``): Pooler → ``layers`` dilated 3×3 convs + ReLU (feature
    extractor) → 2×2 stride-2 deconv + ReLU → 1×1 conv to ``numClasses`` logits; the post-processor
    takes the sigmoid mask of each box's label.  Input Table(features Table, boxes, labels)
    → Table(mask_features, masks [K, 1, 2R, 2R])."""

    def __init__(self, in_channels, resolution, scales, sampling_ratio, layers, dilation, num_classes,
                 use_gn=False):
        super().__init__()
        from .conv import SpatialFullConvolution, SpatialDilatedConvolution
        from ..initialization_method import MsraFiller, Zeros
        self.pooler = Pooler(resolution, scales, sampling_ratio)
        convs, c = [], in_channels
        for l in layers:
            convs.append(SpatialDilatedConvolution(c, l, 3, 3, 1, 1, dilation, dilation, dilation, dilation)
                         .setInitMethod(MsraFiller(False), Zeros()))
            c = l
        self.convs = convs
        self.deconv = SpatialFullConvolution(c, c, 2, 2, 2, 2)
        self.logits = SpatialConvolution(c, num_classes, 1, 1).setInitMethod(MsraFiller(False), Zeros())
        self.modules = self.convs + [self.deconv, self.logits]
        self.numClasses, self.useGn = num_classes, use_gn

    def updateOutput(self, input):
        feats, boxes, labels = input[1], input[2], input[3]
        x = self.pooler.forward(Table(feats, boxes))
        for cv in self.convs:
            x = torch.relu(cv.forward(x))
        feat = x
        x = torch.relu(self.deconv.forward(x))
        m = torch.sigmoid(self.logits.forward(x).float())
        idx = labels.flatten().long().clamp(0, self.numClasses - 1)
        return Table(feat, m[torch.arange(m.shape[0], device=m.device), idx].unsqueeze(1))
