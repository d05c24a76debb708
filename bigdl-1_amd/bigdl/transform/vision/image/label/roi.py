"""Detection labels: ``RoiLabel(classes, bboxes, masks)`` and the transforms that keep boxes in
sync with image geometry (``label/roi/{RoiLabel,RoiTransformer}.scala``, ``util/BboxUtil.scala``).
Boxes are ``[N, 4]`` (x1, y1, x2, y2); ``classes`` is ``[N]`` or ``[2, N]`` (class, difficult)."""
from __future__ import annotations

from typing import Optional

import torch

from ..image_feature import FeatureTransformer, ImageFeature


class RoiLabel:
    def __init__(self, classes: torch.Tensor, bboxes: torch.Tensor, masks=None):
        self.classes = torch.as_tensor(classes, dtype=torch.float32)
        self.bboxes = torch.as_tensor(bboxes, dtype=torch.float32).reshape(-1, 4)
        self.masks = masks

    def size(self) -> int:
        return self.bboxes.shape[0]

    def copy(self):
        return RoiLabel(self.classes.clone(), self.bboxes.clone(), self.masks)

    def __repr__(self):
        return f"RoiLabel(n={self.size()})"


def _label(f) -> Optional[RoiLabel]:
    lab = f.get(ImageFeature.label)
    return lab if isinstance(lab, RoiLabel) else None


class RoiNormalize(FeatureTransformer):
    """Absolute pixel boxes → [0, 1] coordinates."""

    def transform_mat(self, f):
        lab = _label(f)
        if lab is None:
            return
        h, w = f.get_height(), f.get_width()
        lab.bboxes = lab.bboxes / torch.tensor([w, h, w, h], dtype=torch.float32)


class RoiHFlip(FeatureTransformer):
    def __init__(self, normalized: bool = True):
        self.normalized = normalized

    def transform_mat(self, f):
        lab = _label(f)
        if lab is None:
            return
        W = 1.0 if self.normalized else float(f.get_width())
        b = lab.bboxes.clone()
        b[:, 0] = W - lab.bboxes[:, 2]
        b[:, 2] = W - lab.bboxes[:, 0]
        lab.bboxes = b


class RoiResize(FeatureTransformer):
    """Scale absolute boxes from the original size to the current mat size."""

    def __init__(self, normalized: bool = False):
        self.normalized = normalized

    def transform_mat(self, f):
        lab = _label(f)
        if lab is None or self.normalized:
            return
        oh, ow = f.get_original_height(), f.get_original_width()
        h, w = f.get_height(), f.get_width()
        lab.bboxes = lab.bboxes * torch.tensor([w / ow, h / oh, w / ow, h / oh], dtype=torch.float32)


class RoiProject(FeatureTransformer):
    """Project normalised boxes into the last crop (``cropBbox``) or expansion (``expandBbox``),
    dropping boxes whose centre falls outside when ``need_meet_center_constraint``."""

    def __init__(self, need_meet_center_constraint: bool = True):
        self.center = need_meet_center_constraint

    def transform_mat(self, f):
        lab = _label(f)
        if lab is None:
            return
        box = f.get(ImageFeature.cropBbox) or f.get(ImageFeature.expandBbox)
        if box is None:
            return
        x1, y1, x2, y2 = box
        bw, bh = x2 - x1, y2 - y1
        b = lab.bboxes
        keep = torch.ones(b.shape[0], dtype=torch.bool)
        if self.center:
            cx = (b[:, 0] + b[:, 2]) / 2
            cy = (b[:, 1] + b[:, 3]) / 2
            keep = (cx >= x1) & (cx <= x2) & (cy >= y1) & (cy <= y2)
        nb = torch.stack([(b[:, 0] - x1) / bw, (b[:, 1] - y1) / bh, (b[:, 2] - x1) / bw, (b[:, 3] - y1) / bh], 1)
        nb = nb.clamp(0, 1)
        keep &= (nb[:, 2] > nb[:, 0]) & (nb[:, 3] > nb[:, 1])
        lab.bboxes = nb[keep]
        lab.classes = lab.classes[..., keep]


class BboxUtil:
    """Box helpers (``BboxUtil.scala``): IoU, encode/decode against priors, clipping, scaling."""

    @staticmethod
    def area(b: torch.Tensor) -> torch.Tensor:
        return (b[..., 2] - b[..., 0]).clamp_min(0) * (b[..., 3] - b[..., 1]).clamp_min(0)

    @staticmethod
    def iou(a: torch.Tensor, b: torch.Tensor, plus_one: float = 0.0) -> torch.Tensor:
        """Pairwise IoU of ``a [N, 4]`` and ``b [M, 4]`` → ``[N, M]``."""
        lt = torch.max(a[:, None, :2], b[None, :, :2])
        rb = torch.min(a[:, None, 2:], b[None, :, 2:])
        wh = (rb - lt + plus_one).clamp_min(0)
        inter = wh[..., 0] * wh[..., 1]
        aa = ((a[:, 2] - a[:, 0] + plus_one) * (a[:, 3] - a[:, 1] + plus_one))[:, None]
        ab = ((b[:, 2] - b[:, 0] + plus_one) * (b[:, 3] - b[:, 1] + plus_one))[None, :]
        return inter / (aa + ab - inter).clamp_min(1e-12)

    jaccard_overlap = iou

    @staticmethod
    def clip_boxes(b: torch.Tensor, h: float, w: float) -> torch.Tensor:
        out = b.clone()
        out[..., 0::2] = out[..., 0::2].clamp(0, w - 1)
        out[..., 1::2] = out[..., 1::2].clamp(0, h - 1)
        return out

    @staticmethod
    def encode(boxes: torch.Tensor, priors: torch.Tensor, variances=(0.1, 0.1, 0.2, 0.2)) -> torch.Tensor:
        """SSD center-size encoding of ``boxes`` w.r.t. ``priors`` (both x1y1x2y2)."""
        pw, ph = priors[:, 2] - priors[:, 0], priors[:, 3] - priors[:, 1]
        pcx, pcy = (priors[:, 0] + priors[:, 2]) / 2, (priors[:, 1] + priors[:, 3]) / 2
        bw, bh = boxes[:, 2] - boxes[:, 0], boxes[:, 3] - boxes[:, 1]
        bcx, bcy = (boxes[:, 0] + boxes[:, 2]) / 2, (boxes[:, 1] + boxes[:, 3]) / 2
        return torch.stack([(bcx - pcx) / pw / variances[0], (bcy - pcy) / ph / variances[1],
                            torch.log(bw / pw) / variances[2], torch.log(bh / ph) / variances[3]], 1)

    @staticmethod
    def decode(loc: torch.Tensor, priors: torch.Tensor, variances=(0.1, 0.1, 0.2, 0.2)) -> torch.Tensor:
        pw, ph = priors[:, 2] - priors[:, 0], priors[:, 3] - priors[:, 1]
        pcx, pcy = (priors[:, 0] + priors[:, 2]) / 2, (priors[:, 1] + priors[:, 3]) / 2
        cx = loc[:, 0] * variances[0] * pw + pcx
        cy = loc[:, 1] * variances[1] * ph + pcy
        w = torch.exp(loc[:, 2] * variances[2]) * pw
        h = torch.exp(loc[:, 3] * variances[3]) * ph
        return torch.stack([cx - w / 2, cy - h / 2, cx + w / 2, cy + h / 2], 1)

    @staticmethod
    def bbox_transform_inv(boxes: torch.Tensor, deltas: torch.Tensor, weights=(1.0, 1.0, 1.0, 1.0)) -> torch.Tensor:
        """Faster-RCNN delta decoding (``+1`` pixel widths)."""
        w = boxes[:, 2] - boxes[:, 0] + 1
        h = boxes[:, 3] - boxes[:, 1] + 1
        cx = boxes[:, 0] + 0.5 * w
        cy = boxes[:, 1] + 0.5 * h
        dx, dy = deltas[:, 0::4] / weights[0], deltas[:, 1::4] / weights[1]
        dw, dh = deltas[:, 2::4] / weights[2], deltas[:, 3::4] / weights[3]
        pcx = dx * w[:, None] + cx[:, None]
        pcy = dy * h[:, None] + cy[:, None]
        pw = torch.exp(dw) * w[:, None]
        ph = torch.exp(dh) * h[:, None]
        out = torch.zeros_like(deltas)
        out[:, 0::4] = pcx - 0.5 * pw
        out[:, 1::4] = pcy - 0.5 * ph
        out[:, 2::4] = pcx + 0.5 * pw - 1
        out[:, 3::4] = pcy + 0.5 * ph - 1
        return out
