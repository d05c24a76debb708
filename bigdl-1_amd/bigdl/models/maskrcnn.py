"""Mask R-CNN (``models/maskrcnn/MaskRCNN.scala``, ``models/maskrcnn/Utils.scala``): ResNet-50 C2–C5
backbone → FPN (P2–P6) → RegionProposal → BoxHead → MaskHead, inference-only as in the reference.

Input Table(images [B, 3, H, W], image_info [B, 4] = (height, width, original_height,
original_width)).  Training mode returns Table(boxes, labels, Table(mask_features, masks), scores);
eval mode returns per-image Tables keyed like ``RoiLabel`` (``masks`` as COCO RLE, ``bboxes`` scaled
back to the original size, ``classes``, ``scores``).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List

import torch
import torch.nn.functional as F

from ..nn import (Sequential, ConcatTable, CAddTable, Identity, ReLU, SpatialMaxPooling, FPN, RegionProposal,
                  BoxHead, MaskHead)
from ..nn.layers.detection import _Composite
from ..utils.table import Table
from .resnet import Convolution, Sbn


@dataclass
class MaskRCNNParams:
    anchorSizes: List[float] = field(default_factory=lambda: [32, 64, 128, 256, 512])
    aspectRatios: List[float] = field(default_factory=lambda: [0.5, 1.0, 2.0])
    anchorStride: List[float] = field(default_factory=lambda: [4, 8, 16, 32, 64])
    preNmsTopNTest: int = 1000
    postNmsTopNTest: int = 1000
    preNmsTopNTrain: int = 2000
    postNmsTopNTrain: int = 2000
    rpnNmsThread: float = 0.7
    minSize: int = 0
    boxResolution: int = 7
    maskResolution: int = 14
    scales: List[float] = field(default_factory=lambda: [0.25, 0.125, 0.0625, 0.03125])
    samplingRatio: int = 2
    boxScoreThresh: float = 0.05
    boxNmsThread: float = 0.5
    maxPerImage: int = 100
    outputSize: int = 1024
    layers: List[int] = field(default_factory=lambda: [256, 256, 256, 256])
    dilation: int = 1
    useGn: bool = False


def _bottleneck(n_in, internal, n_out, stride, use_conv):
    s = (Sequential().add(Convolution(n_in, internal, 1, 1, stride, stride)).add(Sbn(internal)).add(ReLU(True))
         .add(Convolution(internal, internal, 3, 3, 1, 1, 1, 1)).add(Sbn(internal)).add(ReLU(True))
         .add(Convolution(internal, n_out, 1, 1)).add(Sbn(n_out)))
    short = (Sequential().add(Convolution(n_in, n_out, 1, 1, stride, stride)).add(Sbn(n_out))
             if use_conv else Identity())
    return Sequential().add(ConcatTable().add(s).add(short)).add(CAddTable(True)).add(ReLU(True))


def _stage(count, n_in, internal, n_out, stride):
    s = Sequential().add(_bottleneck(n_in, internal, n_out, stride, True))
    for _ in range(count - 1):
        s.add(_bottleneck(n_out, internal, n_out, 1, False))
    return s


class _ResNet50C2C5(_Composite):
    """ResNet-50 trunk returning Table(C2, C3, C4, C5) (``MaskRCNN.scala:81``)."""

    def __init__(self, in_channels):
        super().__init__()
        self.stem = (Sequential().add(Convolution(3, 64, 7, 7, 2, 2, 3, 3, propagate_back=False)).add(Sbn(64))
                     .add(ReLU(True)).add(SpatialMaxPooling(3, 3, 2, 2, 1, 1)))
        self.stages = [_stage(3, 64, 64, in_channels, 1), _stage(4, in_channels, 128, in_channels * 2, 2),
                       _stage(6, in_channels * 2, 256, in_channels * 4, 2),
                       _stage(3, in_channels * 4, 512, in_channels * 8, 2)]
        self.modules = [self.stem] + self.stages

    def updateOutput(self, input):
        x = self.stem.forward(input)
        outs = []
        for st in self.stages:
            x = st.forward(x)
            outs.append(x)
        return Table(*outs)


def _paste_mask(mask: torch.Tensor, box: torch.Tensor, h: int, w: int, thresh: float = 0.5,
                padding: int = 1) -> torch.Tensor:
    """Paste one M×M probability mask into an h×w image inside ``box`` (``Utils.scala:101``): pad the
    mask by ``padding``, expand the box by the same ratio, bilinearly resize into the integer box and
    threshold."""
    M = mask.shape[-1]
    scale = (M + 2 * padding) / M
    pm = F.pad(mask.view(1, 1, M, M).float(), (padding,) * 4)
    x1, y1, x2, y2 = [float(v) for v in box]
    cx, cy, hw, hh = (x1 + x2) / 2, (y1 + y2) / 2, (x2 - x1) / 2 * scale, (y2 - y1) / 2 * scale
    bx1, by1, bx2, by2 = int(cx - hw), int(cy - hh), int(cx + hw), int(cy + hh)
    bw, bh = max(bx2 - bx1 + 1, 1), max(by2 - by1 + 1, 1)
    res = F.interpolate(pm, size=(bh, bw), mode="bilinear", align_corners=False)[0, 0] > thresh
    out = torch.zeros(h, w, dtype=torch.bool, device=mask.device)
    xa, xb = max(bx1, 0), min(bx2 + 1, w)
    ya, yb = max(by1, 0), min(by2 + 1, h)
    if xb > xa and yb > ya:
        out[ya:yb, xa:xb] = res[ya - by1:yb - by1, xa - bx1:xb - bx1]
    return out


class MaskRCNN(_Composite):
    def __init__(self, in_channels: int = 256, out_channels: int = 256, num_classes: int = 81,
                 config: MaskRCNNParams = None):
        super().__init__()
        c = config or MaskRCNNParams()
        self.config, self.inChannels, self.outChannels, self.numClasses = c, in_channels, out_channels, num_classes
        self.resnet = _ResNet50C2C5(in_channels)
        self.fpn = FPN([in_channels, in_channels * 2, in_channels * 4, in_channels * 8], out_channels, top_blocks=1)
        self.rpn = RegionProposal(out_channels, c.anchorSizes, c.aspectRatios, c.anchorStride, c.preNmsTopNTest,
                                  c.postNmsTopNTest, c.preNmsTopNTrain, c.postNmsTopNTrain, c.rpnNmsThread, c.minSize)
        self.boxHead = BoxHead(out_channels, c.boxResolution, c.scales, c.samplingRatio, c.boxScoreThresh,
                               c.boxNmsThread, c.maxPerImage, c.outputSize, num_classes)
        self.maskHead = MaskHead(out_channels, c.maskResolution, c.scales, c.samplingRatio, c.layers, c.dilation,
                                 num_classes, c.useGn)
        self.modules = [self.resnet, self.fpn, self.rpn, self.boxHead, self.maskHead]

    def updateOutput(self, input):
        images, info = input[1], input[2]
        size = torch.tensor([float(images.shape[2]), float(images.shape[3])])
        feats = self.fpn.forward(self.resnet.forward(images))
        proposals = self.rpn.forward(Table(feats, size))
        was_train = self.boxHead.train
        self.boxHead.evaluate()  # box post-processing always runs (MaskRCNN.scala:162)
        post = self.boxHead.forward(Table(feats, proposals, size))[2]
        self.boxHead.training(was_train)
        labels, boxes, scores = post[1], post[2], post[3]
        masks = self.maskHead.forward(Table(feats, boxes, labels))
        if self.train:
            return Table(boxes, labels, masks, scores)
        return self._post(boxes, labels, masks[2], scores, info)

    def _post(self, boxes, labels, masks, scores, info):
        from ..dataset.segmentation import MaskUtils
        out, start = Table(), 0
        info = info.view(-1, 4)
        for i in range(len(boxes)):
            h, w, oh, ow = [int(v) for v in info[i].tolist()]
            b = boxes[i + 1].clone()
            n = b.shape[0]
            if (h, w) != (oh, ow):
                b[:, 0::2] *= ow / w
                b[:, 1::2] *= oh / h
            rles = [MaskUtils.binary_to_rle(_paste_mask(masks[start + j, 0], b[j], oh, ow).cpu()) for j in range(n)]
            t = Table()
            t["masks"], t["bboxes"] = rles, b
            t["classes"], t["scores"] = labels[start:start + n], scores[start:start + n]
            out.insert(t)
            start += n
        return out

    def updateGradInput(self, input, gradOutput):
        raise NotImplementedError("MaskRCNN model only supports inference (MaskRCNN.scala)")
