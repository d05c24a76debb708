"""Segmentation masks and the COCO dataset (``DL/dataset/segmentation/{MaskUtils,COCODataset}.scala``).

RLE masks are COCO's "uncompressed RLE": alternating run lengths of 0s and 1s over the
COLUMN-major flattened ``height × width`` mask, starting with a run of 0s.  ``rle2string`` /
``string2rle`` implement COCO's compact LEB128-like encoding (6 bits per char, ASCII 48-111, runs
after the second delta-coded), ``MaskApi.c``-compatible.  Polygons are rasterised with PIL's
scan-line fill (COCO upsamples edges ×5; pixel coverage differs only on boundary pixels).
"""
from __future__ import annotations

import json
import os
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch


class SegmentationMasks:
    def to_rle(self) -> "RLEMasks":
        raise NotImplementedError

    toRLE = to_rle


class RLEMasks(SegmentationMasks):
    def __init__(self, counts: Sequence[int], height: int, width: int):
        self.counts = [int(c) for c in counts]
        self.height, self.width = int(height), int(width)

    def to_rle(self):
        return self

    def get(self, i: int) -> int:
        return self.counts[i] & 0xFFFFFFFF

    def __eq__(self, o):
        return isinstance(o, RLEMasks) and self.counts == o.counts and self.height == o.height and \
            self.width == o.width

    def __hash__(self):
        return hash((tuple(self.counts), self.height, self.width))

    def __repr__(self):
        return f"RLEMasks({self.height}x{self.width}, {len(self.counts)} runs)"


class PolyMasks(SegmentationMasks):
    def __init__(self, poly: Sequence[Sequence[float]], height: int, width: int):
        self.poly = [list(map(float, p)) for p in poly]
        self.height, self.width = int(height), int(width)

    def to_rle(self):
        return MaskUtils.poly_to_single_rle(self, self.height, self.width)


class MaskUtils:
    @staticmethod
    def rle2string(rle: RLEMasks) -> str:
        s = []
        cnts = rle.counts
        for i in range(len(cnts)):
            x = int(cnts[i])
            if i > 2:
                x -= int(cnts[i - 2])
            more = True
            while more:
                c = x & 0x1F
                x >>= 5
                more = (x != -1) if (c & 0x10) else (x != 0)
                if more:
                    c |= 0x20
                s.append(chr(c + 48))
        return "".join(s)

    RLE2String = rle2string

    @staticmethod
    def string2rle(s: str, h: int, w: int) -> RLEMasks:
        cnts: List[int] = []
        p = 0
        while p < len(s):
            x = 0
            k = 0
            more = True
            while more:
                c = ord(s[p]) - 48
                x |= (c & 0x1F) << (5 * k)
                more = bool(c & 0x20)
                k += 1
                p += 1
                if not more and (c & 0x10):
                    x |= -1 << (5 * k)
            if len(cnts) > 2:
                x += cnts[-2]
            cnts.append(int(x))
        return RLEMasks(cnts, h, w)

    string2RLE = string2rle

    @staticmethod
    def binary_to_rle(mask) -> RLEMasks:
        m = torch.as_tensor(mask)
        h, w = m.shape
        flat = (m.t().reshape(-1) > 0).to(torch.int8).numpy()
        # run lengths from the change points (column-major, first run counts zeros)
        edges = np.flatnonzero(np.diff(flat)) + 1
        bounds = np.concatenate([[0], edges, [flat.size]])
        counts = np.diff(bounds).tolist()
        if flat.size and flat[0] == 1:
            counts = [0] + counts
        return RLEMasks(counts, h, w)

    binaryToRLE = binary_to_rle

    @staticmethod
    def rle_to_binary(rle: RLEMasks) -> torch.Tensor:
        flat = np.zeros(rle.height * rle.width, dtype=np.uint8)
        pos, val = 0, 0
        for c in rle.counts:
            if val:
                flat[pos:pos + c] = 1
            pos += c
            val ^= 1
        return torch.from_numpy(flat.reshape(rle.width, rle.height).T.copy())

    @staticmethod
    def poly2rle(poly: PolyMasks, height: int, width: int) -> List[RLEMasks]:
        from PIL import Image, ImageDraw
        out = []
        for xy in poly.poly:
            img = Image.new("L", (width, height), 0)
            pts = [(xy[i], xy[i + 1]) for i in range(0, len(xy) - 1, 2)]
            if len(pts) >= 2:
                ImageDraw.Draw(img).polygon(pts, outline=1, fill=1)
            out.append(MaskUtils.binary_to_rle(torch.from_numpy(np.array(img, dtype=np.uint8))))
        return out

    poly2RLE = poly2rle

    @staticmethod
    def merge_rles(rles: Sequence[RLEMasks], intersect: bool) -> RLEMasks:
        m = MaskUtils.rle_to_binary(rles[0]).bool()
        for r in rles[1:]:
            b = MaskUtils.rle_to_binary(r).bool()
            m = (m & b) if intersect else (m | b)
        return MaskUtils.binary_to_rle(m.to(torch.uint8))

    mergeRLEs = merge_rles

    @staticmethod
    def poly_to_single_rle(poly: PolyMasks, height: int, width: int) -> RLEMasks:
        return MaskUtils.merge_rles(MaskUtils.poly2rle(poly, height, width), False)

    polyToSingleRLE = poly_to_single_rle

    @staticmethod
    def rle_area(r: RLEMasks) -> int:
        return int(sum(r.counts[1::2]))

    rleArea = rle_area

    @staticmethod
    def rle_iou(det: RLEMasks, gt: RLEMasks, is_crowd: bool) -> float:
        a = MaskUtils.rle_to_binary(det).bool()
        b = MaskUtils.rle_to_binary(gt).bool()
        inter = int((a & b).sum())
        union = int(a.sum()) if is_crowd else int((a | b).sum())
        return inter / union if union > 0 else 0.0

    rleIOU = rle_iou

    @staticmethod
    def bbox_iou(gt: Tuple[float, float, float, float], dt: Tuple[float, float, float, float],
                 is_crowd: bool) -> float:
        gx1, gy1, gx2, gy2 = gt
        dx1, dy1, dx2, dy2 = dt
        iw = min(gx2, dx2) - max(gx1, dx1)
        ih = min(gy2, dy2) - max(gy1, dy1)
        if iw <= 0 or ih <= 0:
            return 0.0
        inter = iw * ih
        da = (dx2 - dx1) * (dy2 - dy1)
        union = da if is_crowd else da + (gx2 - gx1) * (gy2 - gy1) - inter
        return inter / union

    bboxIOU = bbox_iou

    @staticmethod
    def rle_to_one_bbox(r: RLEMasks) -> Tuple[float, float, float, float]:
        m = MaskUtils.rle_to_binary(r)
        ys, xs = torch.nonzero(m, as_tuple=True)
        if len(xs) == 0:
            return 0.0, 0.0, 0.0, 0.0
        return float(xs.min()), float(ys.min()), float(xs.max()) + 1, float(ys.max()) + 1

    rleToOneBbox = rle_to_one_bbox


class COCOCategory:
    def __init__(self, id, name, supercategory=""):
        self.id, self.name, self.supercategory = int(id), name, supercategory


class COCOImage:
    def __init__(self, id, height, width, file_name, img_root=""):
        self.id, self.height, self.width, self.file_name = int(id), int(height), int(width), file_name
        self.img_root = img_root
        self.annotations: List["COCOAnnotation"] = []

    @property
    def path(self):
        return os.path.join(self.img_root, self.file_name)

    def data(self) -> bytes:
        with open(self.path, "rb") as f:
            return f.read()


class COCOAnnotation:
    def __init__(self, id, image_id, category_id, bbox, area, is_crowd, segmentation):
        self.id, self.image_id, self.category_id = int(id), int(image_id), int(category_id)
        self.bbox = tuple(float(v) for v in bbox)  # x, y, w, h
        self.area, self.is_crowd, self.segmentation = float(area), bool(is_crowd), segmentation


class COCODataset:
    """``COCODataset.load(jsonPath, imgRoot)``: images, annotations and categories, with the
    1-based contiguous category index used as training labels."""

    def __init__(self, info, images, annotations, categories, img_root=""):
        self.info = info
        self.images = images
        self.annotations = annotations
        self.categories = sorted(categories, key=lambda c: c.id)
        self._img = {im.id: im for im in images}
        self._cat2idx = {c.id: i + 1 for i, c in enumerate(self.categories)}
        for a in annotations:
            if a.image_id in self._img:
                self._img[a.image_id].annotations.append(a)

    @staticmethod
    def load(json_path: str, img_root: str = "") -> "COCODataset":
        with open(json_path) as f:
            d = json.load(f)
        images = [COCOImage(i["id"], i["height"], i["width"], i["file_name"], img_root) for i in d.get("images", [])]
        hw = {im.id: (im.height, im.width) for im in images}
        anns = []
        for a in d.get("annotations", []):
            seg = a.get("segmentation")
            h, w = hw.get(a["image_id"], (0, 0))
            if isinstance(seg, list):
                seg = PolyMasks(seg, h, w)
            elif isinstance(seg, dict):
                cnt = seg["counts"]
                sh, sw = seg["size"]
                seg = MaskUtils.string2rle(cnt, sh, sw) if isinstance(cnt, str) else RLEMasks(cnt, sh, sw)
            anns.append(COCOAnnotation(a["id"], a["image_id"], a["category_id"], a["bbox"], a.get("area", 0),
                                       a.get("iscrowd", 0), seg))
        cats = [COCOCategory(c["id"], c["name"], c.get("supercategory", "")) for c in d.get("categories", [])]
        return COCODataset(d.get("info", {}), images, anns, cats, img_root)

    def get_image_by_id(self, id_):
        return self._img[int(id_)]

    getImageById = get_image_by_id

    def category_id2idx(self, id_) -> int:
        return self._cat2idx[int(id_)]

    categoryId2Idx = category_id2idx

    def get_category_by_idx(self, idx: int) -> COCOCategory:
        return self.categories[idx - 1]

    getCategoryByIdx = get_category_by_idx

    def to_image_features(self):
        """Each image → ImageFeature with bytes, uri and a RoiLabel (1-based class indices,
        x1y1x2y2 boxes, masks) — the input of a detection pipeline."""
        from ..transform.vision.image import ImageFeature, RoiLabel
        feats = []
        for im in self.images:
            anns = [a for a in im.annotations]
            classes = torch.tensor([float(self.category_id2idx(a.category_id)) for a in anns])
            boxes = torch.tensor([[a.bbox[0], a.bbox[1], a.bbox[0] + a.bbox[2], a.bbox[1] + a.bbox[3]]
                                  for a in anns]) if anns else torch.zeros(0, 4)
            f = ImageFeature(uri=im.path)
            f[ImageFeature.label] = RoiLabel(classes, boxes, [a.segmentation for a in anns])
            f[ImageFeature.originalSize] = (im.height, im.width, 3)
            feats.append(f)
        return feats
