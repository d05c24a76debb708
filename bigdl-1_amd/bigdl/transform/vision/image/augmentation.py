"""Image augmentations (``DL/transform/vision/image/augmentation/*.scala``), on ``[H, W, C]`` BGR
float tensors (host or device).  Randomness comes from the framework RNG (``RandomGenerator``)."""
from __future__ import annotations

import math
from typing import Optional, Sequence

import torch
import torch.nn.functional as F

from ....utils.random import RNG
from .image_feature import FeatureTransformer, ImageFeature

_INTERP = {"NEAREST": "nearest", "LINEAR": "bilinear", "CUBIC": "bicubic", "AREA": "area", 0: "nearest",
           1: "bilinear", 2: "bicubic", 3: "area"}


def resize_mat(m: torch.Tensor, h: int, w: int, mode="LINEAR") -> torch.Tensor:
    mode = _INTERP.get(mode, "bilinear")
    x = m.permute(2, 0, 1).unsqueeze(0)
    kw = {} if mode in ("nearest", "area") else {"align_corners": False}
    y = F.interpolate(x, size=(int(h), int(w)), mode=mode, **kw)
    if mode == "bicubic":
        y = y.clamp(float(m.min()), float(m.max()))
    return y.squeeze(0).permute(1, 2, 0).contiguous()


# ---------------------------------------------------------------------------------------------- colour
def bgr_to_hsv(m: torch.Tensor) -> torch.Tensor:
    """BGR in [0, 255] → H in [0, 360), S in [0, 1], V in [0, 255] (OpenCV float convention)."""
    b, g, r = m[..., 0], m[..., 1], m[..., 2]
    v, _ = m[..., :3].max(-1)
    mn, _ = m[..., :3].min(-1)
    d = v - mn
    s = torch.where(v > 0, d / v.clamp_min(1e-12), torch.zeros_like(v))
    dz = d.clamp_min(1e-12)
    h = torch.where(v == r, 60 * (g - b) / dz, torch.where(v == g, 120 + 60 * (b - r) / dz, 240 + 60 * (r - g) / dz))
    h = torch.where(d == 0, torch.zeros_like(h), h)
    h = torch.remainder(h, 360.0)
    return torch.stack([h, s, v], -1)


def hsv_to_bgr(hsv: torch.Tensor) -> torch.Tensor:
    h, s, v = hsv[..., 0], hsv[..., 1], hsv[..., 2]
    c = v * s
    hp = torch.remainder(h, 360.0) / 60.0
    x = c * (1 - torch.abs(torch.remainder(hp, 2) - 1))
    z = torch.zeros_like(h)
    i = hp.floor().long().clamp(0, 5)
    r = torch.stack([c, x, z, z, x, c], -1).gather(-1, i.unsqueeze(-1)).squeeze(-1)
    g = torch.stack([x, c, c, x, z, z], -1).gather(-1, i.unsqueeze(-1)).squeeze(-1)
    b = torch.stack([z, z, x, c, c, x], -1).gather(-1, i.unsqueeze(-1)).squeeze(-1)
    mm = v - c
    return torch.stack([b + mm, g + mm, r + mm], -1)


class Brightness(FeatureTransformer):
    """``mat += U(deltaLow, deltaHigh)``."""

    def __init__(self, delta_low: float, delta_high: float):
        self.delta_low, self.delta_high = delta_low, delta_high

    def transform_mat(self, f):
        d = RNG.uniform(self.delta_low, self.delta_high)
        f.set_mat(f.opencv_mat() + d)


class Contrast(FeatureTransformer):
    """``mat *= U(deltaLow, deltaHigh)``."""

    def __init__(self, delta_low: float, delta_high: float):
        self.delta_low, self.delta_high = delta_low, delta_high

    def transform_mat(self, f):
        a = RNG.uniform(self.delta_low, self.delta_high)
        if abs(a - 1) > 1e-3:
            f.set_mat(f.opencv_mat() * a)


class Saturation(FeatureTransformer):
    def __init__(self, delta_low: float, delta_high: float):
        self.delta_low, self.delta_high = delta_low, delta_high

    def transform_mat(self, f):
        a = RNG.uniform(self.delta_low, self.delta_high)
        if abs(a - 1) <= 1e-3:
            return
        m = f.opencv_mat()
        hsv = bgr_to_hsv(m)
        hsv[..., 1] = (hsv[..., 1] * a).clamp(0, 1)
        out = m.clone()
        out[..., :3] = hsv_to_bgr(hsv)
        f.set_mat(out)


class Hue(FeatureTransformer):
    def __init__(self, delta_low: float, delta_high: float):
        self.delta_low, self.delta_high = delta_low, delta_high

    def transform_mat(self, f):
        d = RNG.uniform(self.delta_low, self.delta_high)
        if abs(d) <= 1e-3:
            return
        m = f.opencv_mat()
        hsv = bgr_to_hsv(m)
        hsv[..., 0] = torch.remainder(hsv[..., 0] + d, 360.0)
        out = m.clone()
        out[..., :3] = hsv_to_bgr(hsv)
        f.set_mat(out)


class ChannelOrder(FeatureTransformer):
    """Random permutation of the channels."""

    def transform_mat(self, f):
        m = f.opencv_mat()
        perm = torch.as_tensor(RNG.permutation(m.shape[2]))
        f.set_mat(m[..., perm].contiguous())


class ColorJitter(FeatureTransformer):
    """``ColorJitter.scala``: brightness / contrast / saturation / hue, each with its probability,
    in the fixed order B, C(before), S, H, C(after) or a random order with ``random_order_prob``."""

    def __init__(self, brightness_prob=0.5, brightness_delta=32.0, contrast_prob=0.5, contrast_lower=0.5,
                 contrast_upper=1.5, hue_prob=0.5, hue_delta=18.0, saturation_prob=0.5, saturation_lower=0.5,
                 saturation_upper=1.5, random_order_prob=0.0, shuffle=False):
        self.bp, self.bd = brightness_prob, brightness_delta
        self.cp, self.cl, self.cu = contrast_prob, contrast_lower, contrast_upper
        self.hp, self.hd = hue_prob, hue_delta
        self.sp, self.sl, self.su = saturation_prob, saturation_lower, saturation_upper
        self.rop = random_order_prob
        self.shuffle = shuffle
        self.brightness = RandomTransformer(Brightness(-brightness_delta, brightness_delta), brightness_prob)
        self.contrast = RandomTransformer(Contrast(contrast_lower, contrast_upper), contrast_prob)
        self.saturation = RandomTransformer(Saturation(saturation_lower, saturation_upper), saturation_prob)
        self.hue = RandomTransformer(Hue(-hue_delta, hue_delta), hue_prob)

    def transform_mat(self, f):
        if RNG.uniform(0, 1) < self.rop:
            order = [self.brightness, self.contrast, self.saturation, self.hue]
            for i in RNG.permutation(4):
                order[i].transform(f)
        elif RNG.uniform(0, 1) > 0.5:
            for t in (self.brightness, self.contrast, self.saturation, self.hue):
                t.transform(f)
        else:
            for t in (self.brightness, self.saturation, self.hue, self.contrast):
                t.transform(f)


# ---------------------------------------------------------------------------------------------- normalise
class ChannelNormalize(FeatureTransformer):
    """``(x - mean_c) / std_c``; arguments in R, G, B order (the mat is BGR)."""

    def __init__(self, mean_r: float, mean_g: float = None, mean_b: float = None, std_r: float = 1.0,
                 std_g: float = 1.0, std_b: float = 1.0):
        if mean_g is None:  # ChannelNormalize(mean, std)
            mean_g = mean_b = mean_r
            std_g = std_b = std_r
        self.means = [mean_b, mean_g, mean_r]
        self.stds = [std_b, std_g, std_r]

    def transform_mat(self, f):
        m = f.opencv_mat()
        mean = torch.tensor(self.means[:m.shape[2]], dtype=m.dtype, device=m.device)
        std = torch.tensor(self.stds[:m.shape[2]], dtype=m.dtype, device=m.device)
        f.set_mat((m - mean) / std)


class ChannelScaledNormalizer(FeatureTransformer):
    """``(x - mean_c) * scale``."""

    def __init__(self, mean_r: int, mean_g: int, mean_b: int, scale: float):
        self.means = [mean_b, mean_g, mean_r]
        self.scale = scale

    def transform_mat(self, f):
        m = f.opencv_mat()
        mean = torch.tensor(self.means, dtype=m.dtype, device=m.device)
        f.set_mat((m - mean) * self.scale)


class PixelNormalizer(FeatureTransformer):
    """Subtract a per-pixel mean image (``means`` flattened in HWC order)."""

    def __init__(self, means: Sequence[float]):
        self.means = torch.as_tensor(means, dtype=torch.float32)

    def transform_mat(self, f):
        m = f.opencv_mat()
        f.set_mat(m - self.means.to(m.device).reshape(m.shape))


# ---------------------------------------------------------------------------------------------- geometry
class HFlip(FeatureTransformer):
    def transform_mat(self, f):
        f.set_mat(f.opencv_mat().flip(1))


class Resize(FeatureTransformer):
    def __init__(self, resize_h: int, resize_w: int, resize_mode="LINEAR", use_scale_factor: bool = True):
        self.h, self.w, self.mode = resize_h, resize_w, resize_mode

    def transform_mat(self, f):
        f.set_mat(resize_mat(f.opencv_mat(), self.h, self.w, self.mode))


class AspectScale(FeatureTransformer):
    """Scale the shorter side to ``min_size`` (longer side ≤ ``max_size``), sizes rounded to
    ``scale_multiple_of`` (``Resize.scala`` AspectScale)."""

    def __init__(self, min_size: int, scale_multiple_of: int = 1, max_size: int = 1000, resize_mode="LINEAR",
                 use_scale_factor: bool = True, min_scale: Optional[float] = None):
        self.min_size, self.mult, self.max_size, self.mode = min_size, scale_multiple_of, max_size, resize_mode
        self.min_scale = min_scale

    @staticmethod
    def get_size(h, w, min_size, mult, max_size, min_scale=None):
        short, long_ = min(h, w), max(h, w)
        scale = min_size / short
        if scale * long_ > max_size:
            scale = max_size / long_
        if min_scale is not None:
            scale = max(scale, min_scale)
        nh, nw = h * scale, w * scale
        if mult > 1:
            nh = int(math.floor(nh / mult) * mult)
            nw = int(math.floor(nw / mult) * mult)
        return int(round(nh)), int(round(nw)), scale

    def transform_mat(self, f):
        m = f.opencv_mat()
        nh, nw, _ = self.get_size(m.shape[0], m.shape[1], self.min_size, self.mult, self.max_size, self.min_scale)
        f.set_mat(resize_mat(m, nh, nw, self.mode))


class RandomAspectScale(AspectScale):
    def __init__(self, scales: Sequence[int], scale_multiple_of: int = 1, max_size: int = 1000):
        super().__init__(scales[0], scale_multiple_of, max_size)
        self.scales = list(scales)

    def transform_mat(self, f):
        self.min_size = self.scales[int(RNG.uniform(0, len(self.scales))) % len(self.scales)]
        super().transform_mat(f)


class RandomResize(FeatureTransformer):
    """Resize to a random square size in [min_size, max_size]."""

    def __init__(self, min_size: int, max_size: int):
        self.min_size, self.max_size = min_size, max_size

    def transform_mat(self, f):
        s = int(RNG.uniform(self.min_size, self.max_size + 1))
        f.set_mat(resize_mat(f.opencv_mat(), s, s))


class ScaleResize(FeatureTransformer):
    """Shorter side → ``min_size`` keeping aspect, longer side ≤ ``max_size``; optionally scales
    the RoiLabel boxes too."""

    def __init__(self, min_size: int, max_size: int = -1, resize_roi: bool = False):
        self.min_size, self.max_size, self.resize_roi = min_size, max_size, resize_roi

    def transform_mat(self, f):
        m = f.opencv_mat()
        h, w = m.shape[0], m.shape[1]
        scale = self.min_size / min(h, w)
        if self.max_size > 0 and round(scale * max(h, w)) > self.max_size:
            scale = self.max_size / max(h, w)
        nh, nw = int(round(h * scale)), int(round(w * scale))
        f.set_mat(resize_mat(m, nh, nw))
        if self.resize_roi and ImageFeature.label in f and hasattr(f[ImageFeature.label], "bboxes"):
            lab = f[ImageFeature.label]
            lab.bboxes = lab.bboxes * torch.tensor([nw / w, nh / h, nw / w, nh / h])


class Crop(FeatureTransformer):
    """Base crop: ``(x1, y1, x2, y2)`` box, normalised or absolute, clipped to the image; stores
    the crop box under ``cropBbox`` (normalised) for ROI transforms."""

    def __init__(self, normalized: bool = True, is_clip: bool = True):
        self.normalized, self.is_clip = normalized, is_clip

    def box(self, f):  # pragma: no cover - abstract
        raise NotImplementedError

    @staticmethod
    def crop(f: ImageFeature, x1, y1, x2, y2, normalized: bool, is_clip: bool):
        m = f.opencv_mat()
        h, w = m.shape[0], m.shape[1]
        if normalized:
            x1, x2 = x1 * w, x2 * w
            y1, y2 = y1 * h, y2 * h
        if is_clip:
            x1, x2 = max(0.0, min(x1, w)), max(0.0, min(x2, w))
            y1, y2 = max(0.0, min(y1, h)), max(0.0, min(y2, h))
        xi1, yi1 = int(x1), int(y1)
        cw, ch = max(1, int(x2 - x1)), max(1, int(y2 - y1))
        f.set_mat(m[yi1:yi1 + ch, xi1:xi1 + cw].contiguous())
        f[ImageFeature.cropBbox] = (xi1 / w, yi1 / h, (xi1 + cw) / w, (yi1 + ch) / h)

    def transform_mat(self, f):
        x1, y1, x2, y2 = self.box(f)
        Crop.crop(f, x1, y1, x2, y2, self.normalized, self.is_clip)


class CenterCrop(Crop):
    def __init__(self, crop_width: int, crop_height: int, is_clip: bool = True):
        super().__init__(False, is_clip)
        self.cw, self.ch = crop_width, crop_height

    def box(self, f):
        h, w = f.get_height(), f.get_width()
        x1 = (w - self.cw) / 2.0
        y1 = (h - self.ch) / 2.0
        return x1, y1, x1 + self.cw, y1 + self.ch


class RandomCrop(Crop):
    def __init__(self, crop_width: int, crop_height: int, is_clip: bool = True):
        super().__init__(False, is_clip)
        self.cw, self.ch = crop_width, crop_height

    def box(self, f):
        h, w = f.get_height(), f.get_width()
        x1 = math.floor(RNG.uniform(0, max(w - self.cw, 0) + 1e-9))
        y1 = math.floor(RNG.uniform(0, max(h - self.ch, 0) + 1e-9))
        x1 = min(x1, max(w - self.cw, 0))
        y1 = min(y1, max(h - self.ch, 0))
        return x1, y1, x1 + self.cw, y1 + self.ch


class FixedCrop(Crop):
    def __init__(self, x1, y1, x2, y2, normalized: bool, is_clip: bool = True):
        super().__init__(normalized, is_clip)
        self.b = (x1, y1, x2, y2)

    def box(self, f):
        return self.b


class DetectionCrop(Crop):
    """Crop to the box stored in the feature under ``roi_key``."""

    def __init__(self, roi_key: str, normalized: bool = True):
        super().__init__(normalized, True)
        self.roi_key = roi_key

    def box(self, f):
        b = f[self.roi_key]
        b = b.reshape(-1).tolist() if isinstance(b, torch.Tensor) else list(b)
        return b[0], b[1], b[2], b[3]


class RandomCropper(FeatureTransformer):
    """Crop ``crop_width × crop_height`` (random or center) with optional random mirror
    (``RandomCropper.scala``)."""

    def __init__(self, crop_width: int, crop_height: int, mirror: bool, cropper_method: str = "Random",
                 channels: int = 3):
        self.cw, self.ch, self.mirror, self.method, self.channels = crop_width, crop_height, mirror, \
            cropper_method, channels

    def transform_mat(self, f):
        m = f.opencv_mat()
        h, w = m.shape[0], m.shape[1]
        if self.method.lower().startswith("random"):
            y = int(RNG.uniform(0, h - self.ch + 1)) if h > self.ch else 0
            x = int(RNG.uniform(0, w - self.cw + 1)) if w > self.cw else 0
        else:
            y, x = (h - self.ch) // 2, (w - self.cw) // 2
        out = m[y:y + self.ch, x:x + self.cw]
        if self.mirror and RNG.uniform(0, 1) < 0.5:
            out = out.flip(1)
        f.set_mat(out[..., :self.channels].contiguous())


class RandomAlterAspect(FeatureTransformer):
    """Inception-style random-area, random-aspect crop resized to ``crop_length``
    (``RandomAlterAspect.scala``; 10 attempts, then a shorter-side resize fallback)."""

    def __init__(self, min_area_ratio=0.08, max_area_ratio=1, min_aspect_ratio_change=0.75, interp_mode="CUBIC",
                 crop_length=224):
        self.min_area, self.max_area = min_area_ratio, max_area_ratio
        self.min_ar = min_aspect_ratio_change
        self.mode, self.L = interp_mode, crop_length

    @staticmethod
    def _rand_ratio(lo, hi):
        return (RNG.uniform(1e-2, (hi - lo) * 1000 + 1) + lo * 1000) / 1000

    def transform_mat(self, f):
        m = f.opencv_mat()
        h, w = m.shape[0], m.shape[1]
        for _ in range(10):
            ar = self._rand_ratio(self.min_area, self.max_area)
            asp = self._rand_ratio(self.min_ar, 1 / self.min_ar)
            na = ar * h * w
            nh, nw = int(math.sqrt(na) * asp), int(math.sqrt(na) / asp)
            if self._rand_ratio(0, 1) < 0.5:
                nh, nw = nw, nh
            if 0 < nh <= h and 0 < nw <= w:
                y = int(RNG.uniform(1e-2, h - nh + 1))
                x = int(RNG.uniform(1e-2, w - nw + 1))
                f.set_mat(resize_mat(m[y:y + nh, x:x + nw], self.L, self.L, self.mode))
                return
        f.set_mat(resize_mat(m, self.L, self.L, self.mode))


class Expand(FeatureTransformer):
    """Place the image on a larger mean-filled canvas (ratio U(min, max)) at a random offset; the
    expansion box (normalised to the new canvas) is stored under ``expandBbox``."""

    def __init__(self, means_r=123, means_g=117, means_b=104, min_expand_ratio=1.0, max_expand_ratio=4.0):
        self.means = [means_b, means_g, means_r]
        self.lo, self.hi = min_expand_ratio, max_expand_ratio

    def transform_mat(self, f):
        ratio = RNG.uniform(self.lo, self.hi)
        if abs(ratio - 1) < 1e-2:
            return
        m = f.opencv_mat()
        h, w, c = m.shape
        eh, ew = int(h * ratio), int(w * ratio)
        y = int(math.floor(RNG.uniform(0, eh - h)))
        x = int(math.floor(RNG.uniform(0, ew - w)))
        canvas = torch.empty((eh, ew, c), dtype=m.dtype, device=m.device)
        canvas[:] = torch.tensor(self.means[:c], dtype=m.dtype, device=m.device)
        canvas[y:y + h, x:x + w] = m
        f.set_mat(canvas)
        f[ImageFeature.expandBbox] = (-x / w, -y / h, (ew - x) / w, (eh - y) / h)


class FixExpand(FeatureTransformer):
    """Zero-pad the image to exactly ``expand_height × expand_width`` (top-left aligned)."""

    def __init__(self, expand_height: int, expand_width: int):
        self.eh, self.ew = expand_height, expand_width

    def transform_mat(self, f):
        m = f.opencv_mat()
        h, w, c = m.shape
        canvas = torch.zeros((max(self.eh, h), max(self.ew, w), c), dtype=m.dtype, device=m.device)
        canvas[:h, :w] = m
        f.set_mat(canvas)


class Filler(FeatureTransformer):
    """Fill the normalised box ``[startX, endX] × [startY, endY]`` with ``value``."""

    def __init__(self, start_x, start_y, end_x, end_y, value=255):
        self.b = (start_x, start_y, end_x, end_y)
        self.value = value

    def transform_mat(self, f):
        m = f.opencv_mat().clone()
        h, w = m.shape[0], m.shape[1]
        x1, y1 = int(self.b[0] * w), int(self.b[1] * h)
        x2, y2 = int(math.ceil(self.b[2] * w)), int(math.ceil(self.b[3] * h))
        m[y1:y2, x1:x2] = float(self.value)
        f.set_mat(m)


class RandomTransformer(FeatureTransformer):
    """Apply ``transformer`` with probability ``max_prob``."""

    def __init__(self, transformer: FeatureTransformer, max_prob: float):
        self.t, self.p = transformer, max_prob

    def transform(self, f):
        if RNG.uniform(0, 1) < self.p:
            return self.t.transform(f)
        return f


# ---------------------------------------------------------------------------------------------- SSD sampling
def _jaccard(a, b) -> float:
    ix1, iy1, ix2, iy2 = max(a[0], b[0]), max(a[1], b[1]), min(a[2], b[2]), min(a[3], b[3])
    if ix2 <= ix1 or iy2 <= iy1:
        return 0.0
    inter = (ix2 - ix1) * (iy2 - iy1)
    ua = (a[2] - a[0]) * (a[3] - a[1]) + (b[2] - b[0]) * (b[3] - b[1]) - inter
    return inter / ua if ua > 0 else 0.0


class BatchSampler:
    """One SSD crop sampler (``label/roi/BatchSampler.scala``): up to ``max_sample`` boxes in
    ``max_trials`` draws of scale ∈ [min_scale, max_scale] and aspect ratio ∈ [min, max] (clamped to
    [scale², 1/scale²]) inside the unit box; a box is kept when some ground-truth box overlaps it
    with Jaccard ∈ [min_overlap, max_overlap] (or always, without constraints)."""

    def __init__(self, max_sample=1, max_trials=50, min_scale=1.0, max_scale=1.0, min_aspect_ratio=1.0,
                 max_aspect_ratio=1.0, min_overlap=None, max_overlap=None):
        if not (0 < min_scale <= max_scale <= 1):
            raise ValueError("scales must satisfy 0 < minScale <= maxScale <= 1")
        if not (0 < min_aspect_ratio <= 1 <= max_aspect_ratio):
            raise ValueError("aspect ratios must satisfy 0 < min <= 1 <= max")
        self.max_sample, self.max_trials = max_sample, max_trials
        self.min_scale, self.max_scale = min_scale, max_scale
        self.min_ar, self.max_ar = min_aspect_ratio, max_aspect_ratio
        self.min_overlap, self.max_overlap = min_overlap, max_overlap

    def _sample_box(self):

        scale = RNG.uniform(self.min_scale, self.max_scale)
        ratio = RNG.uniform(self.min_ar, self.max_ar)
        ratio = min(max(ratio, scale * scale), 1.0 / scale / scale)
        w, h = scale * ratio ** 0.5, scale / ratio ** 0.5
        x1, y1 = RNG.uniform(0, 1 - w), RNG.uniform(0, 1 - h)
        return (x1, y1, x1 + w, y1 + h)

    def _ok(self, box, gt) -> bool:
        if self.min_overlap is None and self.max_overlap is None:
            return True
        for g in gt:
            o = _jaccard(box, g)
            if (self.min_overlap is None or o >= self.min_overlap) and (self.max_overlap is None or o <= self.max_overlap):
                return True
        return False

    def sample(self, gt, out: list):
        found = 0
        for _ in range(self.max_trials):
            if found >= self.max_sample:
                return
            b = self._sample_box()
            if self._ok(b, gt):
                found += 1
                out.append(b)

    @staticmethod
    def generate_batch_samples(gt, samplers) -> list:
        boxes = []
        for s in samplers:
            s.sample(gt, boxes)
        return boxes


class RandomSampler(Crop):
    """SSD training crop (``label/roi/RandomSampler.scala``): the seven default batch samplers
    (whole image; scale ≥ 0.3, aspect ∈ [1/2, 2] with min Jaccard 0.1/0.3/0.5/0.7/0.9 to a
    ground-truth box; max Jaccard 1.0), one of the sampled boxes picked uniformly, the image cropped
    to it; follow with ``RoiProject`` to move the labels (``RandomSampler()`` in pyspark returns the
    pair)."""

    def __init__(self):
        super().__init__(normalized=True, is_clip=True)
        self.samplers = [BatchSampler(max_trials=1)] + [
            BatchSampler(min_scale=0.3, min_aspect_ratio=0.5, max_aspect_ratio=2, min_overlap=o)
            for o in (0.1, 0.3, 0.5, 0.7, 0.9)] + [
            BatchSampler(min_scale=0.3, min_aspect_ratio=0.5, max_aspect_ratio=2, max_overlap=1.0)]

    def box(self, f):

        lab = f.get(ImageFeature.label)
        gt = lab.bboxes.tolist() if hasattr(lab, "bboxes") else []
        boxes = BatchSampler.generate_batch_samples(gt, self.samplers)
        if not boxes:
            return (0.0, 0.0, 1.0, 1.0)
        return boxes[min(len(boxes) - 1, int(RNG.uniform(0, 1) * len(boxes)))]


class PixelNormalize(PixelNormalizer):
    """pyspark name of :class:`PixelNormalizer` (``data(i) - mean(i)``, means in H·W·C order)."""
