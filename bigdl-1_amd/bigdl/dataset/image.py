"""Legacy labeled-image pipeline (``DL/dataset/image/*.scala``): LabeledBGRImage / LabeledGreyImage,
BytesToBGRImg, BytesToGreyImg, BGRImgCropper / BGRImgRdmCropper / GreyImgCropper,
BGRImgNormalizer / GreyImgNormalizer / BGRImgPixelNormalizer, HFlip, ColorJitter, Lighting,
BGRImgToBatch / GreyImgToBatch / MTLabeledBGRImgToBatch, BGRImgToSample / GreyImgToSample,
LocalImageFiles.  Images are ``[H, W, C]`` float tensors (content already divided by
``normalize``, default 255)."""
from __future__ import annotations

import os
from concurrent.futures import ThreadPoolExecutor
from typing import Iterator, List, Optional, Tuple

import numpy as np
import torch

from ..utils.random import RNG
from .core import MiniBatch, Sample, Transformer


class ByteRecord:
    def __init__(self, data: bytes, label: float):
        self.data, self.label = data, label


class LabeledBGRImage:
    def __init__(self, content: torch.Tensor = None, label: float = 0.0):
        self.content = content if content is not None else torch.zeros(0, 0, 3)
        self._label = float(label)

    def width(self):
        return self.content.shape[1]

    def height(self):
        return self.content.shape[0]

    def label(self):
        return self._label

    def setLabel(self, l):
        self._label = float(l)
        return self

    def hflip(self):
        self.content = self.content.flip(1).contiguous()
        return self

    def clone(self):
        return type(self)(self.content.clone(), self._label)

    def to_chw(self, to_rgb=True):
        c = self.content
        if to_rgb and c.shape[2] == 3:
            c = c.flip(2)
        return c.permute(2, 0, 1).contiguous()


class LabeledGreyImage(LabeledBGRImage):
    def __init__(self, content: torch.Tensor = None, label: float = 0.0):
        super().__init__(content if content is not None else torch.zeros(0, 0, 1), label)


class BytesToBGRImg(Transformer):
    """Decode (JPEG/PNG or raw ``int32 w, int32 h, BGR bytes`` records) and scale by 1/normalize."""

    def __init__(self, normalize: float = 255.0, resize_w: int = -1, resize_h: int = -1):
        self.normalize, self.rw, self.rh = normalize, resize_w, resize_h

    def _decode(self, b: bytes) -> torch.Tensor:
        if len(b) > 8:
            w = int.from_bytes(b[0:4], "big")
            h = int.from_bytes(b[4:8], "big")
            if w > 0 and h > 0 and 8 + w * h * 3 == len(b):
                a = np.frombuffer(b, dtype=np.uint8, offset=8).reshape(h, w, 3)
                return torch.from_numpy(a.copy()).float()
        from ..transform.vision.image.convertor import decode_bytes
        t = decode_bytes(b).float()
        if t.shape[2] == 1:
            t = t.expand(-1, -1, 3).contiguous()
        return t

    def apply(self, it):
        from ..transform.vision.image.augmentation import resize_mat
        for rec in it:
            m = self._decode(rec.data)
            if self.rw > 0 and self.rh > 0:
                m = resize_mat(m, self.rh, self.rw)
            yield LabeledBGRImage(m / self.normalize, rec.label)


class BytesToGreyImg(Transformer):
    """MNIST-style records: ``row × col`` uint8 pixels scaled to [0, 1]."""

    def __init__(self, row: int, col: int):
        self.row, self.col = row, col

    def apply(self, it):
        for rec in it:
            a = np.frombuffer(rec.data, dtype=np.uint8)[-self.row * self.col:].reshape(self.row, self.col, 1)
            yield LabeledGreyImage(torch.from_numpy(a.copy()).float() / 255.0, rec.label)


class _Cropper(Transformer):
    def __init__(self, crop_width: int, crop_height: int, cropper_method: str = "random"):
        self.cw, self.ch, self.method = crop_width, crop_height, cropper_method.lower()

    def apply(self, it):
        for img in it:
            h, w = img.height(), img.width()
            if "random" in self.method:
                y = int(np.floor(RNG.uniform(0, h - self.ch + 1))) if h > self.ch else 0
                x = int(np.floor(RNG.uniform(0, w - self.cw + 1))) if w > self.cw else 0
            else:
                y, x = (h - self.ch) // 2, (w - self.cw) // 2
            img.content = img.content[y:y + self.ch, x:x + self.cw].contiguous()
            yield img


class BGRImgCropper(_Cropper):
    pass


class GreyImgCropper(_Cropper):
    pass


class BGRImgRdmCropper(Transformer):
    """Pad then random-crop (CIFAR augmentation)."""

    def __init__(self, crop_width: int, crop_height: int, padding: int):
        self.cw, self.ch, self.pad = crop_width, crop_height, padding

    def apply(self, it):
        for img in it:
            c = img.content
            p = self.pad
            padded = torch.zeros(c.shape[0] + 2 * p, c.shape[1] + 2 * p, c.shape[2])
            padded[p:p + c.shape[0], p:p + c.shape[1]] = c
            y = int(RNG.uniform(0, padded.shape[0] - self.ch + 1))
            x = int(RNG.uniform(0, padded.shape[1] - self.cw + 1))
            img.content = padded[y:y + self.ch, x:x + self.cw].contiguous()
            yield img


class BGRImgNormalizer(Transformer):
    """Per-channel ``(x - mean) / std``; arguments in R, G, B order."""

    def __init__(self, mean_r, mean_g=None, mean_b=None, std_r=1.0, std_g=1.0, std_b=1.0):
        if isinstance(mean_r, (tuple, list)):
            (mean_r, mean_g, mean_b), (std_r, std_g, std_b) = mean_r, mean_g
        self.mean = torch.tensor([mean_b, mean_g, mean_r], dtype=torch.float32)
        self.std = torch.tensor([std_b, std_g, std_r], dtype=torch.float32)

    @staticmethod
    def from_dataset(images: List[LabeledBGRImage], samples: int = -1) -> "BGRImgNormalizer":
        imgs = images if samples <= 0 else images[:samples]
        allpx = torch.cat([i.content.reshape(-1, 3) for i in imgs])
        m = allpx.mean(0)
        s = allpx.std(0, unbiased=False)
        return BGRImgNormalizer(float(m[2]), float(m[1]), float(m[0]), float(s[2]), float(s[1]), float(s[0]))

    def getMean(self):
        return float(self.mean[2]), float(self.mean[1]), float(self.mean[0])

    def getStd(self):
        return float(self.std[2]), float(self.std[1]), float(self.std[0])

    def apply(self, it):
        for img in it:
            img.content = (img.content - self.mean) / self.std
            yield img


class GreyImgNormalizer(Transformer):
    def __init__(self, mean: float, std: float):
        self.mean, self.std = mean, std

    def apply(self, it):
        for img in it:
            img.content = (img.content - self.mean) / self.std
            yield img


class BGRImgPixelNormalizer(Transformer):
    def __init__(self, means: torch.Tensor):
        self.means = torch.as_tensor(means, dtype=torch.float32)

    def apply(self, it):
        for img in it:
            img.content = img.content - self.means.reshape(img.content.shape)
            yield img


class HFlip(Transformer):
    def __init__(self, threshold: float = 0.5):
        self.threshold = threshold

    def apply(self, it):
        for img in it:
            if RNG.uniform(0, 1) >= self.threshold:
                img.hflip()
            yield img


class ColorJitter(Transformer):
    """Random-order brightness / contrast / saturation jitter (fb.resnet.torch style,
    ``dataset/image/ColorJitter.scala``), strength 0.4 each."""

    def __init__(self, brightness=0.4, contrast=0.4, saturation=0.4):
        self.b, self.c, self.s = brightness, contrast, saturation

    @staticmethod
    def _grey(c):
        return (0.299 * c[..., 2] + 0.587 * c[..., 1] + 0.114 * c[..., 0]).unsqueeze(-1)

    def apply(self, it):
        for img in it:
            for i in RNG.permutation(3):
                c = img.content
                if i == 0:
                    a = 1 + RNG.uniform(-self.b, self.b)
                    img.content = c * a
                elif i == 1:
                    a = 1 + RNG.uniform(-self.c, self.c)
                    img.content = c * a + self._grey(c).mean() * (1 - a)
                else:
                    a = 1 + RNG.uniform(-self.s, self.s)
                    img.content = c * a + self._grey(c) * (1 - a)
            yield img


class Lighting(Transformer):
    """AlexNet-style PCA lighting noise (``dataset/image/Lighting.scala``)."""

    alphastd = 0.1
    eigval = torch.tensor([0.2175, 0.0188, 0.0045])
    eigvec = torch.tensor([[-0.5675, 0.7192, 0.4009], [-0.5808, -0.0045, -0.8140], [-0.5836, -0.6948, 0.4203]])

    def apply(self, it):
        for img in it:
            alpha = torch.tensor([RNG.uniform(0, self.alphastd) for _ in range(3)])
            rgb = (self.eigvec * alpha.view(1, 3) * self.eigval.view(1, 3)).sum(1)
            img.content = img.content + rgb
            yield img


class _ToBatch(Transformer):
    def __init__(self, batch_size: int, to_rgb: bool = True):
        self.bs, self.to_rgb = batch_size, to_rgb

    def _make(self, buf):
        x = torch.stack([i.to_chw(self.to_rgb) for i in buf])
        y = torch.tensor([i.label() for i in buf])
        return MiniBatch(x, y)

    def apply(self, it):
        buf = []
        for img in it:
            buf.append(img)
            if len(buf) == self.bs:
                yield self._make(buf)
                buf = []
        if buf:
            yield self._make(buf)


class BGRImgToBatch(_ToBatch):
    pass


class GreyImgToBatch(_ToBatch):
    def __init__(self, batch_size: int):
        super().__init__(batch_size, False)


class MTLabeledBGRImgToBatch(_ToBatch):
    """Batches of ``width × height`` built by ``num_threads`` workers running ``transformer`` on
    each record (``MTLabeledBGRImgToBatch.scala``)."""

    def __init__(self, width: int, height: int, batch_size: int, transformer: Transformer, to_rgb: bool = True,
                 num_threads: int = 4):
        super().__init__(batch_size, to_rgb)
        self.w, self.h, self.t = width, height, transformer
        self.pool = ThreadPoolExecutor(max(1, num_threads))

    def _one(self, rec):
        return next(iter(self.t(iter([rec]))))

    def apply(self, it):
        buf = []
        for rec in it:
            buf.append(rec)
            if len(buf) == self.bs:
                yield self._make(list(self.pool.map(self._one, buf)))
                buf = []
        if buf:
            yield self._make(list(self.pool.map(self._one, buf)))


class BGRImgToSample(Transformer):
    def __init__(self, to_rgb: bool = True):
        self.to_rgb = to_rgb

    def apply(self, it):
        for img in it:
            yield Sample(img.to_chw(self.to_rgb), torch.tensor([img.label()]))


class GreyImgToSample(Transformer):
    def apply(self, it):
        for img in it:
            yield Sample(img.content.permute(2, 0, 1).contiguous(), torch.tensor([img.label()]))


class LocalImageFiles:
    """Scan a class-per-subfolder directory → [(path, 1-based label)] (``LocalImageFiles.scala``)."""

    @staticmethod
    def read_paths(root: str) -> List[Tuple[str, float]]:
        classes = sorted(d for d in os.listdir(root) if os.path.isdir(os.path.join(root, d)))
        out = []
        for li, c in enumerate(classes):
            for f in sorted(os.listdir(os.path.join(root, c))):
                out.append((os.path.join(root, c, f), float(li + 1)))
        return out

    readPaths = read_paths


class LocalImgReader(Transformer):
    """(path, label) → LabeledBGRImage, optionally rescaling the shorter side to ``scale_to``."""

    def __init__(self, scale_to: int = -1, normalize: float = 255.0):
        self.scale_to, self.normalize = scale_to, normalize

    def apply(self, it):
        from ..transform.vision.image.augmentation import resize_mat
        from ..transform.vision.image.convertor import decode_bytes
        for path, label in it:
            with open(path, "rb") as f:
                m = decode_bytes(f.read()).float()
            if self.scale_to > 0:
                h, w = m.shape[0], m.shape[1]
                s = self.scale_to / min(h, w)
                m = resize_mat(m, int(round(h * s)), int(round(w * s)))
            yield LabeledBGRImage(m / self.normalize, label)
