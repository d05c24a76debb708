"""Decoding and batching (``DL/transform/vision/image/{Convertor,MTImageFeatureToBatch}.scala``).

* ``BytesToMat`` decodes encoded bytes (JPEG/PNG/…; PIL stands in for OpenCV ``imdecode``) into
  a BGR float ``[H, W, C]`` mat; ``PixelBytesToMat`` reinterprets raw HWC uint8 pixels.
* ``MatToTensor`` / ``MatToFloats`` / ``ImageFrameToSample`` / ``ImageFeatureToMiniBatch``.
* ``MTImageFeatureToBatch``: the training-batch assembler.  On a GPU it uploads the uint8 pixels
  once (pinned, async) and runs the fused crop + mirror + per-channel normalise + bf16 NHWC cast
  HIP kernel (``ops.image_crop_flip_norm``, kernel K25) — the device-side replacement of the
  reference's per-image OpenCV loop.
"""
from __future__ import annotations

import io
from concurrent.futures import ThreadPoolExecutor
from typing import List, Optional, Sequence

import numpy as np
import torch

from ....dataset import MiniBatch, Sample, SampleToMiniBatch
from ....utils.engine import Engine
from ....utils.random import RNG
from ....utils.table import Table
from .image_feature import FeatureTransformer, ImageFeature


def decode_bytes(b: bytes) -> torch.Tensor:
    from PIL import Image
    img = Image.open(io.BytesIO(b))
    if img.mode not in ("RGB", "L"):
        img = img.convert("RGB")
    a = np.asarray(img, dtype=np.uint8)
    if a.ndim == 2:
        a = a[:, :, None]
    else:
        a = a[:, :, ::-1]  # RGB → BGR
    return torch.from_numpy(np.ascontiguousarray(a))


class BytesToMat(FeatureTransformer):
    def __init__(self, byte_key: str = ImageFeature.bytes):
        self.key = byte_key

    def transform_mat(self, f):
        f.set_mat(decode_bytes(f[self.key]).float())


class PixelBytesToMat(FeatureTransformer):
    """Raw pixel bytes in HWC order; the size comes from ``originalSize``."""

    def __init__(self, byte_key: str = ImageFeature.bytes):
        self.key = byte_key

    def transform_mat(self, f):
        h, w, c = f[ImageFeature.originalSize]
        a = np.frombuffer(f[self.key], dtype=np.uint8).reshape(h, w, c)
        f.set_mat(torch.from_numpy(a.copy()).float())


class MatToFloats(FeatureTransformer):
    def __init__(self, valid_height: int = 300, valid_width: int = 300, valid_channels: int = 3,
                 out_key: str = ImageFeature.floats, share_buffer: bool = True):
        self.h, self.w, self.c, self.key = valid_height, valid_width, valid_channels, out_key

    def transform_mat(self, f):
        m = f.opencv_mat() if ImageFeature.mat in f else torch.zeros(self.h, self.w, self.c)
        f[self.key] = m.reshape(-1).float()


class MatToTensor(FeatureTransformer):
    """HWC BGR mat → CHW tensor (RGB with ``to_rgb``) under ``tensor_key``."""

    def __init__(self, to_rgb: bool = False, tensor_key: str = ImageFeature.imageTensor, share_buffer: bool = True,
                 greyToRGB: bool = False):
        self.to_rgb, self.key, self.grey_to_rgb = to_rgb, tensor_key, greyToRGB

    def transform_mat(self, f):
        t = f.to_chw(self.to_rgb)
        if self.grey_to_rgb and t.shape[0] == 1:
            t = t.expand(3, -1, -1).contiguous()
        f[self.key] = t


class ImageFrameToSample(FeatureTransformer):
    def __init__(self, input_keys: Sequence[str] = (ImageFeature.imageTensor,), target_keys: Sequence[str] = None,
                 sample_key: str = ImageFeature.sample):
        self.inputs, self.targets, self.key = list(input_keys), list(target_keys or []), sample_key

    def transform_mat(self, f):
        feats = [f[k] for k in self.inputs]
        labs = [torch.as_tensor(f[k], dtype=torch.float32).reshape(-1) for k in self.targets if k in f]
        f[self.key] = Sample(feats, labs if labs else None)


class ImageFeatureToMiniBatch:
    """ImageFeatures (with ``sample``) → MiniBatches of ``batch_size``."""

    def __init__(self, batch_size: int, feature_padding=None, label_padding=None, partition_num=None,
                 sample_key: str = ImageFeature.sample):
        self.stm = SampleToMiniBatch(batch_size, feature_padding, label_padding, partition_num)
        self.key = sample_key

    def __call__(self, features):
        return self.stm(f[self.key] for f in features if f.is_valid())

    apply = __call__


class MTImageFeatureToBatch:
    """Classification batches of ``width × height``: each feature is transformed by
    ``transformer`` on ``num_threads`` host threads (decode, resize, jitter …); the final crop /
    mirror / normalise / cast runs either per image on the host, or — ``device="cuda"`` — as one
    fused HIP kernel over the whole batch.  Output: MiniBatch(input NCHW-logical channels-last,
    target 1-based labels)."""

    def __init__(self, width: int, height: int, batch_size: int, transformer: Optional[FeatureTransformer] = None,
                 to_rgb: bool = True, mean=(0.0, 0.0, 0.0), std=(1.0, 1.0, 1.0), random_crop: bool = False,
                 mirror: bool = False, device: Optional[str] = None, num_threads: int = 4,
                 out_dtype: Optional[torch.dtype] = None):
        self.w, self.h, self.bs = width, height, batch_size
        self.transformer = transformer
        self.to_rgb, self.mean, self.std = to_rgb, list(mean), list(std)
        self.random_crop, self.mirror = random_crop, mirror
        self.device = torch.device(device) if device else Engine.device()
        self.pool = ThreadPoolExecutor(max(1, num_threads))
        self.out_dtype = out_dtype

    def _prep(self, f: ImageFeature):
        if self.transformer is not None:
            f = self.transformer.transform(f)
        return f

    def __call__(self, features):
        buf = []
        for f in features:
            buf.append(f)
            if len(buf) == self.bs:
                yield self._make(buf)
                buf = []
        if buf:
            yield self._make(buf)

    apply = __call__

    def _make(self, feats: List[ImageFeature]) -> MiniBatch:
        feats = [f for f in self.pool.map(self._prep, feats) if f.is_valid()]
        mats = [f.opencv_mat() for f in feats]
        H = min(m.shape[0] for m in mats)
        W = min(m.shape[1] for m in mats)
        C = mats[0].shape[2]
        B = len(mats)
        oy, ox, fl = [], [], []
        for m in mats:
            hh, ww = m.shape[0], m.shape[1]
            if self.random_crop:
                oy.append(int(RNG.uniform(0, hh - self.h + 1)) if hh > self.h else 0)
                ox.append(int(RNG.uniform(0, ww - self.w + 1)) if ww > self.w else 0)
            else:
                oy.append(max(0, (hh - self.h) // 2))
                ox.append(max(0, (ww - self.w) // 2))
            fl.append(1 if (self.mirror and RNG.uniform(0, 1) < 0.5) else 0)
        labels = torch.tensor([float(f.get_label() if f.get_label() is not None else 0) for f in feats])
        # gather the crop windows (plus a margin-free stack) so the kernel sees one dense batch
        crops = torch.stack([m[y:y + self.h, x:x + self.w] for m, y, x in zip(mats, oy, ox)])
        from .... import ops
        mean = self.mean[::-1] if not self.to_rgb else self.mean
        std = self.std[::-1] if not self.to_rgb else self.std
        x = ops.image_crop_flip_norm(crops.to(self.device, non_blocking=True), torch.zeros(B, dtype=torch.int32),
                                     torch.zeros(B, dtype=torch.int32), torch.tensor(fl, dtype=torch.int32),
                                     self.h, self.w, mean, std, self.to_rgb,
                                     self.out_dtype or (Engine.compute_dtype() if self.device.type == "cuda"
                                                        else torch.float32))
        return MiniBatch(x, labels.to(self.device))
