"""ImageFeature / ImageFrame / FeatureTransformer (``DL/transform/vision/image/{ImageFeature,
ImageFrame,FeatureTransformer}.scala``).

An image ("mat") is a torch tensor ``[H, W, C]`` float32 in **BGR** channel order, the OpenCV
convention the reference's transforms assume.  It may live on the host or on the GPU: every
augmentation below is written with torch tensor ops, so after ``ToDevice`` the whole chain runs
in HBM (and the common crop/flip/normalise tail has a fused HIP kernel, ``bigdl.ops``).
"""
from __future__ import annotations

import os
from typing import Callable, Iterable, List, Optional

import numpy as np
import torch

from ....utils.engine import Engine


class ImageFeature(dict):
    uri = "uri"
    mat = "mat"
    bytes = "bytes"
    floats = "floats"
    size = "size"
    originalSize = "originalSize"
    label = "label"
    predict = "predict"
    boundingBox = "boundingBox"
    sample = "sample"
    imageTensor = "imageTensor"
    cropBbox = "cropBbox"
    expandBbox = "expandBbox"

    def __init__(self, bytes_=None, label=None, uri: Optional[str] = None, image=None):
        super().__init__()
        self._valid = True
        if bytes_ is not None:
            self[ImageFeature.bytes] = bytes_
        if label is not None:
            self[ImageFeature.label] = label
        if uri is not None:
            self[ImageFeature.uri] = uri
        if image is not None:
            self.set_mat(image)

    # --- accessors (ImageFeature.scala) ---------------------------------------------------------
    def is_valid(self) -> bool:
        return self._valid

    isValid = is_valid

    def set_valid(self, v: bool):
        self._valid = v

    def opencv_mat(self) -> torch.Tensor:
        return self[ImageFeature.mat]

    opencvMat = opencv_mat

    def set_mat(self, m: torch.Tensor):
        if isinstance(m, np.ndarray):
            m = torch.from_numpy(np.ascontiguousarray(m))
        if m.dim() == 2:
            m = m.unsqueeze(-1)
        self[ImageFeature.mat] = m.float()
        if ImageFeature.originalSize not in self:
            self[ImageFeature.originalSize] = (m.shape[0], m.shape[1], m.shape[2])
        return self

    def get_size(self):
        m = self.get(ImageFeature.mat)
        return None if m is None else (m.shape[0], m.shape[1], m.shape[2])

    getSize = get_size

    def get_height(self):
        return self.get_size()[0]

    def get_width(self):
        return self.get_size()[1]

    def get_original_size(self):
        return self.get(ImageFeature.originalSize)

    getOriginalSize = get_original_size

    def get_original_height(self):
        return self.get_original_size()[0]

    def get_original_width(self):
        return self.get_original_size()[1]

    def get_label(self):
        return self.get(ImageFeature.label)

    getLabel = get_label

    def get_uri(self):
        return self.get(ImageFeature.uri)

    def get_image(self, key: str = "imageTensor"):
        return self.get(key)

    def get_sample(self):
        return self.get(ImageFeature.sample)

    getSample = get_sample

    def get_predict(self, key: str = "predict"):
        return self.get(key)

    def has_label(self):
        return ImageFeature.label in self

    def to_chw(self, to_rgb: bool = False) -> torch.Tensor:
        m = self.opencv_mat()
        if to_rgb and m.shape[2] == 3:
            m = m.flip(2)
        return m.permute(2, 0, 1).contiguous()

    def clone(self):
        f = ImageFeature()
        for k, v in self.items():
            f[k] = v.clone() if isinstance(v, torch.Tensor) else v
        f._valid = self._valid
        return f


class FeatureTransformer:
    """Transforms an ImageFeature in place; ``a >> b`` (Scala ``->``) chains.  A failing transform
    marks the feature invalid instead of raising (``FeatureTransformer.transform``)."""

    ignore_exception = False

    def transform_mat(self, feature: ImageFeature):
        pass

    def transform(self, feature: ImageFeature) -> ImageFeature:
        if not feature.is_valid():
            return feature
        try:
            self.transform_mat(feature)
        except Exception:  # noqa: BLE001 - reference marks the feature invalid
            if not self.ignore_exception:
                feature.set_valid(False)
                raise
            feature.set_valid(False)
        return feature

    def __call__(self, x):
        if isinstance(x, ImageFrame):
            return x.transform(self)
        if isinstance(x, ImageFeature):
            return self.transform(x)
        return (self.transform(f) for f in x)

    def apply(self, it):
        return self(it)

    def __rshift__(self, other: "FeatureTransformer") -> "FeatureTransformer":
        return ChainedFeatureTransformer(self, other)

    def enable_ignore_exception(self):
        self.ignore_exception = True
        return self


class ChainedFeatureTransformer(FeatureTransformer):
    def __init__(self, first: FeatureTransformer, last: FeatureTransformer):
        self.first, self.last = first, last

    def transform(self, feature):
        return self.last.transform(self.first.transform(feature))


class Pipeline(FeatureTransformer):
    """Convenience: ``Pipeline([t1, t2, ...])`` = ``t1 >> t2 >> ...``."""

    def __init__(self, transformers: List[FeatureTransformer]):
        self.transformers = list(transformers)

    def transform(self, feature):
        for t in self.transformers:
            feature = t.transform(feature)
        return feature


class ImageFrame:
    """Collection of ImageFeatures: ``LocalImageFrame`` (an array) or ``DistributedImageFrame``
    (this rank's shard of the frame — the reference's RDD partitions)."""

    @staticmethod
    def array(features: Iterable[ImageFeature]) -> "LocalImageFrame":
        return LocalImageFrame(list(features))

    @staticmethod
    def read(path: str, distributed: bool = False, with_label: bool = False) -> "ImageFrame":
        """Read every image file under ``path`` (a file or a directory; with ``with_label`` the
        sub-directory index, 1-based in sorted order, becomes the label)."""
        files, labels = [], []
        if os.path.isdir(path):
            subdirs = sorted(d for d in os.listdir(path) if os.path.isdir(os.path.join(path, d)))
            if with_label and subdirs:
                for li, d in enumerate(subdirs):
                    for f in sorted(os.listdir(os.path.join(path, d))):
                        files.append(os.path.join(path, d, f))
                        labels.append(float(li + 1))
            else:
                for root, _, fs in sorted(os.walk(path)):
                    for f in sorted(fs):
                        files.append(os.path.join(root, f))
        else:
            files = [path]
        feats = []
        for i, fp in enumerate(files):
            with open(fp, "rb") as fh:
                b = fh.read()
            feats.append(ImageFeature(b, labels[i] if labels else None, fp))
        from .convertor import BytesToMat
        frame = LocalImageFrame(feats) if not distributed else DistributedImageFrame(feats)
        return frame.transform(BytesToMat())

    def transform(self, t: FeatureTransformer) -> "ImageFrame":
        raise NotImplementedError

    def __rshift__(self, t):
        return self.transform(t)

    def is_local(self):
        return isinstance(self, LocalImageFrame)

    isLocal = is_local

    def is_distributed(self):
        return isinstance(self, DistributedImageFrame)

    isDistributed = is_distributed


class LocalImageFrame(ImageFrame):
    def __init__(self, array: List[ImageFeature]):
        self.array = array

    def transform(self, t):
        self.array = [t.transform(f) for f in self.array]
        return self

    def to_local(self):
        return self

    toLocal = to_local

    def to_distributed(self, rank: Optional[int] = None, world: Optional[int] = None):
        return DistributedImageFrame(self.array, rank, world)

    def __iter__(self):
        return iter(self.array)

    def __len__(self):
        return len(self.array)

    def get_image(self, key="imageTensor"):
        return [f.get(key) for f in self.array]

    def get_label(self):
        return [f.get_label() for f in self.array]

    def get_predict(self, key="predict"):
        return [(f.get_uri(), f.get(key)) for f in self.array]

    def get_sample(self):
        return [f.get_sample() for f in self.array]


class DistributedImageFrame(LocalImageFrame):
    """Holds this rank's contiguous shard of the features."""

    def __init__(self, features: List[ImageFeature], rank: Optional[int] = None, world: Optional[int] = None):
        r = Engine.rank() if rank is None else rank
        w = Engine.world_size() if world is None else world
        n = len(features)
        per = (n + w - 1) // w
        super().__init__(list(features[r * per:(r + 1) * per]))
        self.rank, self.world, self.total = r, w, n

    def to_local(self):
        return LocalImageFrame(self.array)
