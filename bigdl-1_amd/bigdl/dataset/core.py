"""Samples, mini-batches, datasets and transformers.

Reference: ``DL/dataset/Sample.scala:39-586`` (``ArraySample``), ``MiniBatch.scala:34-764``
(``slice`` 1-based, padding strategies), ``Transformer.scala`` (``->`` chaining,
``SampleToMiniBatch`` 309-391), ``DataSet.scala:53-669`` (``LocalArrayDataSet``, ``CachedDistriDataSet``
with an infinite shuffled iterator in train mode at 247-324).

One process per GPU replaces the Spark partition: ``DistributedDataSet`` gives each rank the
shard ``data[rank::world]`` and a per-epoch reshuffle seeded identically on every rank, and
``DevicePrefetcher`` moves the next batch to HBM on a side stream while the current one runs.
"""
from __future__ import annotations

import math
from typing import Callable, Iterable, Iterator, List, Optional, Sequence

import numpy as np
import torch

from ..utils.random import RNG
from ..utils.table import Table


def _t(x):
    if isinstance(x, torch.Tensor):
        return x
    if hasattr(x, "data") and isinstance(getattr(x, "data"), torch.Tensor):
        return x.data
    return torch.as_tensor(np.asarray(x))


class Sample:
    """Features and labels, each a list of tensors (``ArraySample``)."""

    def __init__(self, features, labels=None):
        self.features: List[torch.Tensor] = [_t(f) for f in (features if isinstance(features, (list, tuple)) else [features])]
        if labels is None:
            self.labels: List[torch.Tensor] = []
        else:
            self.labels = [_t(l) for l in (labels if isinstance(labels, (list, tuple)) else [labels])]

    @staticmethod
    def from_ndarray(features, labels=None):
        if isinstance(labels, (int, float, np.integer, np.floating)):
            labels = np.array([labels], dtype=np.float32)
        return Sample(features, labels)

    @staticmethod
    def from_tensor(features, labels=None):
        return Sample(features, labels)

    def feature(self, i: int = 0):
        return self.features[i]

    def label(self, i: int = 0):
        return self.labels[i] if self.labels else None

    def numFeature(self):
        return len(self.features)

    def numLabel(self):
        return len(self.labels)

    def getFeatureSize(self):
        return [list(f.shape) for f in self.features]

    def getLabelSize(self):
        return [list(l.shape) for l in self.labels]

    def __repr__(self):
        return f"Sample(features={[tuple(f.shape) for f in self.features]}, labels={[tuple(l.shape) for l in self.labels]})"


class PaddingParam:
    """Pad variable-length features in a batch (``MiniBatch.scala:528-580``)."""

    def __init__(self, padding_tensor=None, fixed_length=None):
        self.paddingTensor = padding_tensor
        self.fixedLength = fixed_length


class MiniBatch:
    """A batch of input / target activities (``MiniBatch.scala:34``; ``ArrayTensorMiniBatch`` 111)."""

    def __init__(self, input, target=None):
        self.input = input
        self.target = target

    def size(self) -> int:
        x = self.input[1] if isinstance(self.input, Table) else self.input
        return int(x.shape[0])

    def getInput(self):
        return self.input

    def getTarget(self):
        return self.target

    def slice(self, offset: int, length: int) -> "MiniBatch":
        def sl(a):
            if a is None:
                return None
            if isinstance(a, Table):
                t = Table()
                for k, v in a.items():
                    t[k] = sl(v)
                return t
            return a.narrow(0, offset - 1, length)
        return MiniBatch(sl(self.input), sl(self.target))

    def to(self, device, non_blocking=True, dtype=None):
        def mv(a):
            if a is None:
                return None
            if isinstance(a, Table):
                t = Table()
                for k, v in a.items():
                    t[k] = mv(v)
                return t
            r = a.to(device, non_blocking=non_blocking)
            if dtype is not None and r.is_floating_point():
                r = r.to(dtype)
            return r
        return MiniBatch(mv(self.input), mv(self.target))

    def pin_memory(self):
        def pn(a):
            if a is None:
                return None
            if isinstance(a, Table):
                t = Table()
                for k, v in a.items():
                    t[k] = pn(v)
                return t
            return a.pin_memory() if (torch.cuda.is_available() and not a.is_cuda) else a
        return MiniBatch(pn(self.input), pn(self.target))


ArrayTensorMiniBatch = MiniBatch


class DefaultPadding(PaddingParam):
    """Pad with zeros to the longest sample (``MiniBatch.scala:528-580``)."""

    def __init__(self):
        super().__init__(None, None)


class SparseMiniBatch(MiniBatch):
    """MiniBatch whose features may be sparse (``MiniBatch.scala:588``): ``set(samples)`` stacks
    dense features densely and sparse (COO) features into one [batch, ...] sparse tensor (the
    reference's ``SparseMiniBatch.batch``: indices shifted by the sample's batch row)."""

    def __init__(self, input=None, target=None):
        super().__init__(input, target)

    @staticmethod
    def _batch(ts: List[torch.Tensor]) -> torch.Tensor:
        if not ts[0].is_sparse:
            return torch.stack([t.to_dense() if t.is_sparse else t for t in ts], 0)
        idx, val = [], []
        for b, t in enumerate(ts):
            t = t.coalesce()
            i = t.indices()
            idx.append(torch.cat([torch.full((1, i.shape[1]), b, dtype=i.dtype), i], 0))
            val.append(t.values())
        shape = (len(ts),) + tuple(ts[0].shape)
        return torch.sparse_coo_tensor(torch.cat(idx, 1), torch.cat(val), shape).coalesce()

    def set(self, samples: Sequence["Sample"]) -> "SparseMiniBatch":
        if not samples:
            raise ValueError("samples is empty")
        nf, nl = len(samples[0].features), len(samples[0].labels)
        feats = [self._batch([s.features[i] for s in samples]) for i in range(nf)]
        labs = [self._batch([s.labels[j] for s in samples]) for j in range(nl)]

        def act(xs):
            if not xs:
                return None
            if len(xs) == 1:
                return xs[0]
            t = Table()
            for k, x in enumerate(xs):
                t[k + 1] = x
            return t
        self.input, self.target = act(feats), act(labs)
        return self

    def size(self) -> int:
        x = self.input[1] if isinstance(self.input, Table) else self.input
        return int(x.shape[0])


def _pad_for(padding: Optional[PaddingParam], i: int) -> Optional[PaddingParam]:
    """The padding of feature / label ``i``: a PaddingParam whose ``paddingTensor`` is a list holds
    one padding tensor per feature (``PaddingParam(Some(Array(t1, t2)))``, MiniBatch.scala:528)."""
    if padding is None or not isinstance(padding.paddingTensor, (list, tuple)):
        return padding
    pts = padding.paddingTensor
    if pts and isinstance(pts[0], (torch.Tensor, list, tuple)) and not all(isinstance(v, (int, float)) for v in pts):
        return PaddingParam(pts[i] if i < len(pts) else None, padding.fixedLength)
    return padding


def _stack(tensors: List[torch.Tensor], padding: Optional[PaddingParam] = None):
    shapes = {tuple(t.shape) for t in tensors}
    if len(shapes) == 1 and (padding is None or padding.fixedLength is None):
        return torch.stack(tensors, 0)
    nd = tensors[0].dim()
    maxs = [max(t.shape[d] for t in tensors) for d in range(nd)]
    if padding is not None and padding.fixedLength is not None:
        maxs[0] = max(maxs[0], padding.fixedLength)
    out = torch.zeros([len(tensors)] + maxs, dtype=tensors[0].dtype)
    if padding is not None and padding.paddingTensor is not None:
        out[:] = _t(padding.paddingTensor).to(out.dtype)
    for i, t in enumerate(tensors):
        out[(i,) + tuple(slice(0, s) for s in t.shape)] = t
    return out


class Transformer:
    """Composable iterator transform; ``a >> b`` (Scala ``a -> b``)."""

    def __call__(self, it: Iterator) -> Iterator:
        return self.apply(it)

    def apply(self, it: Iterator) -> Iterator:
        raise NotImplementedError

    def __rshift__(self, other: "Transformer") -> "Transformer":
        return ChainedTransformer(self, other)

    def clone_transformer(self):
        import copy
        return copy.deepcopy(self)


class ChainedTransformer(Transformer):
    def __init__(self, first, last):
        self.first, self.last = first, last

    def apply(self, it):
        return self.last.apply(self.first.apply(it))


class FnTransformer(Transformer):
    def __init__(self, fn: Callable):
        self.fn = fn

    def apply(self, it):
        for x in it:
            yield self.fn(x)


class SampleToMiniBatch(Transformer):
    """Group Samples into MiniBatches (``Transformer.scala:309-391``)."""

    def __init__(self, batch_size: int, feature_padding: PaddingParam = None, label_padding: PaddingParam = None,
                 partition_num: Optional[int] = None, drop_last: bool = False):
        self.batchSize = batch_size
        self.featurePadding, self.labelPadding = feature_padding, label_padding
        self.dropLast = drop_last

    def _make(self, buf: List[Sample]) -> MiniBatch:
        nf = buf[0].numFeature()
        nl = buf[0].numLabel()
        feats = [_stack([s.features[i] for s in buf], _pad_for(self.featurePadding, i)) for i in range(nf)]
        labs = [_stack([s.labels[i] for s in buf], _pad_for(self.labelPadding, i)) for i in range(nl)]
        inp = feats[0] if nf == 1 else Table(*feats)
        tgt = None if nl == 0 else (labs[0] if nl == 1 else Table(*labs))
        return MiniBatch(inp, tgt)

    def apply(self, it):
        buf = []
        for s in it:
            buf.append(s)
            if len(buf) == self.batchSize:
                yield self._make(buf)
                buf = []
        if buf and not self.dropLast:
            yield self._make(buf)


class AbstractDataSet:
    def data(self, train: bool) -> Iterator:
        raise NotImplementedError

    def size(self) -> int:
        raise NotImplementedError

    def shuffle(self):
        pass

    def transform(self, t: Transformer) -> "AbstractDataSet":
        return TransformedDataSet(self, t)

    def __rshift__(self, t: Transformer):
        return self.transform(t)

    def toLocal(self):
        return self

    def toDistributed(self):
        return self


class LocalArrayDataSet(AbstractDataSet):
    def __init__(self, buffer: Sequence):
        self.buffer = list(buffer)
        self.index = np.arange(len(self.buffer))

    def size(self):
        return len(self.buffer)

    def shuffle(self):
        RNG.shuffle(self.index)

    def data(self, train: bool):
        if not train:
            for i in range(len(self.buffer)):
                yield self.buffer[i]
            return
        # infinite loop with a random start offset (DataSet.scala:247-324)
        n = len(self.buffer)
        if n == 0:
            return
        pos = RNG.random() % n
        while True:
            yield self.buffer[self.index[pos % n]]
            pos += 1


class DistributedDataSet(LocalArrayDataSet):
    """Rank-sharded dataset: rank r sees items ``r, r+W, r+2W, …`` of a globally shuffled order
    (same seed on every rank, so shards are disjoint and cover the data)."""

    def __init__(self, buffer: Sequence, rank: Optional[int] = None, world: Optional[int] = None, seed: int = 1234):
        super().__init__(buffer)
        from ..utils.engine import Engine
        self.rank = Engine.rank() if rank is None else rank
        self.world = Engine.world_size() if world is None else world
        self.seed = seed
        self.epoch = 0
        self._reshard()

    def _reshard(self):
        g = np.random.RandomState(self.seed + self.epoch)
        order = g.permutation(len(self.buffer))
        self.index = order[self.rank::self.world]

    def shuffle(self):
        self.epoch += 1
        self._reshard()

    def size(self):
        return len(self.buffer)

    def local_size(self):
        return len(self.index)

    def data(self, train: bool):
        if not train:
            for i in self.index:
                yield self.buffer[i]
            return
        n = len(self.index)
        pos = 0
        while True:
            yield self.buffer[self.index[pos % n]]
            pos += 1
            if pos % n == 0:
                self.shuffle()


class TransformedDataSet(AbstractDataSet):
    def __init__(self, base: AbstractDataSet, t: Transformer):
        self.base, self.t = base, t

    def data(self, train):
        return self.t.apply(self.base.data(train))

    def size(self):
        return self.base.size()

    def shuffle(self):
        self.base.shuffle()

    def local_size(self):
        return getattr(self.base, "local_size", self.base.size)()

    def transform(self, t):
        return TransformedDataSet(self.base, ChainedTransformer(self.t, t))


class SyntheticDataSet(AbstractDataSet):
    """Constant device-resident batches (the reference's perf harness trick,
    ``DL/models/utils/DistriOptimizerPerf.scala:114-119``)."""

    def __init__(self, batch: MiniBatch, epoch_size: int):
        self.batch = batch
        self.epoch_size = epoch_size

    def data(self, train):
        if train:
            while True:
                yield self.batch
        else:
            for _ in range(max(1, self.epoch_size // self.batch.size())):
                yield self.batch

    def size(self):
        return self.epoch_size

    def local_size(self):
        return self.epoch_size


class DataSet:
    """Factory (``object DataSet``)."""

    @staticmethod
    def array(data: Sequence, distributed: bool = False) -> AbstractDataSet:
        return DistributedDataSet(data) if distributed else LocalArrayDataSet(data)

    @staticmethod
    def rdd(data: Sequence) -> AbstractDataSet:
        """pyspark RDD inputs become a rank-sharded in-process collection."""
        return DistributedDataSet(list(data))

    @staticmethod
    def from_samples(samples: Sequence[Sample], batch_size: int, distributed: bool = False):
        return DataSet.array(samples, distributed).transform(SampleToMiniBatch(batch_size))

    @staticmethod
    def imageFrame(frame, distributed: bool = False) -> AbstractDataSet:
        """DataSet of the ImageFeatures of an ImageFrame (``DataSet.imageFrame``)."""
        feats = frame.to_local().array if hasattr(frame, "to_local") else list(frame)
        return DataSet.array(list(feats), distributed)

    image_frame = imageFrame

    class ImageFolder:
        """Class-per-subfolder image trees (``DataSet.scala:424-481``): subfolder i (sorted) is
        label i + 1."""

        @staticmethod
        def paths(path: str, distributed: bool = False) -> AbstractDataSet:
            from .image import LocalImageFiles
            return DataSet.array(LocalImageFiles.read_paths(path), distributed)

        @staticmethod
        def images(path: str, scale_to: int = -1, distributed: bool = False) -> AbstractDataSet:
            """Decoded LabeledBGRImage records (pixels / 255, shorter side scaled to ``scale_to``),
            cached in memory like the reference."""
            from .image import LocalImageFiles, LocalImgReader
            imgs = list(LocalImgReader(scale_to).apply(iter(LocalImageFiles.read_paths(path))))
            return DataSet.array(imgs, distributed)

    class SeqFileFolder:
        """Hadoop SequenceFile image folders (``DataSet.scala:486-640``): LabeledBGRImage records
        (pixels / 255) of every ``.seq`` file under ``path``."""

        @staticmethod
        def files(path: str, class_num: Optional[int] = None, distributed: bool = False) -> AbstractDataSet:
            from .image import LabeledBGRImage
            from .seqfile import SeqFileFolder as _SF
            recs = [LabeledBGRImage(torch.from_numpy(img.astype(np.float32) / 255.0), label)
                    for img, label, _ in _SF.read(path, class_num)]
            return DataSet.array(recs, distributed)


class DevicePrefetcher:
    """Double-buffered H2D copies on a side HIP stream (pinned host → HBM)."""

    def __init__(self, it: Iterator[MiniBatch], device, dtype=None):
        self.it = it
        self.device = torch.device(device)
        self.dtype = dtype
        self.stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None
        self._next = None
        self._preload()

    def _preload(self):
        try:
            b = next(self.it)
        except StopIteration:
            self._next = None
            return
        if self.stream is None:
            self._next = b.to(self.device, dtype=self.dtype) if self.dtype else b
            return
        if _on_device(b, self.device):
            self._next = b
            return
        b = b.pin_memory()
        with torch.cuda.stream(self.stream):
            self._next = b.to(self.device, non_blocking=True)

    def __iter__(self):
        return self

    def __next__(self):
        if self._next is None:
            raise StopIteration
        if self.stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.stream)
        b = self._next
        self._preload()
        return b


def _on_device(b: MiniBatch, device) -> bool:
    x = b.input[1] if isinstance(b.input, Table) else b.input
    return isinstance(x, torch.Tensor) and x.device == device
