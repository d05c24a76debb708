"""``NativeBatchLoader``: C++ worker threads assemble augmented minibatches straight into pinned
host slots; the iterator copies each slot to the device asynchronously on a side stream and hands
the slot back to the workers once that copy has completed (event-tracked).

Reference behaviour: ``MTLabeledBGRImgToBatch`` / ``MTImageFeatureToBatch`` (multi-threaded batch
assembly, ``DL/dataset/image/MTLabeledBGRImgToBatch.scala``) with the usual CIFAR/ImageNet
augmentations (``BGRImgRdmCropper`` with padding, ``HFlip``, ``BGRImgNormalizer``) and the infinite
shuffled iterator of ``CachedDistriDataSet`` (``DL/dataset/DataSet.scala:247-324``).  With
``rank``/``world`` each rank reads its own contiguous partition of the array.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional, Sequence

import numpy as np
import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "lib", "libbigdl_runtime.so")
_lib = None


def runtime_library():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            from ..ops.build import build_runtime
            build_runtime(verbose=False)
        lib = C.CDLL(_LIB_PATH)
        lib.bigdl_loader_create.restype = C.c_void_p
        lib.bigdl_loader_create.argtypes = [
            C.c_void_p, C.c_void_p, C.c_longlong, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
            C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_ulonglong,
            C.c_int, C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]
        lib.bigdl_loader_next.restype = C.c_int
        lib.bigdl_loader_next.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_longlong)]
        lib.bigdl_loader_release.argtypes = [C.c_void_p, C.c_int]
        lib.bigdl_loader_batches_per_epoch.restype = C.c_longlong
        lib.bigdl_loader_batches_per_epoch.argtypes = [C.c_void_p]
        lib.bigdl_loader_destroy.argtypes = [C.c_void_p]
        _lib = lib
    return _lib


class NativeBatchLoader:
    def __init__(self, images: np.ndarray, labels: Optional[np.ndarray], batch_size: int,
                 crop: Optional[Sequence[int]] = None, pad: int = 0, flip: bool = False, train: bool = True,
                 mean: Optional[Sequence[float]] = None, std: Optional[Sequence[float]] = None,
                 dtype: torch.dtype = torch.float32, layout: str = "NCHW", shuffle: bool = True,
                 drop_last: bool = True, seed: int = 1, threads: int = 4, prefetch: int = 4,
                 device: Optional[torch.device] = None, rank: int = 0, world: int = 1):
        if images.dtype != np.uint8 or images.ndim != 4:
            raise ValueError("images must be a uint8 array [N, H, W, C]")
        if world > 1:
            per = images.shape[0] // world
            images = images[rank * per:(rank + 1) * per]
            labels = labels[rank * per:(rank + 1) * per] if labels is not None else None
        self.images = np.ascontiguousarray(images)
        n, h, w, c = self.images.shape
        self.labels = None
        ld = 0
        if labels is not None:
            lab = np.ascontiguousarray(labels, dtype=np.float32).reshape(n, -1)
            self.labels, ld = lab, lab.shape[1]
        ch, cw = (crop or (h, w))
        if dtype not in (torch.float32, torch.bfloat16):
            raise ValueError("dtype must be float32 or bfloat16")
        self.batch, self.c, self.ch, self.cw, self.ld = batch_size, c, ch, cw, ld
        self.layout = layout.upper()
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        pin = self.device.type == "cuda"
        k = max(2, int(prefetch))
        shape = (batch_size, ch, cw, c) if self.layout == "NHWC" else (batch_size, c, ch, cw)
        self._x = [torch.empty(shape, dtype=dtype, pin_memory=pin) for _ in range(k)]
        self._y = [torch.empty((batch_size, max(ld, 1)), dtype=torch.float32, pin_memory=pin) for _ in range(k)]
        self._mean = np.asarray(mean if mean is not None else [0.0] * c, dtype=np.float32)
        self._std = np.asarray(std if std is not None else [1.0] * c, dtype=np.float32)
        xs = (C.c_void_p * k)(*[t.data_ptr() for t in self._x])
        ys = (C.c_void_p * k)(*[t.data_ptr() for t in self._y])
        lib = runtime_library()
        self._h = lib.bigdl_loader_create(
            self.images.ctypes.data, self.labels.ctypes.data if self.labels is not None else None, n, h, w, c, ld,
            batch_size, ch, cw, pad, int(flip), int(train), self._mean.ctypes.data, self._std.ctypes.data,
            int(dtype == torch.bfloat16), int(self.layout == "NHWC"), int(shuffle), int(drop_last), seed,
            max(1, threads), k, xs, ys)
        if not self._h:
            raise ValueError("invalid NativeBatchLoader configuration")
        self._pending = []  # (slot, event) copies in flight
        self._stream = torch.cuda.Stream(self.device) if pin else None

    def batches_per_epoch(self) -> int:
        return int(runtime_library().bigdl_loader_batches_per_epoch(self._h))

    def _recycle(self, block: bool):
        keep = []
        for slot, ev in self._pending:
            if ev is None or block or ev.query():
                if ev is not None:
                    ev.synchronize()
                runtime_library().bigdl_loader_release(self._h, slot)
            else:
                keep.append((slot, ev))
        self._pending = keep

    def next_batch(self):
        """(x, y) on the target device; x is (rows, C, H, W) or (rows, H, W, C), y (rows[, L])."""
        from ..dataset import MiniBatch
        self._recycle(block=len(self._pending) >= len(self._x) - 1)
        rows, bi = C.c_int(0), C.c_longlong(0)
        slot = runtime_library().bigdl_loader_next(self._h, C.byref(rows), C.byref(bi))
        r = rows.value
        x, y = self._x[slot][:r], self._y[slot][:r]
        if self.ld == 1:
            y = y[:, 0]
        if self._stream is not None:
            with torch.cuda.stream(self._stream):
                xd = x.to(self.device, non_blocking=True)
                yd = y.to(self.device, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self._stream)
            torch.cuda.current_stream(self.device).wait_event(ev)
            xd.record_stream(torch.cuda.current_stream(self.device))
            yd.record_stream(torch.cuda.current_stream(self.device))
            self._pending.append((slot, ev))
        else:
            xd, yd = x.clone(), y.clone()
            self._pending.append((slot, None))
        if self.layout == "NHWC" and xd.dim() == 4:
            xd = xd.permute(0, 3, 1, 2)  # logical NCHW view of NHWC memory (channels_last)
        return MiniBatch(xd, yd if self.ld else None)

    def __iter__(self):
        while True:
            yield self.next_batch()

    def data(self, train: bool = True):
        """Training: the infinite shuffled stream.  ``train=False`` (validation / evaluation): one
        pass over the partition, ``batches_per_epoch()`` batches."""
        if train:
            return iter(self)
        return (self.next_batch() for _ in range(self.batches_per_epoch()))

    # AbstractDataSet protocol (the optimizers take a loader directly as their data set)
    def size(self) -> int:
        return int(self.images.shape[0])

    local_size = size

    def shuffle(self):
        return self  # the workers reshuffle every epoch themselves

    def transform(self, t):
        raise TypeError("NativeBatchLoader batches are final; apply transforms before building it")

    def close(self):
        if getattr(self, "_h", None):
            self._recycle(block=True)
            runtime_library().bigdl_loader_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
