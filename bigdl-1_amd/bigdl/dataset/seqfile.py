"""Hadoop SequenceFile image datasets (``DataSet.SeqFileFolder``, ``DL/dataset/DataSet.scala:486-640``;
writer ``BGRImgToLocalSeqFile``, ``DL/dataset/image/BGRImgToLocalSeqFile.scala``; pyspark
``SeqFileFolder.files_to_image_frame``).

The reference's ImageNet pipeline stores images in Hadoop SequenceFiles: key = ``Text`` holding
``"<label>"`` or ``"<name>\\n<label>"``, value = ``Text`` holding ``int32 width, int32 height``
(big-endian) followed by the raw BGR bytes.  This module reads and writes that container format
directly (SequenceFile version 6, uncompressed records, 16-byte sync markers; ``Text`` and
``BytesWritable`` keys/values) — no Hadoop/JVM is involved.
"""
from __future__ import annotations

import io
import os
import struct
from typing import Iterator, List, Optional, Tuple

import numpy as np

TEXT = "org.apache.hadoop.io.Text"
BYTES = "org.apache.hadoop.io.BytesWritable"


# ---------------------------------------------------------------------------------- Hadoop varints
def write_vlong(out: io.BufferedIOBase, i: int):
    """``WritableUtils.writeVLong``."""
    if -112 <= i <= 127:
        out.write(struct.pack(">b", i))
        return
    ln = -112
    if i < 0:
        i = ~i
        ln = -120
    tmp = i
    while tmp != 0:
        tmp >>= 8
        ln -= 1
    out.write(struct.pack(">b", ln))
    n = -(ln + 120) if ln < -120 else -(ln + 112)
    for idx in range(n, 0, -1):
        out.write(bytes([(i >> ((idx - 1) * 8)) & 0xFF]))


def read_vlong(buf: io.BufferedIOBase) -> int:
    first = struct.unpack(">b", buf.read(1))[0]
    if first >= -112:
        return first
    neg = first < -120
    n = (-119 - first) if neg else (-111 - first)
    v = 0
    for _ in range(n - 1):
        v = (v << 8) | buf.read(1)[0]
    return ~v if neg else v


def _write_text(out, s: bytes):
    write_vlong(out, len(s))
    out.write(s)


def _read_text(buf) -> bytes:
    return buf.read(read_vlong(buf))


# ---------------------------------------------------------------------------------- container
class SequenceFileWriter:
    def __init__(self, path: str, key_class: str = TEXT, value_class: str = TEXT, sync_interval: int = 2000):
        self.f = open(path, "wb")
        self.key_class, self.value_class = key_class, value_class
        self.sync = os.urandom(16)
        self.sync_interval = sync_interval
        self.f.write(b"SEQ" + bytes([6]))
        _write_text(self.f, key_class.encode())
        _write_text(self.f, value_class.encode())
        self.f.write(b"\x00\x00")          # not compressed, not block-compressed
        self.f.write(struct.pack(">i", 0))  # metadata: no entries
        self.f.write(self.sync)
        self._last_sync = self.f.tell()

    def _ser(self, cls, data: bytes) -> bytes:
        b = io.BytesIO()
        if cls == TEXT:
            _write_text(b, data)
        elif cls == BYTES:
            b.write(struct.pack(">i", len(data)) + data)
        else:
            raise ValueError(f"unsupported writable {cls}")
        return b.getvalue()

    def append(self, key: bytes, value: bytes):
        if self.f.tell() - self._last_sync >= self.sync_interval:
            self.f.write(struct.pack(">i", -1) + self.sync)
            self._last_sync = self.f.tell()
        k, v = self._ser(self.key_class, key), self._ser(self.value_class, value)
        self.f.write(struct.pack(">ii", len(k) + len(v), len(k)) + k + v)

    def close(self):
        self.f.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def read_sequence_file(path: str) -> Iterator[Tuple[bytes, bytes]]:
    """(key, value) payloads of an uncompressed SequenceFile with Text / BytesWritable records."""
    with open(path, "rb") as f:
        data = f.read()
    buf = io.BytesIO(data)
    if buf.read(3) != b"SEQ":
        raise ValueError(f"{path}: not a SequenceFile")
    version = buf.read(1)[0]
    key_cls = _read_text(buf).decode()
    val_cls = _read_text(buf).decode()
    compressed, block = buf.read(1)[0], buf.read(1)[0]
    if compressed or block:
        raise NotImplementedError(f"{path}: compressed SequenceFiles are not supported")
    if version >= 6:
        for _ in range(struct.unpack(">i", buf.read(4))[0]):
            _read_text(buf)
            _read_text(buf)
    sync = buf.read(16)

    def payload(cls, raw: bytes) -> bytes:
        b = io.BytesIO(raw)
        if cls == TEXT:
            return _read_text(b)
        if cls == BYTES:
            return b.read(struct.unpack(">i", b.read(4))[0])
        return raw
    while True:
        head = buf.read(4)
        if len(head) < 4:
            return
        rec_len = struct.unpack(">i", head)[0]
        if rec_len == -1:
            if buf.read(16) != sync:
                raise ValueError(f"{path}: corrupt sync marker")
            continue
        key_len = struct.unpack(">i", buf.read(4))[0]
        raw = buf.read(rec_len)
        yield payload(key_cls, raw[:key_len]), payload(val_cls, raw[key_len:])


# ---------------------------------------------------------------------------------- image datasets
def read_label(key: bytes) -> str:
    parts = key.decode().split("\n")
    return parts[0] if len(parts) == 1 else parts[1]


def read_name(key: bytes) -> str:
    parts = key.decode().split("\n")
    if len(parts) < 2:
        raise ValueError("key in seq file only contains label, no name")
    return parts[0]


def decode_bgr_record(value: bytes) -> np.ndarray:
    """``int32 width, int32 height`` + BGR bytes → uint8 [H, W, 3]."""
    w, h = struct.unpack(">ii", value[:8])
    return np.frombuffer(value[8:8 + w * h * 3], dtype=np.uint8).reshape(h, w, 3)


def encode_bgr_record(img: np.ndarray) -> bytes:
    h, w = img.shape[:2]
    return struct.pack(">ii", w, h) + np.ascontiguousarray(img, dtype=np.uint8).tobytes()


class BGRImgToLocalSeqFile:
    """Write (BGR uint8 image, label[, name]) items into ``<base>_<i>.seq`` files of ``block_size``
    records (``BGRImgToLocalSeqFile.scala``); returns the file names."""

    def __init__(self, block_size: int, base_file_name: str, has_name: bool = False):
        self.block_size, self.base, self.has_name = block_size, base_file_name, has_name

    def __call__(self, items) -> List[str]:
        files, it, idx = [], iter(items), 0
        done = False
        while not done:
            name = f"{self.base}_{idx}.seq"
            n = 0
            with SequenceFileWriter(name) as w:
                for img, label, *rest in it:
                    key = f"{rest[0]}\n{int(label)}" if (self.has_name and rest) else f"{int(label)}"
                    w.append(key.encode(), encode_bgr_record(img))
                    n += 1
                    if n >= self.block_size:
                        break
                else:
                    done = True
            if n:
                files.append(name)
            elif os.path.exists(name):
                os.remove(name)
            idx += 1
        return files


class SeqFileFolder:
    @staticmethod
    def find_files(path: str) -> List[str]:
        if os.path.isfile(path):
            return [path]
        return sorted(os.path.join(path, f) for f in os.listdir(path) if f.endswith(".seq"))

    @staticmethod
    def read(path: str, class_num: Optional[int] = None):
        """(BGR uint8 image, 1-based float label, name or None) records of every ``.seq`` file."""
        for fp in SeqFileFolder.find_files(path):
            for k, v in read_sequence_file(fp):
                label = float(read_label(k))
                if class_num is not None and not (1 <= label <= class_num):
                    raise ValueError(f"label {label} outside [1, {class_num}]")
                parts = k.decode().split("\n")
                yield decode_bgr_record(v), label, (parts[0] if len(parts) > 1 else None)

    @staticmethod
    def files_to_image_frame(url: str, sc=None, class_num: Optional[int] = None, partition_num: int = -1,
                             bigdl_type="float"):
        """ImageFrame of the seq-file images (``mat`` = BGR float image, ``label``, ``uri`` = name)."""
        from ..transform.vision.image import ImageFeature, ImageFrame
        feats = []
        for img, label, name in SeqFileFolder.read(url, class_num):
            f = ImageFeature(label=label, uri=name, image=img.astype(np.float32))
            feats.append(f)
        return ImageFrame.array(feats)

    filesToImageFrame = files_to_image_frame

    @staticmethod
    def to_arrays(url: str, class_num: Optional[int] = None):
        """(uint8 [N, H, W, 3], float labels [N]) for fixed-size images — the input of
        :class:`bigdl.runtime.NativeBatchLoader`."""
        imgs, labels = [], []
        for img, label, _ in SeqFileFolder.read(url, class_num):
            imgs.append(img)
            labels.append(label)
        return np.stack(imgs), np.asarray(labels, dtype=np.float32)
