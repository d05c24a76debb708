"""TFRecord framing (``DL/utils/tf/TFRecordIterator.scala``, ``TFRecordWriter.scala``):
``uint64 length | uint32 masked_crc32c(length) | data | uint32 masked_crc32c(data)``."""
from __future__ import annotations

import struct
from typing import Iterator

from ...visualization.tensorboard import masked_crc32c


class TFRecordIterator:
    def __init__(self, path: str, check_crc: bool = True):
        self.path, self.check_crc = path, check_crc

    def __iter__(self) -> Iterator[bytes]:
        with open(self.path, "rb") as f:
            while True:
                head = f.read(12)
                if len(head) < 12:
                    return
                (n,) = struct.unpack("<Q", head[:8])
                if self.check_crc and struct.unpack("<I", head[8:])[0] != masked_crc32c(head[:8]):
                    raise IOError(f"{self.path}: corrupt record length")
                data = f.read(n)
                crc = f.read(4)
                if self.check_crc and struct.unpack("<I", crc)[0] != masked_crc32c(data):
                    raise IOError(f"{self.path}: corrupt record data")
                yield data


class TFRecordWriter:
    def __init__(self, path: str):
        self.f = open(path, "wb")

    def write(self, data: bytes):
        head = struct.pack("<Q", len(data))
        self.f.write(head + struct.pack("<I", masked_crc32c(head)) + data + struct.pack("<I", masked_crc32c(data)))

    def close(self):
        self.f.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
