"""TensorFlow V2 checkpoints (tensor bundles) read and written without TensorFlow.

The reference loads variables from a "bin file" that its ``export_tf_checkpoint.py`` script makes
from a TF checkpoint with TensorFlow itself (``DL/utils/tf/TensorflowLoader.scala:88,142-172``).
Here the checkpoint is read directly:

* ``<prefix>.index`` — a LevelDB-format table (data blocks of prefix-compressed key/value entries
  with a restart array, a 5-byte trailer per block, an index block of block handles, a 48-byte
  footer ending in the magic ``0xdb4775248b80fb57``).  Key ``""`` holds a ``BundleHeaderProto``;
  every other key is a tensor name whose value is a ``BundleEntryProto`` (dtype, shape, shard id,
  offset, size, crc32c).
* ``<prefix>.data-SSSSS-of-NNNNN`` — the raw little-endian tensor bytes at those offsets.

Only uncompressed blocks are supported (TF writes the bundle index uncompressed).  Protobuf
messages are decoded / encoded by hand (a few varint and length-delimited fields), so neither
TensorFlow nor its generated protos are needed.  :func:`write_checkpoint` produces the same
format (one shard), which is what the tests and :meth:`Session.saveParameters` use.
"""
from __future__ import annotations

import os
import struct
from typing import Dict, Iterator, List, Tuple

import numpy as np

MAGIC = 0xDB4775248B80FB57

# tensorflow.DataType → numpy
_DT = {1: np.float32, 2: np.float64, 3: np.int32, 4: np.uint8, 5: np.int16, 6: np.int8, 9: np.int64,
       10: np.bool_, 14: None, 17: np.uint16, 19: np.float16, 22: np.uint32, 23: np.uint64}
_DT_INV = {np.dtype(np.float32): 1, np.dtype(np.float64): 2, np.dtype(np.int32): 3, np.dtype(np.uint8): 4,
           np.dtype(np.int16): 5, np.dtype(np.int8): 6, np.dtype(np.int64): 9, np.dtype(np.bool_): 10,
           np.dtype(np.float16): 19}
_BF16 = 14


# ------------------------------------------------------------------------------------------ varints
def _varint(buf: bytes, pos: int) -> Tuple[int, int]:
    r, shift = 0, 0
    while True:
        b = buf[pos]
        pos += 1
        r |= (b & 0x7F) << shift
        if b < 0x80:
            return r, pos
        shift += 7


def _enc_varint(v: int) -> bytes:
    v &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _fields(buf: bytes) -> Iterator[Tuple[int, int, object]]:
    """(field number, wire type, value) of a protobuf message."""
    pos = 0
    while pos < len(buf):
        key, pos = _varint(buf, pos)
        fno, wt = key >> 3, key & 7
        if wt == 0:
            v, pos = _varint(buf, pos)
        elif wt == 1:
            v = struct.unpack_from("<Q", buf, pos)[0]
            pos += 8
        elif wt == 2:
            n, pos = _varint(buf, pos)
            v = buf[pos:pos + n]
            pos += n
        elif wt == 5:
            v = struct.unpack_from("<I", buf, pos)[0]
            pos += 4
        else:
            raise ValueError(f"unsupported protobuf wire type {wt}")
        yield fno, wt, v


def _parse_shape(buf: bytes) -> List[int]:
    dims = []
    for fno, _, v in _fields(buf):
        if fno == 2:  # TensorShapeProto.dim
            size = 0
            for f2, _, v2 in _fields(v):
                if f2 == 1:
                    size = v2 - (1 << 64) if v2 >= 1 << 63 else v2
            dims.append(size)
    return dims


def _parse_entry(buf: bytes) -> dict:
    e = {"dtype": 0, "shape": [], "shard_id": 0, "offset": 0, "size": 0, "crc32c": None, "slices": 0}
    for fno, _, v in _fields(buf):
        if fno == 1:
            e["dtype"] = v
        elif fno == 2:
            e["shape"] = _parse_shape(v)
        elif fno == 3:
            e["shard_id"] = v
        elif fno == 4:
            e["offset"] = v
        elif fno == 5:
            e["size"] = v
        elif fno == 6:
            e["crc32c"] = v
        elif fno == 7:
            e["slices"] += 1
    return e


def _parse_header(buf: bytes) -> dict:
    h = {"num_shards": 1, "endianness": 0}
    for fno, _, v in _fields(buf):
        if fno == 1:
            h["num_shards"] = v
        elif fno == 2:
            h["endianness"] = v
    return h


# ------------------------------------------------------------------------------------------ table
def _block(data: bytes, handle: Tuple[int, int]) -> bytes:
    off, size = handle
    blk = data[off:off + size]
    ctype = data[off + size]
    if ctype != 0:
        raise ValueError("compressed checkpoint index blocks are not supported")
    return blk


def _block_entries(blk: bytes) -> Iterator[Tuple[bytes, bytes]]:
    n_restarts = struct.unpack_from("<I", blk, len(blk) - 4)[0]
    end = len(blk) - 4 - 4 * n_restarts
    pos, key = 0, b""
    while pos < end:
        shared, pos = _varint(blk, pos)
        unshared, pos = _varint(blk, pos)
        vlen, pos = _varint(blk, pos)
        key = key[:shared] + blk[pos:pos + unshared]
        pos += unshared
        val = blk[pos:pos + vlen]
        pos += vlen
        yield key, val


def _handle(buf: bytes, pos: int = 0) -> Tuple[Tuple[int, int], int]:
    off, pos = _varint(buf, pos)
    size, pos = _varint(buf, pos)
    return (off, size), pos


def read_index(prefix: str) -> Tuple[dict, Dict[str, dict]]:
    with open(prefix + ".index", "rb") as f:
        data = f.read()
    if len(data) < 48 or struct.unpack_from("<Q", data, len(data) - 8)[0] != MAGIC:
        raise ValueError(f"{prefix}.index is not a TensorFlow checkpoint index (bad magic)")
    footer = data[-48:]
    _, pos = _handle(footer, 0)            # metaindex handle (unused)
    index_handle, _ = _handle(footer, pos)
    header, entries = {"num_shards": 1}, {}
    for _, hval in _block_entries(_block(data, index_handle)):
        bh, _ = _handle(hval)
        for k, v in _block_entries(_block(data, bh)):
            if k == b"":
                header = _parse_header(v)
            else:
                entries[k.decode()] = _parse_entry(v)
    return header, entries


def read_checkpoint(prefix: str) -> Dict[str, np.ndarray]:
    """Every (unsliced) tensor of the checkpoint ``prefix`` as numpy arrays, by variable name."""
    header, entries = read_index(prefix)
    n = int(header.get("num_shards", 1))
    shards = {}
    out = {}
    for name, e in entries.items():
        if e["slices"]:
            continue  # partitioned variables: not supported (stored as slices)
        sid = e["shard_id"]
        if sid not in shards:
            with open(f"{prefix}.data-{sid:05d}-of-{n:05d}", "rb") as f:
                shards[sid] = f.read()
        raw = shards[sid][e["offset"]:e["offset"] + e["size"]]
        shape = e["shape"]
        if e["dtype"] == _BF16:
            u = np.frombuffer(raw, dtype="<u2").astype(np.uint32) << 16
            arr = u.view(np.float32)
        elif e["dtype"] == 7:  # DT_STRING: skip (not a weight)
            continue
        else:
            dt = _DT.get(e["dtype"])
            if dt is None:
                continue
            arr = np.frombuffer(raw, dtype=np.dtype(dt).newbyteorder("<"))
        out[name] = arr.reshape(shape).copy()
    return out


# ------------------------------------------------------------------------------------------ writer
def _crc32c_table():
    t = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
        t.append(c)
    return t


_CRC_T = _crc32c_table()


def crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    for b in data:
        c = _CRC_T[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def _masked(c: int) -> int:
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def _pb_field(fno: int, wt: int, payload) -> bytes:
    key = _enc_varint((fno << 3) | wt)
    if wt == 0:
        return key + _enc_varint(payload)
    if wt == 2:
        return key + _enc_varint(len(payload)) + payload
    if wt == 5:
        return key + struct.pack("<I", payload)
    raise ValueError(wt)


def _entry_pb(dtype: int, shape, offset: int, size: int, crc: int) -> bytes:
    shp = b"".join(_pb_field(2, 2, _pb_field(1, 0, int(d))) for d in shape)
    out = _pb_field(1, 0, dtype) + _pb_field(2, 2, shp)
    if offset:
        out += _pb_field(4, 0, offset)
    out += _pb_field(5, 0, size) + _pb_field(6, 5, crc)
    return out


def _build_block(items: List[Tuple[bytes, bytes]]) -> bytes:
    body = bytearray()
    restarts = []
    for k, v in items:  # restart interval 1: every key stored whole
        restarts.append(len(body))
        body += _enc_varint(0) + _enc_varint(len(k)) + _enc_varint(len(v)) + k + v
    for r in restarts or [0]:
        body += struct.pack("<I", r)
    body += struct.pack("<I", len(restarts) or 1)
    return bytes(body)


def write_checkpoint(prefix: str, tensors: Dict[str, np.ndarray]) -> None:
    """One-shard TF V2 checkpoint (``prefix.index`` + ``prefix.data-00000-of-00001``)."""
    os.makedirs(os.path.dirname(os.path.abspath(prefix)), exist_ok=True)
    data = bytearray()
    items = [(b"", _pb_field(1, 0, 1) + _pb_field(3, 2, _pb_field(1, 0, 1)))]  # header: 1 shard, version 1
    for name in sorted(tensors):
        a = np.require(np.asarray(tensors[name]), requirements="C")  # (ascontiguousarray makes 0-d 1-d)
        if a.dtype not in _DT_INV:
            a = a.astype(np.float32)
        raw = a.astype(a.dtype.newbyteorder("<")).tobytes()
        items.append((name.encode(), _entry_pb(_DT_INV[a.dtype], a.shape, len(data), len(raw), _masked(crc32c(raw)))))
        data += raw
    with open(prefix + ".data-00000-of-00001", "wb") as f:
        f.write(bytes(data))
    out = bytearray()

    def put_block(blk: bytes) -> Tuple[int, int]:
        off = len(out)
        out.extend(blk)
        trailer = b"\x00"
        out.extend(trailer + struct.pack("<I", _masked(crc32c(blk + trailer))))
        return off, len(blk)

    data_h = put_block(_build_block(items))
    meta_h = put_block(_build_block([]))
    last_key = items[-1][0]
    index_h = put_block(_build_block([(last_key, _enc_varint(data_h[0]) + _enc_varint(data_h[1]))]))
    footer = _enc_varint(meta_h[0]) + _enc_varint(meta_h[1]) + _enc_varint(index_h[0]) + _enc_varint(index_h[1])
    footer += b"\x00" * (40 - len(footer)) + struct.pack("<Q", MAGIC)
    out.extend(footer)
    with open(prefix + ".index", "wb") as f:
        f.write(bytes(out))


def is_checkpoint(prefix: str) -> bool:
    return os.path.exists(prefix + ".index")


__all__ = ["read_checkpoint", "write_checkpoint", "read_index", "is_checkpoint", "crc32c"]
