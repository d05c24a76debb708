"""TensorBoard event files: TFRecord framing with masked CRC32C, an async writer and a reader.

Reference: ``DL/visualization/tensorboard/{FileWriter,EventWriter,RecordWriter,FileReader}.scala``
and ``DL/utils/Crc32.scala``.  The ``Event`` / ``Summary`` / ``HistogramProto`` messages are
re-declared with TensorFlow's field numbers (``tensorflow/core/util/event.proto``,
``framework/summary.proto``) so the files open in stock TensorBoard.

Layout of one record: ``uint64 len | uint32 masked_crc(len) | data | uint32 masked_crc(data)``.
The writer runs one daemon thread draining a queue and flushing every ``flush_secs`` (the
reference's EventWriter thread, flushMillis = 1000).
"""
from __future__ import annotations

import os
import queue
import socket
import struct
import threading
import time
from typing import Iterator, List, Tuple

from ..serialization.proto_builder import F, Msg, build

# ---------------------------------------------------------------------------------------- CRC32C
_POLY = 0x82F63B78


def _make_table():
    t = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ _POLY if c & 1 else c >> 1
        t.append(c)
    return t


_TABLE = _make_table()


def crc32c(data: bytes) -> int:
    crc = 0xFFFFFFFF
    tbl = _TABLE
    for b in data:
        crc = tbl[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def masked_crc32c(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


# ---------------------------------------------------------------------------------------- protos
_PKG = "tensorflow"
_HISTO = Msg("HistogramProto", [
    F("min", 1, "double"), F("max", 2, "double"), F("num", 3, "double"), F("sum", 4, "double"),
    F("sum_squares", 5, "double"), F("bucket_limit", 6, "double", "repeated", packed=True),
    F("bucket", 7, "double", "repeated", packed=True)])
_SUMMARY = Msg("Summary", [F("value", 1, "msg", "repeated", type_name=".tensorflow.Summary.Value")], nested=[
    Msg("Value", [F("node_name", 7, "string"), F("tag", 1, "string"),
                  F("simple_value", 2, "float", oneof="value"),
                  F("obsolete_old_style_histogram", 3, "bytes", oneof="value"),
                  F("histo", 5, "msg", type_name=".tensorflow.HistogramProto", oneof="value")])])
_EVENT = Msg("Event", [
    F("wall_time", 1, "double"), F("step", 2, "int64"),
    F("file_version", 3, "string", oneof="what"), F("graph_def", 4, "bytes", oneof="what"),
    F("summary", 5, "msg", type_name=".tensorflow.Summary", oneof="what")])

_pool, _classes, _ = build("bigdl_tf_event.proto", _PKG, [_HISTO, _SUMMARY, _EVENT], syntax="proto3")
Event = _classes["tensorflow.Event"]
Summary = _classes["tensorflow.Summary"]
HistogramProto = _classes["tensorflow.HistogramProto"]


# ---------------------------------------------------------------------------------------- records
def encode_record(data: bytes) -> bytes:
    header = struct.pack("<Q", len(data))
    return header + struct.pack("<I", masked_crc32c(header)) + data + struct.pack("<I", masked_crc32c(data))


def read_records(path: str, check_crc: bool = True) -> Iterator[bytes]:
    with open(path, "rb") as f:
        while True:
            header = f.read(8)
            if len(header) < 8:
                return
            (n,) = struct.unpack("<Q", header)
            (hcrc,) = struct.unpack("<I", f.read(4))
            data = f.read(n)
            tail = f.read(4)
            if len(data) < n or len(tail) < 4:
                return  # truncated trailing record (writer still running)
            if check_crc:
                if hcrc != masked_crc32c(header) or struct.unpack("<I", tail)[0] != masked_crc32c(data):
                    raise IOError(f"corrupt TFRecord in {path}")
            yield data


class RecordWriter:
    """``RecordWriter.scala``: appends framed records to one file."""

    def __init__(self, path: str):
        self._f = open(path, "ab")

    def write(self, data: bytes):
        self._f.write(encode_record(data))

    def flush(self):
        self._f.flush()

    def close(self):
        self._f.close()


class EventWriter(threading.Thread):
    """Drains a queue of Event messages into ``events.out.tfevents.<ts>.<host>`` (EventWriter.scala)."""

    def __init__(self, log_dir: str, flush_secs: float = 1.0):
        super().__init__(daemon=True)
        os.makedirs(log_dir, exist_ok=True)
        fname = f"events.out.tfevents.{int(time.time()):010d}.{socket.gethostname()}"
        self.path = os.path.join(log_dir, fname)
        self._w = RecordWriter(self.path)
        self._q: "queue.Queue" = queue.Queue()
        self._flush_secs = flush_secs
        self._closed = False
        self._lock = threading.Lock()
        ev = Event(wall_time=time.time(), file_version="brain.Event:2")
        self._w.write(ev.SerializeToString())
        self._w.flush()

    def add(self, ev):
        self._q.put(ev)

    def run(self):
        last = time.time()
        while True:
            try:
                ev = self._q.get(timeout=self._flush_secs)
            except queue.Empty:
                ev = None
            if ev is _STOP:
                self._q.task_done()
                break
            if ev is not None:
                with self._lock:
                    self._w.write(ev.SerializeToString())
                self._q.task_done()
            if time.time() - last >= self._flush_secs:
                self._w.flush()
                last = time.time()
        self._w.flush()

    def close(self):
        if not self._closed:
            self._closed = True
            self._q.put(_STOP)
            self.join(timeout=10)
            self._w.close()


_STOP = object()


class FileWriter:
    """``FileWriter.scala``: ``addSummary(summary, step)`` / ``addEvent`` / ``flush`` / ``close``."""

    def __init__(self, log_dir: str, flush_secs: float = 1.0):
        self.log_dir = log_dir
        self._ew = EventWriter(log_dir, flush_secs)
        self._ew.start()

    def add_summary(self, summary, step: int):
        self._ew.add(Event(wall_time=time.time(), step=int(step), summary=summary))
        return self

    addSummary = add_summary

    def add_event(self, ev):
        self._ew.add(ev)
        return self

    def flush(self):
        # synchronous: wait until every queued event has been written
        self._ew._q.join()
        with self._ew._lock:
            self._ew._w.flush()

    def close(self):
        self._ew.close()


class FileReader:
    """``FileReader.scala``: list event files and read one scalar tag back."""

    @staticmethod
    def list_files(folder: str) -> List[str]:
        if not os.path.isdir(folder):
            return []
        return sorted(os.path.join(folder, f) for f in os.listdir(folder) if "tfevents" in f)

    @staticmethod
    def read_scalar(folder: str, tag: str) -> List[Tuple[int, float, float]]:
        out = []
        for path in FileReader.list_files(folder):
            for rec in read_records(path):
                ev = Event()
                ev.ParseFromString(rec)
                if ev.WhichOneof("what") != "summary":
                    continue
                for v in ev.summary.value:
                    if v.tag == tag and v.WhichOneof("value") == "simple_value":
                        out.append((int(ev.step), float(v.simple_value), float(ev.wall_time)))
        out.sort(key=lambda r: r[0])
        return out

    readScalar = read_scalar
