"""``HashFunc`` (``DL/utils/HashFunc.scala``): ``stringHashBucket32`` = Scala's
``MurmurHash3.stringHash`` (UTF-16 code units mixed two at a time, seed ``0xf7ca7fd2``) modulo the
bucket count, made non-negative — so feature-column hashing buckets strings exactly as the
reference does."""
from __future__ import annotations

_M = 0xFFFFFFFF
STRING_SEED = 0xF7CA7FD2


def _rotl(x: int, r: int) -> int:
    return ((x << r) | (x >> (32 - r))) & _M


def _mix_last(h: int, k: int) -> int:
    k = (k * 0xCC9E2D51) & _M
    k = _rotl(k, 15)
    k = (k * 0x1B873593) & _M
    return h ^ k


def _mix(h: int, k: int) -> int:
    h = _mix_last(h, k)
    h = _rotl(h, 13)
    return (h * 5 + 0xE6546B64) & _M


def _avalanche(h: int) -> int:
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & _M
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & _M
    h ^= h >> 16
    return h


def _signed(x: int) -> int:
    return x - (1 << 32) if x & 0x80000000 else x


def string_hash(s: str, seed: int = STRING_SEED) -> int:
    """``scala.util.hashing.MurmurHash3.stringHash`` (signed 32-bit result)."""
    units = s.encode("utf-16-le")
    cu = [units[i] | (units[i + 1] << 8) for i in range(0, len(units), 2)]
    h = seed & _M
    i = 0
    while i + 1 < len(cu):
        h = _mix(h, ((cu[i] << 16) + cu[i + 1]) & _M)
        i += 2
    if i < len(cu):
        h = _mix_last(h, cu[i])
    return _signed(_avalanche(h ^ len(cu)))


def stringHashBucket32(s: str, buckets: int) -> int:
    v = string_hash(s)
    r = int(v - buckets * int(v / buckets))  # Java/Scala % (truncated toward zero)
    return r + buckets if r < 0 else r


string_hash_bucket32 = stringHashBucket32


class HashFunc:
    stringHashBucket32 = staticmethod(stringHashBucket32)
