"""Plain-Python reference implementations the native/HIP data plane is checked against."""
from __future__ import annotations

import struct

import numpy as np
import xxhash

POLY = 0x82F63B78
_TABLE = []
for _v in range(256):
    _c = _v
    for _ in range(8):
        _c = (_c >> 1) ^ POLY if _c & 1 else _c >> 1
    _TABLE.append(_c)


def crc32c_py(data: bytes, crc: int = 0) -> int:
    crc ^= 0xFFFFFFFF
    for byte in data:
        crc = (crc >> 8) ^ _TABLE[(crc ^ byte) & 0xFF]
    return crc ^ 0xFFFFFFFF


def crc32c_np(data: bytes) -> int:
    """Byte-serial CRC32C in numpy-free Python but tolerable for a few hundred KB."""
    return crc32c_py(data)


def shard_hash_py(data: bytes, shard_bytes: int = 1 << 20, seed: int = 0):
    """Striped-XXH64 shard digests (definition in csrc/common/xxh64.h)."""
    out = []
    for base in range(0, len(data), shard_bytes):
        d = data[base:base + shard_bytes]
        nstripes = (len(d) + 31) // 32
        digests = []
        for lane in range(256):
            msg = b"".join(d[32 * s:32 * s + 32] for s in range(lane, nstripes, 256))
            digests.append(xxhash.xxh64(msg, seed=seed).intdigest())
        out.append(xxhash.xxh64(struct.pack("<256Q", *digests), seed=seed).intdigest())
    return np.array(out, dtype=np.uint64)
