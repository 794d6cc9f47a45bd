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


def _a16(x: int) -> int:
    return (x + 15) & ~15


def _huf_plane_py(blob: bytes, off: int, n: int, ngroups: int, m: int, nesc: int,
                  dictionary: np.ndarray) -> np.ndarray:
    """HUF plane: canonical Huffman over dictionary + escape (symbol m, then 8 raw bits),
    LSB-first bits, substream s = groups s, s+256, ... (spec: csrc/common/tpz.h)."""
    streams = min(256, ngroups)
    lens = list(blob[off:off + 16])
    ends = [int(x) for x in np.frombuffer(blob, np.uint32, streams, off + 16)]
    base = off + 16 + _a16(4 * streams)
    table = {}  # (length, MSB-first code) -> symbol
    code = 0
    for length in range(1, 12):
        for s in range(m + 1):
            if lens[s] == length:
                table[(length, code)] = s
                code += 1
        code <<= 1
    vals = np.zeros(n, np.uint8)
    start = 0
    for s in range(streams):
        raw = np.frombuffer(blob, np.uint8, 4 * (ends[s] - start), base + 4 * start)
        bits = np.unpackbits(raw, bitorder="little").tolist() + [0] * 32
        pos = 0
        for g in range(s, ngroups, 256):
            for i in range(g * 32, min(g * 32 + 32, n)):
                c, length = 0, 0
                while (length, c) not in table:
                    c = (c << 1) | bits[pos]
                    pos += 1
                    length += 1
                    assert length <= 11, "no code"
                sym = table[(length, c)]
                if sym == m:
                    vals[i] = sum(bits[pos + b] << b for b in range(8))
                    pos += 8
                else:
                    vals[i] = dictionary[sym]
        assert pos <= 32 * (ends[s] - start)
        start = ends[s]
    assert start == nesc
    return vals


def tpz_decode_tile_py(blob: bytes, length: int) -> np.ndarray:
    """Independent numpy decoder of one TPZ1 tile blob (spec: csrc/common/tpz.h)."""
    n = length // 4
    ngroups = (n + 31) // 32
    out = np.zeros(length, np.uint8)
    off = 96
    for p in range(4):
        k, m, _, _, nesc = struct.unpack_from("<BBBBI", blob, 24 * p)
        dictionary = np.frombuffer(blob, np.uint8, 16, 24 * p + 8)
        if k == 8:  # raw plane
            out[p::4] = np.frombuffer(blob, np.uint8, n, off)
            off += ngroups * 32
            continue
        if k == 9:  # Huffman plane
            out[p::4] = _huf_plane_py(blob, off, n, ngroups, m, nesc, dictionary)
            off += 16 + _a16(4 * min(256, ngroups)) + _a16(4 * nesc)
            continue
        if k == 0:  # constant plane
            out[p::4] = dictionary[0]
            continue
        esc_code = (1 << k) - 1
        words = np.frombuffer(blob, np.uint32, ngroups * k, off)
        bits = np.unpackbits(words.view(np.uint8), bitorder="little")
        codes = bits[:ngroups * 32 * k].reshape(-1, k).astype(np.uint32)
        codes = (codes << np.arange(k, dtype=np.uint32)).sum(axis=1)[:n]
        escapes = np.frombuffer(blob, np.uint8, nesc, off + _a16(ngroups * 4 * k))
        vals = dictionary[np.minimum(codes, m - 1)].copy()
        is_esc = codes == esc_code
        assert int(is_esc.sum()) == nesc
        vals[is_esc] = escapes
        out[p::4] = vals
        off += _a16(ngroups * 4 * k) + _a16(nesc)
    return out
