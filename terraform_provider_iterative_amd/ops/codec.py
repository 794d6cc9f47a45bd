"""TPZ1 byte-plane checkpoint codec (format: ``csrc/common/tpz.h``).

Lossless, tile-local: every CRC tile of a packed stream becomes one self-describing blob.
Host buffers use the C++ reference (``csrc/native/hostops.cpp``); device tensors use the CDNA4
kernels (``csrc/hip/codec.hip``).  Both produce byte-identical blobs, so a stream encoded on
one side decodes on the other.

The reference has no tensor codec at all (its checkpoint is an rclone file sync,
``machine-script.sh.tpl:118-124``); this exists because the MI355X spill is PCIe-bound.
"""
from __future__ import annotations

import os
from typing import Any, Tuple

import numpy as np

from ._loader import hip, native
from .hashing import DEFAULT_TILE_BYTES, _device_view, _is_device_tensor, _stream, host_buffer

NAME = "tpz1"


def _threads() -> int:
    return min(16, os.cpu_count() or 1)


def bound(total: int, tile_bytes: int = DEFAULT_TILE_BYTES) -> int:
    """Worst-case encoded size of a ``total``-byte stream."""
    full, rest = divmod(total, tile_bytes)
    n = native()
    return full * n.tpz_bound(tile_bytes) + (n.tpz_bound(rest) if rest else 0)


def offsets(csizes: np.ndarray) -> np.ndarray:
    """Blob offsets (ntiles + 1 entries) from blob sizes."""
    out = np.zeros(len(csizes) + 1, np.uint64)
    np.cumsum(np.asarray(csizes, np.uint64), out=out[1:])
    return out


def encode(data: Any, tile_bytes: int = DEFAULT_TILE_BYTES) -> Tuple[Any, Any]:
    """Encode a buffer (length multiple of 16) -> (blob stream, per-tile sizes).

    Device tensors give device outputs (uint8 tensor trimmed to the encoded length, int32
    sizes); host buffers give numpy arrays.
    """
    if _is_device_tensor(data):
        import torch

        ptr, nbytes = _device_view(data)
        _check(nbytes, tile_bytes)
        ntiles = -(-nbytes // tile_bytes)
        out = torch.empty(bound(nbytes, tile_bytes), dtype=torch.uint8, device=data.device)
        # analyze -> encode scratch: plane headers, HUF code lengths and substream sizes
        meta = torch.empty(native().tpz_meta_bytes(max(ntiles, 1)), dtype=torch.uint8,
                           device=data.device)
        csize = torch.empty(max(ntiles, 1), dtype=torch.int32, device=data.device)
        lib = hip()
        lib.check(lib.tpi_tpz_encode_device(ptr, nbytes, tile_bytes, meta.data_ptr(),
                                            csize.data_ptr(), out.data_ptr(), _stream(data)),
                  "tpz encode")
        csize = csize[:ntiles]
        used = int(csize.to(torch.int64).sum().item()) if ntiles else 0
        return out[:used], csize
    addr, nbytes, _keep = host_buffer(data)
    _check(nbytes, tile_bytes)
    ntiles = -(-nbytes // tile_bytes)
    out = np.empty(bound(nbytes, tile_bytes), np.uint8)
    csizes = np.zeros(ntiles, np.uint32)
    used = native().tpz_encode_ptr(addr, nbytes, tile_bytes, out.ctypes.data,
                                   csizes.ctypes.data, _threads())
    return out[:used], csizes


def decode(blobs: Any, csizes: Any, total: int,
           tile_bytes: int = DEFAULT_TILE_BYTES) -> Tuple[Any, int]:
    """Decode -> (raw stream, first malformed tile or -1).

    On the device a malformed blob decodes as zeros (the tile CRC catches it); the host path
    reports the first malformed tile directly.
    """
    _check(total, tile_bytes)
    if _is_device_tensor(blobs):
        import torch

        sizes = csizes.to("cpu").numpy().astype(np.uint64) if hasattr(csizes, "to") else \
            np.asarray(csizes, np.uint64)
        coff = torch.from_numpy(offsets(sizes).view(np.int64)).to(blobs.device)
        out = torch.empty(total, dtype=torch.uint8, device=blobs.device)
        lib = hip()
        lib.check(lib.tpi_tpz_decode_device(blobs.data_ptr(), coff.data_ptr(), total, tile_bytes,
                                            out.data_ptr(), _stream(blobs)), "tpz decode")
        torch.cuda.current_stream(blobs.device).synchronize()  # keep coff alive until done
        return out, -1
    addr, nbytes, _keep = host_buffer(blobs)
    sizes = np.ascontiguousarray(csizes, np.uint32)
    if int(sizes.astype(np.uint64).sum()) > nbytes:
        raise ValueError("blob sizes exceed the encoded buffer")
    out = np.empty(total, np.uint8)
    first = native().tpz_decode_ptr(addr, sizes.ctypes.data, total, tile_bytes,
                                    out.ctypes.data, _threads())
    return out, int(first)


def _check(nbytes: int, tile_bytes: int) -> None:
    if nbytes % 16:
        raise ValueError("codec streams are multiples of 16 bytes")
    if tile_bytes <= 0 or tile_bytes % 4096:
        raise ValueError("tile_bytes must be a positive multiple of 4096")
