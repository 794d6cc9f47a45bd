"""CRC32C tiles and striped-XXH64 shard hashes on host buffers or device tensors."""
from __future__ import annotations

from typing import Any, Tuple

import numpy as np

from ._loader import hip, native

DEFAULT_TILE_BYTES = 1 << 20
DEFAULT_SHARD_BYTES = 1 << 20


def _is_device_tensor(data: Any) -> bool:
    try:
        import torch
    except ImportError:  # pragma: no cover
        return False
    return isinstance(data, torch.Tensor) and data.device.type == "cuda"


def host_buffer(data: Any) -> Tuple[int, int, Any]:
    """(address, nbytes, keepalive) of a contiguous host buffer-like object."""
    try:
        import torch

        if isinstance(data, torch.Tensor):
            if data.device.type != "cpu":
                raise TypeError("device tensor passed where a host buffer is required")
            if not data.is_contiguous():
                data = data.contiguous()
            return data.data_ptr(), data.numel() * data.element_size(), data
    except ImportError:  # pragma: no cover
        pass
    if isinstance(data, np.ndarray):
        arr = np.ascontiguousarray(data)
        return arr.ctypes.data, arr.nbytes, arr
    mv = memoryview(data)
    if not mv.contiguous:
        mv = memoryview(bytes(mv))
    arr = np.frombuffer(mv, dtype=np.uint8) if mv.nbytes else np.zeros(0, np.uint8)
    return arr.ctypes.data, mv.nbytes, (arr, mv)


def _device_view(t):
    if not t.is_contiguous():
        raise ValueError("device buffer must be contiguous")
    return t.data_ptr(), t.numel() * t.element_size()


def _stream(t) -> int:
    import torch

    return torch.cuda.current_stream(t.device).cuda_stream


def crc32c(data: Any, crc: int = 0) -> int:
    """Standard CRC32C (Castagnoli) of a host buffer, optionally continuing ``crc``."""
    addr, nbytes, _keep = host_buffer(data)
    return native().crc32c_ptr(addr, nbytes, crc)


def crc32c_combine(crc_a: int, crc_b: int, len_b: int) -> int:
    return native().crc32c_combine(crc_a, crc_b, len_b)


def crc32c_tiles(data: Any, tile_bytes: int = DEFAULT_TILE_BYTES, threads: int = 8):
    """CRC32C of every ``tile_bytes`` tile.  Device tensors -> int32 device tensor (bit
    pattern of the uint32 CRCs), host buffers -> ``np.uint32`` array."""
    if _is_device_tensor(data):
        import torch

        ptr, nbytes = _device_view(data)
        ntiles = (nbytes + tile_bytes - 1) // tile_bytes
        out = torch.empty(max(ntiles, 1), dtype=torch.int32, device=data.device)[:ntiles]
        lib = hip()
        with torch.cuda.device(data.device):
            lib.check(lib.tpi_crc32c_tiles(ptr, nbytes, tile_bytes, out.data_ptr(),
                                           _stream(data)), "crc32c_tiles")
        return out
    addr, nbytes, _keep = host_buffer(data)
    out = np.zeros((nbytes + tile_bytes - 1) // tile_bytes, dtype=np.uint32)
    native().crc32c_tiles_ptr(addr, nbytes, tile_bytes, out.ctypes.data, threads)
    return out


def shard_hash(data: Any, shard_bytes: int = DEFAULT_SHARD_BYTES, seed: int = 0,
               threads: int = 8):
    """Striped XXH64 digest of every shard (format: ``csrc/common/xxh64.h``).

    Device tensors -> int64 device tensor, host buffers -> ``np.uint64`` array.
    """
    if shard_bytes <= 0 or shard_bytes % 32:
        raise ValueError("shard_bytes must be a positive multiple of 32")
    if _is_device_tensor(data):
        import torch

        ptr, nbytes = _device_view(data)
        nshards = (nbytes + shard_bytes - 1) // shard_bytes
        out = torch.empty(max(nshards, 1), dtype=torch.int64, device=data.device)[:nshards]
        lib = hip()
        with torch.cuda.device(data.device):
            lib.check(lib.tpi_shard_hash(ptr, nbytes, shard_bytes, seed & (2**64 - 1),
                                         out.data_ptr(), _stream(data)), "shard_hash")
        return out
    addr, nbytes, _keep = host_buffer(data)
    out = np.zeros((nbytes + shard_bytes - 1) // shard_bytes, dtype=np.uint64)
    native().shard_hash_ptr(addr, nbytes, shard_bytes, seed & (2**64 - 1), out.ctypes.data,
                            threads)
    return out


def dirty_shards(previous, current) -> np.ndarray:
    """Indices of shards whose digest changed (new shards count as dirty)."""
    cur = current.cpu().numpy() if hasattr(current, "cpu") else np.asarray(current)
    if previous is None:
        return np.arange(len(cur))
    prev = previous.cpu().numpy() if hasattr(previous, "cpu") else np.asarray(previous)
    cur = cur.view(np.uint64)
    prev = prev.view(np.uint64)
    n = min(len(prev), len(cur))
    changed = np.nonzero(prev[:n] != cur[:n])[0]
    if len(cur) > n:
        changed = np.concatenate([changed, np.arange(n, len(cur))])
    return changed
