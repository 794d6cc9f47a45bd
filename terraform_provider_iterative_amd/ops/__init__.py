"""Data-plane operators: CRC32C tiles, striped XXH64 shard hashes, tensor pack/unpack.

Every operator dispatches on where the data lives: device tensors go to the hand-written
CDNA4 kernels in ``libtpi_hip.so`` (``csrc/hip/kernels.hip``); host tensors / buffers to the
C++ implementations in ``_tpi_native`` (``csrc/native/hostops.cpp``), which define the same
formats bit for bit.
"""
from ._loader import HipError, gpu_visible, hip, native
from .hashing import (DEFAULT_SHARD_BYTES, DEFAULT_TILE_BYTES, crc32c, crc32c_combine,
                      crc32c_tiles, dirty_shards, shard_hash)
from .packing import SEG_DTYPE, PackPlan, TensorEntry, pack, unpack

__all__ = [
    "HipError", "gpu_visible", "hip", "native", "DEFAULT_SHARD_BYTES", "DEFAULT_TILE_BYTES",
    "crc32c", "crc32c_combine", "crc32c_tiles", "dirty_shards", "shard_hash", "SEG_DTYPE",
    "PackPlan", "TensorEntry", "pack", "unpack",
]
