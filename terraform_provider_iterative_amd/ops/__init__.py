"""Data-plane operators: CRC32C tiles, striped XXH64 shard hashes, tensor pack/unpack.

Every operator dispatches on where the data lives: device tensors go to the hand-written
CDNA4 kernels in ``libtpi_hip.so`` (``csrc/hip/kernels.hip``); host tensors / buffers to the
C++ implementations in ``_tpi_native`` (``csrc/native/hostops.cpp``), which define the same
formats bit for bit.

Attributes are resolved lazily so control-plane tools (``leo``/``tpi``) that only need the
native loader do not pay for importing numpy/torch.
"""
from ._loader import HipError, gpu_visible, hip, native

_LAZY = {
    "DEFAULT_SHARD_BYTES": "hashing", "DEFAULT_TILE_BYTES": "hashing", "crc32c": "hashing",
    "crc32c_combine": "hashing", "crc32c_tiles": "hashing", "dirty_shards": "hashing",
    "shard_hash": "hashing", "SEG_DTYPE": "packing", "PackPlan": "packing",
    "TensorEntry": "packing", "pack": "packing", "unpack": "packing", "codec": None,
}

__all__ = ["HipError", "gpu_visible", "hip", "native"] + sorted(_LAZY)


def __getattr__(name):
    module = _LAZY.get(name)
    import importlib

    if name not in _LAZY:
        raise AttributeError(name)
    if module is None:  # a submodule
        value = importlib.import_module("." + name, __name__)
    else:
        value = getattr(importlib.import_module("." + module, __name__), name)
    globals()[name] = value
    return value
