"""The ctypes side of the HBM workdir (:mod:`.stage`): zero-copy torch views of device memory
through DLPack (kDLROCM), and ``tpi_loader`` (files <-> image bytes through a NUMA-local pinned
ring), used by the stager binary's Python twin, ranks, benches and tests."""
from __future__ import annotations

import ctypes
import os
from typing import Dict, List


class _DLDevice(ctypes.Structure):
    _fields_ = [("device_type", ctypes.c_int32), ("device_id", ctypes.c_int32)]


class _DLDataType(ctypes.Structure):
    _fields_ = [("code", ctypes.c_uint8), ("bits", ctypes.c_uint8), ("lanes", ctypes.c_uint16)]


class _DLTensor(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("device", _DLDevice), ("ndim", ctypes.c_int32),
                ("dtype", _DLDataType), ("shape", ctypes.POINTER(ctypes.c_int64)),
                ("strides", ctypes.POINTER(ctypes.c_int64)), ("byte_offset", ctypes.c_uint64)]


class _DLManagedTensor(ctypes.Structure):
    _fields_ = [("dl_tensor", _DLTensor), ("manager_ctx", ctypes.c_void_p),
                ("deleter", ctypes.c_void_p)]


_KDL_ROCM = 10
_KEEP: List[object] = []  # DLPack structs of live mappings (the mapping outlives the tensor)


def _device_tensor(ptr: int, nbytes: int, device: int):
    """A 1-D uint8 torch tensor over ``nbytes`` of device memory at ``ptr`` (no copy),
    through a DLPack capsule (kDLROCM)."""
    import torch
    import torch.utils.dlpack

    shape = (ctypes.c_int64 * 1)(nbytes)
    mt = _DLManagedTensor()
    mt.dl_tensor.data = ptr
    mt.dl_tensor.device = _DLDevice(_KDL_ROCM, device)
    mt.dl_tensor.ndim = 1
    mt.dl_tensor.dtype = _DLDataType(1, 8, 1)  # kDLUInt, 8 bits
    mt.dl_tensor.shape = shape
    mt.dl_tensor.strides = None
    mt.dl_tensor.byte_offset = 0
    mt.manager_ctx = None
    mt.deleter = None
    _KEEP.append((mt, shape))
    capsule_new = ctypes.pythonapi.PyCapsule_New
    capsule_new.restype = ctypes.py_object
    capsule_new.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p]
    capsule = capsule_new(ctypes.addressof(mt), b"dltensor", None)
    return torch.utils.dlpack.from_dlpack(capsule)


# ---- native loader (used by the stager binary; exposed for ranks, benches and tests) ----------

class _File(ctypes.Structure):
    _fields_ = [("path", ctypes.c_char_p), ("offset", ctypes.c_uint64),
                ("size", ctypes.c_uint64)]


class _Stats(ctypes.Structure):
    _fields_ = [("pack_ms", ctypes.c_double), ("copy_ms", ctypes.c_double),
                ("bytes", ctypes.c_uint64), ("chunks", ctypes.c_uint64)]


class Loader:
    """``tpi_loader``: files <-> image bytes.  ``device >= 0``: the image is device memory,
    filled through a NUMA-local pinned ring (pread workers overlap the H2D copies);
    ``device = -1``: a host image."""

    def __init__(self, device: int = -1, chunk_bytes: int = 64 << 20, nbuf: int = 4,
                 threads: int = 16, numa_node: int = -1):
        from ..ops import hip

        self.lib = hip()
        self.handle = self.lib.tpi_loader_create(device, chunk_bytes, nbuf, threads, numa_node)
        if not self.handle:
            raise RuntimeError("loader: %s" % self.lib.error())

    @staticmethod
    def _files(root: str, files):
        paths = [os.path.join(root, f[0]).encode() for f in files]
        arr = (_File * max(1, len(files)))()
        for i, (f, p) in enumerate(zip(files, paths)):
            arr[i] = _File(p, int(f[1]), int(f[2]))
        return arr, paths

    def load(self, root: str, files, lo: int, hi: int, dst: int) -> Dict[str, float]:
        """Fill image bytes ``[lo, hi)`` of the image at address ``dst``."""
        arr, _keep = self._files(root, files)
        st = _Stats()
        self.lib.check(self.lib.tpi_loader_load(self.handle, arr, len(files), lo, hi,
                                                ctypes.c_void_p(dst), ctypes.byref(st)),
                       "tpi_loader_load")
        return {"ms": st.copy_ms, "read_ms": st.pack_ms, "bytes": int(st.bytes),
                "chunks": int(st.chunks)}

    def store(self, root: str, files, ranges, src: int) -> Dict[str, float]:
        """Write image ``ranges`` (``[(lo, hi), ...]``) of the image at ``src`` to the files."""
        arr, _keep = self._files(root, files)
        flat = (ctypes.c_uint64 * max(1, 2 * len(ranges)))(*[x for r in ranges for x in r])
        st = _Stats()
        self.lib.check(self.lib.tpi_loader_store(self.handle, arr, len(files), flat, len(ranges),
                                                 ctypes.c_void_p(src), ctypes.byref(st)),
                       "tpi_loader_store")
        return {"ms": st.copy_ms, "bytes": int(st.bytes)}

    def close(self) -> None:
        if self.handle:
            self.lib.tpi_loader_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
