"""Loading of the in-tree native libraries.

``native()`` returns the pybind11 host module; ``hip()`` the ctypes view of
``libtpi_hip.so``.  The HIP library is always loaded AFTER ``import torch`` so that it binds to
the ``libamdhip64.so.7`` torch already mapped (one HIP runtime per process).  On a machine with
a visible GPU a missing or broken HIP library is an error, never a silent CPU fallback.
"""
from __future__ import annotations

import importlib.util
import os
import threading
from typing import Optional

from .. import _build

ABI_VERSION = 7  # TPI_ABI_VERSION of csrc/hip/tpi_hip.h

_lock = threading.Lock()
_native = None
_hip = None


def _auto_build() -> bool:
    return os.environ.get("TPI_NO_AUTOBUILD", "") not in ("1", "true", "yes")


def native():
    """The host native module (builds it in-tree on first use if missing)."""
    global _native
    if _native is not None:
        return _native
    with _lock:
        if _native is None:
            if _auto_build():  # content-stamped: a no-op unless the sources changed
                _build.build_native()
            spec = importlib.util.spec_from_file_location("_tpi_native", _build.NATIVE_SO)
            if spec is None or spec.loader is None:
                raise ImportError("native module not found at %s (run __graft_entry__.build())"
                                  % _build.NATIVE_SO)
            module = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(module)
            _native = module
    return _native


_torch_ext = None


def torch_ext():
    """``_tpi_torch`` (``csrc/torchext``): torch helpers that release the GIL, e.g.
    ``empty(shape, like)``.  Loaded after ``import torch`` (it links torch's libraries)."""
    global _torch_ext
    if _torch_ext is not None:
        return _torch_ext
    with _lock:
        if _torch_ext is None:
            import torch  # noqa: F401

            if _auto_build():
                _build.build_torch_ext()
            spec = importlib.util.spec_from_file_location("_tpi_torch", _build.TORCH_EXT)
            if spec is None or spec.loader is None:
                raise ImportError("_tpi_torch not found at %s (run __graft_entry__.build())"
                                  % _build.TORCH_EXT)
            module = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(module)
            _torch_ext = module
    return _torch_ext


class HipError(RuntimeError):
    pass


class HipLib:
    """ctypes bindings of ``csrc/hip/tpi_hip.h``."""

    def __init__(self, path: str):
        self.path = path
        import ctypes  # the HIP bindings only: `tpi apply` never loads them

        lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        c = ctypes
        u64, i64, i32, vp = c.c_uint64, c.c_int64, c.c_int, c.c_void_p
        sig = {
            "tpi_last_error": (c.c_char_p, []),
            "tpi_version": (i32, []),
            "tpi_version_string": (c.c_char_p, []),
            "tpi_device_count": (i32, [c.POINTER(i32)]),
            "tpi_device_numa_node": (i32, [i32, c.POINTER(i32)]),
            "tpi_device_pci_bus_id": (i32, [i32, c.c_char_p, i32]),
            "tpi_engine_create": (vp, [i32, u64, i32, u64]),
            "tpi_engine_destroy": (None, [vp]),
            "tpi_engine_tile_bytes": (u64, [vp]),
            "tpi_engine_chunk_bytes": (u64, [vp]),
            "tpi_engine_d2h_engine": (c.c_uint32, [vp]),
            "tpi_engine_split_chunks": (u64, [vp]),
            "tpi_engine_set_progress": (i32, [vp, vp]),
            "tpi_engine_reserve": (i32, [vp, i32, u64, i32]),
            "tpi_engine_alloc_staging": (i32, [vp]),
            "tpi_engine_set_h2d_sdma": (i32, [vp, i32]),
            "tpi_ipc_export": (i32, [vp, vp, c.POINTER(u64), c.POINTER(u64)]),
            "tpi_mem_range": (i32, [vp, c.POINTER(u64), c.POINTER(u64)]),
            "tpi_copy_segments": (i32, [vp, vp, vp, i32, u64, u64, c.POINTER(u64), vp]),
            "tpi_restore_stream": (i32, [vp, vp, i32, u64, vp, vp, vp, vp, c.c_double, u64,
                                         c.POINTER(u64), c.POINTER(i64), vp]),
            "tpi_restore_stream_at": (i32, [vp, vp, i32, u64, vp, vp, vp, vp, u64, c.c_double,
                                            u64, c.POINTER(u64), c.POINTER(i64), vp]),
            "tpi_save": (i32, [vp, vp, i32, u64, vp, vp, i32, u64, vp]),
            "tpi_restore": (i32, [vp, vp, i32, u64, vp, vp, i32, u64, c.POINTER(u64),
                                  c.POINTER(i64), vp]),
            "tpi_sync": (i32, [vp, vp, i32, u64, vp, vp, vp, i32, u64, c.POINTER(u64), vp]),
            "tpi_save_z": (i32, [vp, vp, i32, u64, vp, vp, vp, u64, c.POINTER(u64), vp]),
            "tpi_restore_z": (i32, [vp, vp, i32, u64, vp, vp, vp, u64, c.POINTER(u64),
                                    c.POINTER(i64), vp]),
            "tpi_snapshot": (i32, [vp, vp, i32, u64, vp, vp, u64]),
            "tpi_spill": (i32, [vp, vp, vp, u64, vp, vp, vp, i32, c.POINTER(u64), vp]),
            "tpi_tpz_encode_device": (i32, [vp, u64, u64, vp, vp, vp, u64]),
            "tpi_tpz_decode_device": (i32, [vp, vp, u64, u64, vp, u64]),
            "tpi_stream_hash": (i32, [vp, i32, u64, u64, u64, vp, u64]),
            "tpi_crc32c_tiles": (i32, [vp, u64, u64, vp, u64]),
            "tpi_shard_hash": (i32, [vp, u64, u64, u64, vp, u64]),
            "tpi_pack_device": (i32, [vp, vp, i32, u64, vp, u64, vp, u64]),
            "tpi_unpack_device": (i32, [vp, vp, i32, u64, vp, u64, vp, vp, u64]),
            "tpi_host_map": (vp, [c.c_char_p, u64, i32, i32]),
            "tpi_host_unmap": (i32, [vp, u64]),
            "tpi_host_register": (i32, [vp, u64]),
            "tpi_host_register_ro": (i32, [vp, u64]),
            "tpi_h2d_async": (i32, [vp, vp, u64, u64]),
            "tpi_host_unregister": (i32, [vp]),
            "tpi_h2d": (i32, [vp, vp, vp, u64]),
            "tpi_d2h": (i32, [vp, vp, vp, u64]),
            "tpi_host_pin_start": (vp, [vp, u64, u64, i32]),
            "tpi_host_pin_ready": (u64, [vp]),
            "tpi_host_pin_hold": (i32, [vp, i32]),
            "tpi_host_pin_window": (u64, [vp]),
            "tpi_host_pin_wait": (i32, [vp]),
            "tpi_host_pin_release": (i32, [vp]),
            "tpi_engine_set_host_region": (i32, [vp, vp, u64, u64, vp]),
            "tpi_loader_create": (vp, [i32, u64, i32, i32, i32]),
            "tpi_loader_destroy": (None, [vp]),
            "tpi_loader_load": (i32, [vp, vp, u64, u64, u64, vp, vp]),
            "tpi_loader_store": (i32, [vp, vp, u64, vp, u64, vp, vp]),
            "tpi_ipc_handle": (i32, [vp, c.c_char_p]),
            "tpi_ipc_open": (i32, [c.c_char_p, i32, c.POINTER(vp)]),
            "tpi_ipc_close": (i32, [vp]),
            "tpi_dmabuf_available": (i32, []),
            "tpi_dmabuf_export": (i32, [vp, u64, c.POINTER(i32), c.POINTER(u64)]),
            "tpi_dmabuf_close": (i32, [i32]),
            "tpi_dmabuf_import": (i32, [i32, i32, c.POINTER(vp), c.POINTER(u64)]),
            "tpi_dmabuf_unmap": (i32, [vp]),
            "tpi_dev_alloc": (i32, [u64, c.POINTER(vp)]),
            "tpi_dev_free": (i32, [vp]),
            "tpi_d2d": (i32, [vp, vp, u64, u64]),
            "tpi_comm_unique_id": (i32, [c.c_char_p]),
            "tpi_comm_init_rank": (vp, [c.c_char_p, i32, i32, i32]),
            "tpi_comm_init_all": (i32, [i32, c.POINTER(i32), c.POINTER(vp)]),
            "tpi_comm_destroy": (None, [vp]),
            "tpi_comm_rank": (i32, [vp]),
            "tpi_comm_size": (i32, [vp]),
            "tpi_comm_allgather_inplace": (i32, [c.POINTER(vp), i32, c.POINTER(vp), u64, i32]),
            "tpi_comm_broadcast": (i32, [c.POINTER(vp), i32, c.POINTER(vp), u64, i32, i32]),
            "tpi_comm_sync": (i32, [c.POINTER(vp), i32]),
            "tpi_nccl_groups_open": (i32, []),
        }
        for name, (res, args) in sig.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        self.lib = lib
        abi = lib.tpi_version()
        if abi != ABI_VERSION:  # a stale build would be called with the wrong signatures
            raise HipError("%s has ABI %d, this package needs %d (rebuild with "
                           "__graft_entry__.build())" % (path, abi, ABI_VERSION))
        self.version = lib.tpi_version_string().decode()

    def error(self) -> str:
        return (self.lib.tpi_last_error() or b"").decode(errors="replace")

    def check(self, rc: int, what: str) -> None:
        if rc != 0:
            raise HipError("%s failed: %s" % (what, self.error()))

    def __getattr__(self, name):
        return getattr(self.lib, name)


def gpu_visible() -> bool:
    try:
        import torch

        return bool(torch.cuda.is_available())
    except Exception:  # pragma: no cover
        return False


def hip(required: bool = True) -> Optional[HipLib]:
    """ctypes handle of libtpi_hip.so; raises if it cannot be loaded and ``required``."""
    global _hip
    if _hip is not None:
        return _hip
    with _lock:
        if _hip is None:
            import torch  # noqa: F401  (maps torch's HIP runtime first)

            try:
                if _auto_build():
                    _build.build_hip()
                _hip = HipLib(_build.HIP_SO)
            except Exception as error:
                if required:
                    raise HipError("libtpi_hip.so unavailable (%s); build it with "
                                   "__graft_entry__.build()" % error) from error
                return None
    return _hip
