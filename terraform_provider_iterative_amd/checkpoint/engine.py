"""The per-device engine of the native checkpoint library (``libtpi_hip.so``) and the pool of
engines prewarmed for the Checkpointer that takes them next.

``DeviceEngine`` wraps one ``tpi_engine`` (``csrc/hip/engine.hip``): its streams, HBM staging
chunks and pinned bounce buffers, and the save / restore / streamed-restore / snapshot /
incremental-sync / HBM hand-off pipelines over them.  ``prewarm_engine`` builds one ahead of
time (a warm or hot standby does, before it blocks) and runs one tiny transfer through every
pipeline, so the first real one loads no code object and allocates nothing.  Reference: the
spot VM restores its data on start (``task/common/machine/machine-script.sh.tpl:89``); these
are the MI355X-side pieces of that restore.
"""
from __future__ import annotations

import ctypes
import threading
import time
from typing import Dict, List, Optional, Tuple

import numpy as np

from ..ops import codec as tpz
from ..ops import hip
from ..ops.packing import PackPlan, align_up
from .base import CheckpointError, TransferResult
from .host import HostRegion

MODES = {"sdma": 0, "direct": 1}


class _Stats(ctypes.Structure):
    _fields_ = [("pack_ms", ctypes.c_double), ("copy_ms", ctypes.c_double),
                ("bytes", ctypes.c_uint64), ("chunks", ctypes.c_uint64)]


class DeviceEngine:
    """Per-device pipeline: compute + copy streams, ``nbuf`` staging chunks in HBM."""

    def __init__(self, device_index: int, chunk_bytes: int, nbuf: int, tile_bytes: int,
                 lite: bool = False):
        """``lite``: leave the HBM staging ring to the first pipeline that needs it (the HBM
        hand-off copy never does): a parked successor's prewarmed engine then holds no
        staging memory.  Otherwise it is allocated now, off any later restore's path."""
        self.lib = hip()
        self.device_index = device_index
        handle = self.lib.tpi_engine_create(device_index, chunk_bytes, nbuf, tile_bytes)
        if not handle:
            raise CheckpointError("engine creation failed: %s" % self.lib.error())
        self.handle = handle
        if not lite and self.lib.tpi_engine_alloc_staging(handle) != 0:
            error = self.lib.error()
            self.lib.tpi_engine_destroy(handle)
            raise CheckpointError("engine staging allocation failed: %s" % error)
        self.chunk_bytes = int(self.lib.tpi_engine_chunk_bytes(handle))
        # which engine moves device -> host bytes: an SDMA copy engine ("sdma<i>") or, with
        # TPI_D2H_ENGINE=blit / no engine, HIP's blit kernels on the CUs ("blit")
        bit = int(self.lib.tpi_engine_d2h_engine(handle))
        self.d2h_engine = "sdma%d" % (bit.bit_length() - 1) if bit else "blit"
        self.split_chunks = 0

    def save(self, plan: PackPlan, host_addr: int, crcs: np.ndarray, mode: int,
             wait_stream: int) -> TransferResult:
        st = _Stats()
        t0 = time.perf_counter()
        rc = self.lib.tpi_save(self.handle, plan.segs.ctypes.data, len(plan.entries), plan.total,
                               ctypes.c_void_p(host_addr), crcs.ctypes.data, mode, wait_stream,
                               ctypes.byref(st))
        self.lib.check(rc, "tpi_save")
        return TransferResult(plan.total, time.perf_counter() - t0, int(st.chunks))

    def restore(self, plan: PackPlan, host_addr: int, crcs: np.ndarray, mode: int,
                signal_stream: int) -> TransferResult:
        st = _Stats()
        bad = ctypes.c_uint64(0)
        first = ctypes.c_int64(-1)
        t0 = time.perf_counter()
        rc = self.lib.tpi_restore(self.handle, plan.segs.ctypes.data, len(plan.entries),
                                  plan.total, ctypes.c_void_p(host_addr), crcs.ctypes.data, mode,
                                  signal_stream, ctypes.byref(bad), ctypes.byref(first),
                                  ctypes.byref(st))
        self.lib.check(rc, "tpi_restore")
        return TransferResult(plan.total, time.perf_counter() - t0, int(st.chunks),
                              int(bad.value), int(first.value))

    def save_z(self, plan: PackPlan, host_addr: int, crcs: np.ndarray, csizes: np.ndarray,
               wait_stream: int) -> TransferResult:
        st = _Stats()
        wire = ctypes.c_uint64(0)
        t0 = time.perf_counter()
        rc = self.lib.tpi_save_z(self.handle, plan.segs.ctypes.data, len(plan.entries),
                                 plan.total, ctypes.c_void_p(host_addr), crcs.ctypes.data,
                                 csizes.ctypes.data, wait_stream, ctypes.byref(wire),
                                 ctypes.byref(st))
        self.lib.check(rc, "tpi_save_z")
        return TransferResult(plan.total, time.perf_counter() - t0, int(st.chunks),
                              wire_bytes=int(wire.value))

    def restore_z(self, plan: PackPlan, host_addr: int, crcs: np.ndarray, csizes: np.ndarray,
                  signal_stream: int) -> TransferResult:
        st = _Stats()
        bad = ctypes.c_uint64(0)
        first = ctypes.c_int64(-1)
        t0 = time.perf_counter()
        rc = self.lib.tpi_restore_z(self.handle, plan.segs.ctypes.data, len(plan.entries),
                                    plan.total, ctypes.c_void_p(host_addr), crcs.ctypes.data,
                                    csizes.ctypes.data, signal_stream, ctypes.byref(bad),
                                    ctypes.byref(first), ctypes.byref(st))
        self.lib.check(rc, "tpi_restore_z")
        return TransferResult(plan.total, time.perf_counter() - t0, int(st.chunks),
                              int(bad.value), int(first.value), wire_bytes=int(st.bytes))

    def copy_segments(self, src: np.ndarray, plan: PackPlan, signal_stream: int,
                      dst: Optional[np.ndarray] = None) -> TransferResult:
        """``src`` -> ``plan``'s tensors (or the descriptors ``dst``: the same stream, possibly
        split into more segments than the plan has, like ``src``)."""
        st = _Stats()
        bad = ctypes.c_uint64(0)
        t0 = time.perf_counter()
        dst = plan.segs if dst is None else dst
        if len(dst) != len(src):
            raise CheckpointError("copy_segments: %d source and %d destination segments"
                                  % (len(src), len(dst)))
        rc = self.lib.tpi_copy_segments(self.handle, src.ctypes.data, dst.ctypes.data,
                                        len(dst), plan.total, signal_stream,
                                        ctypes.byref(bad), ctypes.byref(st))
        self.lib.check(rc, "tpi_copy_segments")
        return TransferResult(plan.total, time.perf_counter() - t0, int(st.chunks),
                              int(bad.value), wire_bytes=0,
                              device_seconds=st.pack_ms / 1e3 if st.pack_ms >= 0 else -1.0)

    def reserve(self, nsegs: int, ntiles: int, codec: bool) -> None:
        """Allocate now the device buffers the first save/restore of that size would."""
        self.lib.check(self.lib.tpi_engine_reserve(self.handle, nsegs, ntiles, 1 if codec else 0),
                       "tpi_engine_reserve")

    def set_h2d_sdma(self, on: bool) -> int:
        """Streamed restores copy host -> device on an SDMA engine of their own (host
        driven), off HIP's H2D engine; returns the engine index, -1 when none is free."""
        return int(self.lib.tpi_engine_set_h2d_sdma(self.handle, 1 if on else 0))

    def set_progress(self, words_addr: int) -> None:
        self.lib.check(self.lib.tpi_engine_set_progress(self.handle,
                                                        ctypes.c_void_p(words_addr or None)),
                       "tpi_engine_set_progress")

    def restore_stream(self, plan: PackPlan, host_addr: int, crcs: np.ndarray,
                       csizes: Optional[np.ndarray], words_addr: int, timeout: float,
                       signal_stream: int, tile_base: int = 0) -> TransferResult:
        """``tile_base``: ``plan`` (and ``host_addr``, ``crcs``, ``csizes``) describe the
        stretch of the writer's stream that starts at that tile; the progress words count the
        whole stream."""
        st = _Stats()
        bad = ctypes.c_uint64(0)
        first = ctypes.c_int64(-1)
        t0 = time.perf_counter()
        rc = self.lib.tpi_restore_stream_at(
            self.handle, plan.segs.ctypes.data, len(plan.entries), plan.total,
            ctypes.c_void_p(host_addr), crcs.ctypes.data,
            ctypes.c_void_p(csizes.ctypes.data if csizes is not None else None),
            ctypes.c_void_p(words_addr), tile_base, ctypes.c_double(timeout), signal_stream,
            ctypes.byref(bad), ctypes.byref(first), ctypes.byref(st))
        self.lib.check(rc, "tpi_restore_stream")
        # chunks copied over two streams because the restore trailed its writer (duplex link)
        self.split_chunks = int(self.lib.tpi_engine_split_chunks(self.handle))
        return TransferResult(plan.total, time.perf_counter() - t0, int(st.chunks),
                              int(bad.value), int(first.value), wire_bytes=int(st.bytes))

    def snapshot(self, plan: PackPlan, dev_dst: int, dev_crcs: int, wait_stream: int) -> None:
        rc = self.lib.tpi_snapshot(self.handle, plan.segs.ctypes.data, len(plan.entries),
                                   plan.total, ctypes.c_void_p(dev_dst),
                                   ctypes.c_void_p(dev_crcs), wait_stream)
        self.lib.check(rc, "tpi_snapshot")

    def spill(self, dev_src: int, dev_crcs: int, total: int, host_addr: int,
              crcs: np.ndarray, csizes: np.ndarray, codec: bool) -> TransferResult:
        st = _Stats()
        wire = ctypes.c_uint64(0)
        t0 = time.perf_counter()
        rc = self.lib.tpi_spill(self.handle, ctypes.c_void_p(dev_src), ctypes.c_void_p(dev_crcs),
                                total, ctypes.c_void_p(host_addr), crcs.ctypes.data,
                                csizes.ctypes.data, 1 if codec else 0, ctypes.byref(wire),
                                ctypes.byref(st))
        self.lib.check(rc, "tpi_spill")
        return TransferResult(total, time.perf_counter() - t0, int(st.chunks),
                              wire_bytes=int(wire.value))

    def sync(self, plan: PackPlan, host_addr: int, crcs: np.ndarray, full: bool,
             wait_stream: int, dev_prev: int = 0) -> TransferResult:
        st = _Stats()
        dirty = ctypes.c_uint64(0)
        t0 = time.perf_counter()
        rc = self.lib.tpi_sync(self.handle, plan.segs.ctypes.data, len(plan.entries), plan.total,
                               ctypes.c_void_p(host_addr), crcs.ctypes.data,
                               ctypes.c_void_p(dev_prev or None), 1 if full else 0,
                               wait_stream, ctypes.byref(dirty), ctypes.byref(st))
        self.lib.check(rc, "tpi_sync")
        res = TransferResult(int(st.bytes), time.perf_counter() - t0, int(st.chunks))
        res.dirty_tiles = int(dirty.value)
        return res

    def close(self) -> None:
        if self.handle:
            self.lib.tpi_engine_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


PREWARM_SEGS, PREWARM_TILES = 4096, 1 << 18
# Engines created ahead of the Checkpointer that takes them (prewarm_engine).
_engine_pool: Dict[Tuple[int, int, int, int], List[DeviceEngine]] = {}
_engine_pool_lock = threading.Lock()


def prewarm_engine(device_index: Optional[int] = None, chunk_bytes: int = 256 << 20,
                   nbuf: int = 3, tile_bytes: int = 1 << 20, lite: bool = False) -> bool:
    """Create a device engine now for the next :class:`Checkpointer` with these parameters.

    Engine creation (streams, HBM staging chunks, pinned bounce buffers, SDMA binding) takes
    ~0.1 s on MI355X.  A warm standby calls this before it blocks (:func:`preemption.standby`),
    so after its activation the Checkpointer starts without it and the HBM hand-off begins
    ~0.1 s earlier.  Returns False when no engine could be made (no GPU, no library)."""
    try:
        if device_index is None:
            import torch

            device_index = torch.cuda.current_device()
        engine = DeviceEngine(device_index, chunk_bytes, nbuf, tile_bytes, lite=lite)
        if lite:  # streams, events and the hand-off kernels' code: what the HBM copy needs
            _warm_handoff(engine, device_index, tile_bytes)
        else:
            # a successor's first restore then allocates nothing (PREWARM_TILES: 256 GB of
            # 1 MiB tiles, a few MB of descriptors); allocating under its predecessor's release
            # of HBM waits for the driver's clearing (profiles/round4/materialize_170g.md)
            engine.reserve(PREWARM_SEGS, PREWARM_TILES, True)
            _warm_engine(engine, device_index, tile_bytes)
    except Exception:
        return False
    with _engine_pool_lock:
        _engine_pool.setdefault((device_index, chunk_bytes, nbuf, tile_bytes), []).append(engine)
    return True


def _warm_engine(engine: DeviceEngine, device_index: int, tile_bytes: int) -> None:
    """One tiny save + restore through every pipeline (raw and TPZ1; contiguous and
    transposed tensors): the first launch of each kernel loads its code object, which
    allocates device memory -- under a predecessor's release of HBM that waits seconds for
    the driver's clearing (profiles/round4/materialize_170g.md)."""
    import torch

    dev = torch.device("cuda", device_index)
    tensors = {"a": torch.ones(4096, device=dev), "t": torch.ones(64, 48, device=dev).t()}
    plan = PackPlan.from_tensors(tensors, tile_bytes)
    region = HostRegion(align_up(2 * max(plan.total, tpz.bound(plan.total, tile_bytes)), 4096),
                        device=True, populate=True)
    try:
        crcs = np.zeros(plan.ntiles, np.uint32)
        csizes = np.zeros(plan.ntiles, np.uint32)
        sig = torch.cuda.current_stream(dev).cuda_stream
        engine.save(plan, region.addr, crcs, MODES["sdma"], sig)
        engine.restore(plan, region.addr, crcs, MODES["sdma"], sig)
        engine.save_z(plan, region.addr, crcs, csizes, sig)
        engine.restore_z(plan, region.addr, crcs, csizes, sig)
        # and the HBM hand-off's copy + read-back kernels (a hot standby's first restore)
        dst = {"a": torch.zeros(4096, device=dev), "t": torch.zeros(64, 48, device=dev).t()}
        engine.copy_segments(plan.segs.copy(), PackPlan.from_tensors(dst, tile_bytes), sig)
        torch.cuda.synchronize(dev)
    finally:
        region.close()


def _warm_handoff(engine: DeviceEngine, device_index: int, tile_bytes: int) -> None:
    """One tiny HBM hand-off copy + read-back (contiguous and transposed): loads the code
    object of the copy kernels and sizes the descriptor buffers, nothing else."""
    import torch

    dev = torch.device("cuda", device_index)
    src = {"a": torch.ones(4096, device=dev), "t": torch.ones(64, 48, device=dev).t()}
    dst = {"a": torch.zeros(4096, device=dev), "t": torch.zeros(64, 48, device=dev).t()}
    plan = PackPlan.from_tensors(src, tile_bytes)
    sig = torch.cuda.current_stream(dev).cuda_stream
    engine.copy_segments(plan.segs.copy(), PackPlan.from_tensors(dst, tile_bytes), sig)
    torch.cuda.synchronize(dev)


def _take_engine(device_index: int, chunk_bytes: int, nbuf: int,
                 tile_bytes: int) -> Optional[DeviceEngine]:
    """The prewarmed engine for these parameters, if any.  Prewarmed engines of the device that
    do not match are released: their staging chunks and pinned buffers would otherwise stay
    allocated for the life of the process."""
    with _engine_pool_lock:
        pool = _engine_pool.get((device_index, chunk_bytes, nbuf, tile_bytes))
        engine = pool.pop() if pool else None
        stale = [k for k in _engine_pool if k[0] == device_index]
        unused = [e for k in stale for e in _engine_pool.pop(k)]
    for other in unused:
        other.close()
    return engine


