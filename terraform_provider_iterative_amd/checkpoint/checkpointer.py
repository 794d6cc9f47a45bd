"""Checkpoint save/restore of tensor sets through host memory.

This is the MI355X replacement of the reference's "transparent checkpoint" (the workdir
sync of ``machine-script.sh.tpl:89,118-124``): on preemption (SIGTERM) a rank packs its
tensors (flatten + CRC32C per tile, ``csrc/hip/kernels.hip``) into pinned host DRAM through
a double-buffered pipeline on a side stream (``csrc/hip/engine.hip``); its successor restores
from the same region (or from the persisted file) and verifies every tile.

Region layout (also the persisted file format)::

    0              b"TPICKPT2" | u64 header_len | u64 entries_offset | u64 entries_len
    32             JSON header (see ``_header``; small: sizes, codec, CRC, metadata)
    entries_offset JSON list of tensor entries (name/dtype/shape/offset; fixed per plan,
                   identified in the header by its SHA-256, so a restore never parses it)
    crc_offset     u32 CRC32C per (raw) tile                  (4 KiB aligned)
    csize_offset   u32 encoded blob size per tile (codec "tpz1" only)
    stream_offset  packed stream (``ops.packing`` layout), or with ``codec="tpz1"`` the
                   concatenated TPZ1 tile blobs (``ops.codec``)   (4 KiB aligned)

The JSON header carries ``"complete": true`` only after a save finished, and is written last;
a *streamed* save (preemption hand-off, :meth:`Checkpointer.save` with ``on_stream``) first
writes a header with ``"streaming": true`` and publishes its progress in a 64-byte block at
``entries_offset - 64`` (u64: magic ``TPIPROG1``, generation, tiles in host memory, stream bytes
of those tiles, state 1 streaming / 2 complete / 3 failed, writer pid), so a successor restores
tile runs as they land instead of after the whole spill;
``"codec"`` / ``"stream_bytes"`` say how the stream section is encoded and how long it is;
``"generation"`` orders the copies of a two-slot region (``Checkpointer(slots=2)``: two such
layouts back to back, the newest complete one is the checkpoint).  The layout does not depend
on the codec, so any reader bound to the same tensors loads either encoding.
"""
from __future__ import annotations

import ctypes
import hashlib
import json
import os
import queue
import socket
import struct
import tempfile
import threading
import time
from dataclasses import dataclass
from typing import Any, Dict, List, Mapping, Optional, Sequence, Tuple, Union

import numpy as np

from ..ops import codec as tpz
from ..ops import hip, native
from ..ops.packing import SEG_CONTIG, PackPlan, TensorEntry, align_up
from ..ops.packing import pack as host_pack, unpack as host_unpack
from . import host
from .host import HostRegion

MAGIC = b"TPICKPT2"
PREAMBLE = 32
FILE_THREADS = 16        # persist / load: native pwrite/pread threads
LOAD_CHUNK = 256 << 20   # load: bytes read (and published to the restore) per step
PROGRESS_MAGIC = struct.unpack("<Q", b"TPIPROG1")[0]
STREAM_RUNNING, STREAM_COMPLETE, STREAM_FAILED = 1, 2, 3
MODES = {"sdma": 0, "direct": 1}
CODECS = ("none", "tpz1")


class CheckpointError(RuntimeError):
    pass


class _Stats(ctypes.Structure):
    _fields_ = [("pack_ms", ctypes.c_double), ("copy_ms", ctypes.c_double),
                ("bytes", ctypes.c_uint64), ("chunks", ctypes.c_uint64)]


@dataclass
class TransferResult:
    bytes: int
    seconds: float
    chunks: int = 0
    bad_tiles: int = 0
    first_bad: int = -1
    crc: int = 0
    dirty_tiles: int = -1  # incremental sync: tiles that changed since the previous sync
    wire_bytes: int = -1   # bytes that crossed the link / landed in the region (codec)
    released_bytes: int = 0  # device memory freed behind the spill (save(release_behind=True))

    def __post_init__(self):
        if self.wire_bytes < 0:
            self.wire_bytes = self.bytes

    @property
    def gbps(self) -> float:
        return self.bytes / self.seconds / 1e9 if self.seconds > 0 else float("inf")


class DeviceEngine:
    """Per-device pipeline: compute + copy streams, ``nbuf`` staging chunks in HBM."""

    def __init__(self, device_index: int, chunk_bytes: int, nbuf: int, tile_bytes: int):
        self.lib = hip()
        self.device_index = device_index
        handle = self.lib.tpi_engine_create(device_index, chunk_bytes, nbuf, tile_bytes)
        if not handle:
            raise CheckpointError("engine creation failed: %s" % self.lib.error())
        self.handle = handle
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
                              int(bad.value), wire_bytes=0)

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
ALLOC_HEADROOM = 512 << 20  # materialize(): free HBM beyond a tensor's size before allocating it
ALLOC_LOOKAHEAD = 3  # materialize(): groups allocated ahead of the restore once HBM runs short
# export_hbm(): the largest PyTorch allocation offered through HIP IPC.  On the MI355X boxes
# (ROCm 7.2, PyTorch 2.10) hipIpcOpenMemHandle never returns for a caching-allocator block of
# 2 GiB or more (2040 MiB opens at once), so a state holding one takes the host path instead of
# hanging its successor (profiles/round4/ipc_lifetime.md).  TPI_IPC_MAX_ALLOC overrides.
IPC_MAX_ALLOC = 2 << 30
# The hand-off's route (TPI_HBM_ROUTE):
# * "auto" (default): every allocation over HIP IPC (exported and opened in microseconds).
#   Tensors in an allocation of IPC_MAX_ALLOC or more -- which HIP IPC cannot open -- are first
#   copied (device to device, ~1 ms per 5 GB) into plain hipMalloc blocks of RELOCATE_CHUNK
#   bytes, and those travel instead (profiles/round5/ipc_cause.md);
# * "dmabuf" (experimental): allocations of IPC_MAX_ALLOC or more as dma-buf descriptors over a
#   Unix socket, mapped with hsa_amd_interop_map_buffer.  Bit-exact when the exporter idles,
#   but a 100 GB hot hand-off faulted the GPU while the exporter's spill ran (round 5, r5f);
#   a dma-buf export + map also costs ~1.5 ms per allocation next to a live 100 GB state;
# * "ipc": HIP IPC only; a state with an allocation of IPC_MAX_ALLOC or more is refused (the
#   successor restores from the host copy).
HBM_ROUTES = ("auto", "dmabuf", "ipc")
RELOCATE_CHUNK = 1 << 30
FDS_PER_MESSAGE = 200  # SCM_RIGHTS batch (the kernel's limit is 253 per message)

# Engines created ahead of the Checkpointer that takes them (prewarm_engine).
_engine_pool: Dict[Tuple[int, int, int, int], List[DeviceEngine]] = {}
_engine_pool_lock = threading.Lock()


def prewarm_engine(device_index: Optional[int] = None, chunk_bytes: int = 256 << 20,
                   nbuf: int = 3, tile_bytes: int = 1 << 20) -> bool:
    """Create a device engine now for the next :class:`Checkpointer` with these parameters.

    Engine creation (streams, HBM staging chunks, pinned bounce buffers, SDMA binding) takes
    ~0.1 s on MI355X.  A warm standby calls this before it blocks (:func:`preemption.standby`),
    so after its activation the Checkpointer starts without it and the HBM hand-off begins
    ~0.1 s earlier.  Returns False when no engine could be made (no GPU, no library)."""
    try:
        if device_index is None:
            import torch

            device_index = torch.cuda.current_device()
        engine = DeviceEngine(device_index, chunk_bytes, nbuf, tile_bytes)
        # a successor's first restore then allocates nothing (PREWARM_TILES: 256 GB of 1 MiB
        # tiles, a few MB of descriptors); allocating under its predecessor's release of HBM
        # waits for the driver's clearing (profiles/round4/materialize_170g.md)
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


def _layout(header_cap: int, entries_len: int, ntiles: int, total: int, tile_bytes: int):
    entries_offset = align_up(PREAMBLE + header_cap, 4096)
    crc_offset = align_up(entries_offset + entries_len, 4096)
    csize_offset = crc_offset + 4 * ntiles
    stream_offset = align_up(csize_offset + 4 * ntiles, 4096)
    capacity = max(total, tpz.bound(total, tile_bytes))
    return entries_offset, crc_offset, csize_offset, stream_offset, stream_offset + capacity


def _writer_alive(pid: int) -> bool:
    """Is the process that published a streamed save still running (zombies count as gone)?
    Our own pid is alive (``load()`` streams from a reader thread of this process)."""
    if pid <= 0:
        return False
    if pid == os.getpid():
        return True
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        return True
    try:
        with open("/proc/%d/stat" % pid) as f:
            state = f.read().rsplit(")", 1)[1].split()[0]
        return state not in ("Z", "X")
    except (OSError, IndexError):
        return True


def streaming_writer(path: str) -> Optional[Dict[str, int]]:
    """``{"pid", "total"}`` of a live process streaming a save into the region file ``path``
    right now (a preempted predecessor), else None.  Reads the file only (no mapping)."""
    try:
        with open(path, "rb") as f:
            head = f.read(PREAMBLE + Checkpointer.HEADER_RESERVE)
            header = Checkpointer.read_header(np.frombuffer(head, np.uint8))
            bases = [0]
            if header.get("entries_len") is not None:
                slot_end = _layout(Checkpointer.HEADER_RESERVE, int(header["entries_len"]),
                                   int(header["ntiles"]), int(header["total"]),
                                   int(header["tile_bytes"]))[4]
                if os.fstat(f.fileno()).st_size >= 2 * align_up(slot_end, 4096):
                    bases.append(align_up(slot_end, 4096))
            for base in bases:
                f.seek(base + int(header["entries_offset"]) - 64)
                prog = np.frombuffer(f.read(64), np.uint64)
                if (len(prog) == 8 and int(prog[0]) == PROGRESS_MAGIC
                        and int(prog[4]) == STREAM_RUNNING and _writer_alive(int(prog[5]))
                        and int(prog[5]) != os.getpid()):
                    return {"pid": int(prog[5]), "total": int(header["total"])}
    except (OSError, ValueError, KeyError, CheckpointError):
        return None
    return None


def _local_scratch(remote_path: str) -> str:
    """Where a checkpoint bound for (or fetched from) another node is staged on this one:
    ``TPI_PERSIST_TMPDIR``, else the task directory, else the temp directory."""
    base = (os.environ.get("TPI_PERSIST_TMPDIR") or os.environ.get("TPI_TASK_DIRECTORY")
            or tempfile.gettempdir())
    return os.path.join(base, ".tpi-persist-%d-%s" % (os.getpid(),
                                                     os.path.basename(remote_path) or "ckpt"))


class PendingSave:
    """An asynchronous save in flight (:meth:`Checkpointer.save_async`)."""

    def __init__(self, stall_s: float):
        self.stall_s = stall_s  # host time the caller spent in save_async
        self._done = threading.Event()
        self._result: Optional[TransferResult] = None
        self._error: Optional[BaseException] = None
        self._thread: Optional[threading.Thread] = None

    def done(self) -> bool:
        return self._done.is_set()

    def result(self, timeout: Optional[float] = None) -> TransferResult:
        if not self._done.wait(timeout):
            raise TimeoutError("checkpoint spill still running")
        if self._error is not None:
            raise CheckpointError("asynchronous save failed: %s" % self._error) from self._error
        return self._result

    wait = result


class _Slot:
    """One checkpoint copy inside the region: ``[preamble | header | entries | CRCs | blob
    sizes | stream]`` at ``base`` (the persisted file format is exactly one slot)."""

    def __init__(self, ck: "Checkpointer", index: int, base: int):
        self.index = index
        self.base = base
        self.crcs = ck.region.array(base + ck.crc_offset, 4 * ck.plan.ntiles, np.uint32)
        self.csizes = ck.region.array(base + ck.csize_offset, 4 * ck.plan.ntiles, np.uint32)
        # streamed-save progress block (see module docstring); words 2-3 are what the engine
        # publishes into
        self.progress = ck.region.array(base + ck.entries_offset - 64, 64, np.uint64)
        self.digests = None          # device u64 per tile: content of this slot (sync)
        self.digests_valid = False   # ... describes what the slot holds right now


class Checkpointer:
    """Save/restore a fixed set of tensors through one host region.

    ``path=None`` keeps the spill in anonymous host DRAM (lives as long as this object);
    a path under ``/dev/shm`` survives the process (preemption), a path on disk survives the
    node.  Device tensors use the HIP pipeline, host tensors the C++ host path.

    ``codec="tpz1"`` encodes every tile with the lossless byte-plane codec before it leaves
    the GPU (``csrc/hip/codec.hip``): the PCIe-bound spill then moves fewer bytes, which is
    what bounds save/restore throughput.  CRCs always cover the raw tiles.

    ``slots=2`` keeps two copies (generation-numbered; a save always writes the older one and
    the newer one stays valid until the new header lands), so a process killed in the middle
    of a save -- past the grace period, OOM, a crash during a periodic :meth:`save_async`
    spill -- still leaves the previous checkpoint to resume from, at twice the host memory.
    With ``slots=1`` (default, the memory-lean choice for a preemption-only spill) a save
    invalidates the one copy first: keep a persisted file (:meth:`persist`) if that gap
    matters.
    """

    HEADER_RESERVE = 1 << 20  # room for metadata (e.g. host-side optimizer scalars)

    def __init__(self, tensors: Union[Mapping[str, Any], Sequence[Any]],
                 path: Optional[str] = None, *, tile_bytes: int = 1 << 20,
                 chunk_bytes: int = 256 << 20, nbuf: int = 3, mode: str = "sdma",
                 numa: bool = True, populate: bool = True, codec: str = "none",
                 slots: int = 1, _plan: Optional[PackPlan] = None):
        t0 = time.perf_counter()
        # _plan: a layout without tensors yet (materialize(): they are allocated group by group)
        self.plan = _plan if _plan is not None else PackPlan.from_tensors(tensors, tile_bytes)
        self.path = path
        self.mode = MODES[mode]
        if codec not in CODECS:
            raise ValueError("codec must be one of %s" % (CODECS,))
        if codec != "none" and self.mode != MODES["sdma"]:
            raise ValueError("the codec needs the staged (sdma) pipeline")
        if slots not in (1, 2):
            raise ValueError("slots must be 1 or 2")
        self.codec = codec
        # entries are serialised once; saves copy the bytes, restores compare the digest
        self._entries_blob = json.dumps([e.to_json() for e in self.plan.entries]).encode()
        self._entries_digest = hashlib.sha256(self._entries_blob).hexdigest()
        self.header_cap = self.HEADER_RESERVE
        (self.entries_offset, self.crc_offset, self.csize_offset, self.stream_offset,
         slot_end) = _layout(self.header_cap, len(self._entries_blob), self.plan.ntiles,
                             self.plan.total, self.plan.tile_bytes)
        self.slot_bytes = align_up(slot_end, 4096)
        self.size = self.slot_bytes * slots if slots > 1 else slot_end
        self.engine = None
        numa_node = -1
        if self.plan.on_device:
            import torch

            dev = torch.device(self.plan.device)
            self.device_index = dev.index if dev.index is not None else torch.cuda.current_device()
            if numa:
                node = ctypes.c_int(-1)
                if hip().tpi_device_numa_node(self.device_index, ctypes.byref(node)) == 0:
                    numa_node = node.value
            t1 = time.perf_counter()
            self.engine = (_take_engine(self.device_index, chunk_bytes, nbuf, tile_bytes)
                           or DeviceEngine(self.device_index, chunk_bytes, nbuf, tile_bytes))
        t2 = time.perf_counter()
        adopted = host.adopt(path, self.size) if path and self.plan.on_device else None
        if adopted is not None and adopted.pinner and self.mode != MODES["sdma"]:
            adopted.close()  # the direct (zero-copy kernel) path needs one registration
            adopted = None
        self.region = adopted or HostRegion(self.size, path, device=self.plan.on_device,
                                            numa_node=numa_node, populate=populate)
        if self.engine is not None and self.region.pinner:
            # a progressively pinned region (prefetch()): copies wait for their 1 GiB window
            hip().tpi_engine_set_host_region(self.engine.handle, ctypes.c_void_p(self.region.addr),
                                             self.region.size, self.region.window,
                                             self.region.pinner)
        self.slots = [_Slot(self, i, i * self.slot_bytes) for i in range(slots)]
        t3 = time.perf_counter()
        # where construction time goes (seconds): plan+layout, device engine, host region
        self.init_times = {"plan": round((t1 if self.engine else t2) - t0, 4),
                           "engine": round(t2 - t1, 4) if self.engine else 0.0,
                           "region": round(t3 - t2, 4)}
        self.saves = 0
        self._snap = self._snap_crcs = None  # HBM snapshot of save_async
        self._pending: Optional[PendingSave] = None
        self.last_save: Optional[TransferResult] = None
        self.last_restore: Optional[TransferResult] = None
        # close() stops wait_stream() pollers and joins the threads that watch this region
        # (the hand-off's durability watcher) before the region is unmapped under them
        self._closing = threading.Event()
        self._watchers: List[threading.Thread] = []

    # -- slots -------------------------------------------------------------------------------
    def _slot_header(self, slot: _Slot) -> Optional[Dict]:
        try:
            header = self.read_header(self.region.array(slot.base, self.crc_offset))
        except (CheckpointError, ValueError):
            return None
        return header if header.get("complete") else None

    def _active(self) -> Optional[Tuple[_Slot, Dict]]:
        """The complete slot with the newest generation, with its header."""
        best = None
        for slot in self.slots:
            header = self._slot_header(slot)
            if header is not None and (best is None or
                                       header.get("generation", 0) > best[1].get("generation", 0)):
                best = (slot, header)
        return best

    def _streaming(self) -> Optional[Tuple[_Slot, Dict]]:
        """A slot a streamed save is writing (or has just finished) that is newer than the
        newest complete checkpoint: what a preempted rank's successor restores.  A slot still
        marked running whose writer process is gone (SIGKILLed past the grace period, OOM) is
        no stream: waiting on it would only time out."""
        active = self._active()
        floor = active[1].get("generation", 0) if active else 0
        best = None
        for slot in self.slots:
            try:
                header = self.read_header(self.region.array(slot.base, self.crc_offset))
            except (CheckpointError, ValueError):
                continue
            prog = slot.progress
            if (header.get("streaming") and not header.get("complete")
                    and int(prog[0]) == PROGRESS_MAGIC
                    and int(prog[1]) == header.get("generation")
                    and int(prog[4]) in (STREAM_RUNNING, STREAM_COMPLETE)
                    and (int(prog[4]) == STREAM_COMPLETE or _writer_alive(int(prog[5])))
                    and header.get("generation", 0) > floor
                    and (best is None or header["generation"] > best[1]["generation"])):
                best = (slot, header)
        return best

    def candidates(self) -> List[Dict]:
        """Every restorable copy in the region, newest first: ``{"generation", "metadata",
        "streaming"}`` (a streamed save in flight, then the complete slots).  Ranks that must
        resume the same step pick a common one (:meth:`TrainingState.resume_consistent`)."""
        out = []
        streaming = self._streaming()
        if streaming is not None:
            out.append({"generation": streaming[1].get("generation", 0), "streaming": True,
                        "metadata": streaming[1].get("metadata", {})})
        for slot in self.slots:
            header = self._slot_header(slot)
            if header is not None:
                out.append({"generation": header.get("generation", 0), "streaming": False,
                            "metadata": header.get("metadata", {})})
        out.sort(key=lambda c: -c["generation"])
        return out

    def latest(self) -> Optional[Dict]:
        """Header of the newest restorable checkpoint -- complete, or being streamed by a
        preempted predecessor -- or None."""
        streaming = self._streaming()
        if streaming is not None:
            return streaming[1]
        active = self._active()
        return active[1] if active else None

    def durable(self, generation: int) -> bool:
        """Does the region hold a complete copy of ``generation`` (or a newer one)?"""
        active = self._active()
        return active is not None and active[1].get("generation", 0) >= generation

    def wait_stream(self, timeout: Optional[float] = None) -> Optional[bool]:
        """Wait until a streamed save by *another* live process (a preempted predecessor
        spilling behind an HBM hand-off) has finished writing this region.  Returns True when
        it completed, False when it failed (or its writer died), None when there was none or
        this checkpointer is being closed.
        Every save / load calls it first: a save must not overwrite a slot that is still
        being written, and must not drop the only host copy before it exists."""
        if timeout is None:
            timeout = float(os.environ.get("TPI_STREAM_TIMEOUT", "30"))
        deadline = time.monotonic() + timeout
        seen = None
        while True:
            foreign = None
            for slot in self.slots:
                prog = slot.progress
                if (int(prog[0]) == PROGRESS_MAGIC and int(prog[4]) == STREAM_RUNNING
                        and int(prog[5]) not in (0, os.getpid())):
                    foreign = slot
            if foreign is None:
                if seen is None:
                    return None
                return int(seen.progress[4]) == STREAM_COMPLETE
            if self._closing.is_set():  # (the outcome above wins over a close racing it)
                return None
            seen = foreign
            if not _writer_alive(int(foreign.progress[5])) or time.monotonic() > deadline:
                return False
            time.sleep(0.002)

    def _wait_writers(self) -> None:
        """:meth:`wait_stream` before writing the region: a foreign writer that is still alive
        after the timeout keeps its slot -- two processes must never write one slot."""
        if self.wait_stream() is not False:
            return
        for slot in self.slots:
            prog = slot.progress
            owner = int(prog[5])
            if (int(prog[0]) == PROGRESS_MAGIC and int(prog[4]) == STREAM_RUNNING
                    and owner not in (0, os.getpid()) and _writer_alive(owner)):
                raise CheckpointError("process %d is still streaming a checkpoint into this "
                                      "region (TPI_STREAM_TIMEOUT passed)" % owner)

    def _target(self) -> Tuple[_Slot, int]:
        """(slot the next save writes, generation it gets): never the active one if there
        are two slots."""
        active = self._active()
        generation = (active[1].get("generation", 0) + 1) if active else 1
        if len(self.slots) == 1 or active is None:
            return self.slots[0], generation
        return self.slots[1 - active[0].index], generation

    @property
    def crcs(self) -> np.ndarray:
        """Tile CRCs of the current checkpoint (or of slot 0 when there is none yet)."""
        active = self._active()
        return (active[0] if active else self.slots[0]).crcs

    @property
    def csizes(self) -> np.ndarray:
        active = self._active()
        return (active[0] if active else self.slots[0]).csizes

    # -- header ------------------------------------------------------------------------------
    def _header(self, complete: bool, crc: int, metadata: Optional[Dict], codec: str = "none",
                stream_bytes: Optional[int] = None, generation: int = 1) -> Dict:
        return {"format": 3, "complete": complete, "tile_bytes": self.plan.tile_bytes,
                "total": self.plan.total, "ntiles": self.plan.ntiles,
                "ntensors": len(self.plan.entries), "entries_sha256": self._entries_digest,
                "entries_offset": self.entries_offset, "entries_len": len(self._entries_blob),
                "crc_offset": self.crc_offset, "csize_offset": self.csize_offset,
                "stream_offset": self.stream_offset, "codec": codec,
                "stream_bytes": self.plan.total if stream_bytes is None else stream_bytes,
                "crc32c": crc, "saved_at": time.time(), "saves": self.saves,
                "generation": generation, "metadata": metadata or {}}

    def _write_header(self, slot: _Slot, header: Dict) -> None:
        blob = json.dumps(header).encode()
        if len(blob) > self.header_cap - 128:  # the progress block sits at the reserve's end
            raise CheckpointError("checkpoint metadata too large (%d bytes)" % len(blob))
        n = len(self._entries_blob)
        self.region.array(slot.base + self.entries_offset, n)[:] = np.frombuffer(
            self._entries_blob, np.uint8)
        pre = self.region.array(slot.base, PREAMBLE + len(blob))
        pre[PREAMBLE:] = np.frombuffer(blob, np.uint8)
        pre[:PREAMBLE] = np.frombuffer(MAGIC + struct.pack("<QQQ", len(blob),
                                                           self.entries_offset, n), np.uint8)

    def _invalidate(self, slot: _Slot) -> None:
        self.region.array(slot.base, 8)[:] = 0
        slot.progress[:] = 0
        slot.digests_valid = False

    @staticmethod
    def read_header(buf: np.ndarray) -> Dict:
        raw = buf[:PREAMBLE].tobytes()
        if raw[:8] != MAGIC:
            raise CheckpointError("no checkpoint (bad magic)")
        (n,) = struct.unpack("<Q", raw[8:16])
        return json.loads(buf[PREAMBLE:PREAMBLE + n].tobytes())

    def entries(self) -> list:
        """Tensor entries recorded in the region (parsed on demand)."""
        active = self._active()
        base = active[0].base if active else 0
        header = active[1] if active else self.header()
        raw = self.region.array(base + header["entries_offset"], header["entries_len"]).tobytes()
        return json.loads(raw)

    def header(self) -> Dict:
        """Header of the current checkpoint; raises :class:`CheckpointError` if none."""
        active = self._active()
        if active is not None:
            return active[1]
        return self.read_header(self.region.array(0, self.crc_offset))

    # -- operations --------------------------------------------------------------------------
    def _release_behind(self, progress: np.ndarray, stop: threading.Event,
                        out: Dict[str, float]) -> None:
        """Free each bound tensor's device storage as soon as the streamed save has
        published (spilled to host memory) every tile of it, and hand the freed segments back
        to the driver (``empty_cache``) every ~8 GB -- a preempted rank's HBM returns while
        its spill runs, so the driver's clearing of it overlaps the PCIe leg instead of
        delaying the successor's allocations.  Storages shared by several bound tensors go
        when the last of them is covered."""
        import torch

        schedule = self.release_schedule(device_only=True)
        tile = self.plan.tile_bytes
        freed = pending = 0
        i = 0
        while i < len(schedule):
            done = int(progress[0]) * tile
            finished = stop.is_set() and out.get("finish", 0.0) == 1.0
            if stop.is_set() and not finished:  # the save failed: keep the rest
                break
            while i < len(schedule) and (schedule[i][0] <= done or finished):
                st = schedule[i][1]
                nbytes = st.nbytes()
                st.resize_(0)
                freed += nbytes
                pending += nbytes
                i += 1
            if pending >= (8 << 30) or (pending and (i == len(schedule) or stop.is_set())):
                torch.cuda.empty_cache()
                pending = 0
            if i < len(schedule):
                stop.wait(0.002)
        out["released_bytes"] = freed

    def release_schedule(self, device_only: bool = False) -> List[Tuple[int, Any]]:
        """``[(end, storage)]`` in release order: each storage behind the bound tensors with
        the byte offset in the packed stream where its last bound tensor ends -- it may be
        freed once the save has published every tile below that offset."""
        ends: Dict[int, int] = {}
        storages: Dict[int, Any] = {}
        for t, e in zip(self.plan._bound, self.plan.entries):
            if device_only and not getattr(t, "is_cuda", False):
                continue
            st = t.untyped_storage()
            key = st.data_ptr()
            ends[key] = max(ends.get(key, 0), e.offset + e.nbytes)
            storages[key] = st
        return [(ends[k], storages[k]) for k in sorted(ends, key=ends.get)]

    def save(self, metadata: Optional[Dict] = None,
             on_stream: Optional[Any] = None, release_behind: bool = False) -> TransferResult:
        """Pack every tensor into the region; returns bytes/seconds (GB/s via ``.gbps``).

        ``on_stream`` (preemption hand-off): the save first writes a ``streaming`` header and
        a progress block, calls ``on_stream()`` -- which lets the successor start -- and then
        publishes every chunk as it reaches host memory, so :meth:`restore` in the successor
        runs behind the spill over the other direction of the link instead of after it.

        ``release_behind`` (a preempted rank whose state is too big for a successor's copy next
        to it): every bound tensor's device memory is freed as soon as its tiles are in host
        memory (:meth:`_release_behind`); the tensors are unusable afterwards.
        """
        self.wait_pending()
        self._wait_writers()
        slot, generation = self._target()
        self._invalidate(slot)
        zipped = self.codec == "tpz1"
        dst = self.region.addr + slot.base + self.stream_offset
        release_behind = release_behind and self.engine is not None
        streaming = on_stream is not None or release_behind
        if on_stream is None:
            on_stream = lambda: None  # noqa: E731 (the progress block alone)
        releaser = None
        released: Dict[str, float] = {}
        stop_release = threading.Event()
        saved_ok = False
        if streaming:
            prog = slot.progress
            prog[1], prog[2], prog[3], prog[5] = generation, 0, 0, os.getpid()
            prog[4] = STREAM_RUNNING
            prog[0] = PROGRESS_MAGIC
            header = self._header(False, 0, metadata, self.codec, None, generation)
            header["streaming"] = True
            self._write_header(slot, header)
        try:
            if streaming:
                on_stream()
            if self.engine is not None:
                import torch

                wait = torch.cuda.current_stream(self.device_index).cuda_stream
                if streaming:
                    self.engine.set_progress(slot.progress.ctypes.data + 16)
                if release_behind:
                    torch.cuda.current_stream(self.device_index).synchronize()
                    releaser = threading.Thread(
                        target=self._release_behind, name="tpi-release-behind",
                        args=(slot.progress[2:3], stop_release, released), daemon=True)
                    releaser.start()
                try:
                    if zipped:
                        res = self.engine.save_z(self.plan, dst, slot.crcs, slot.csizes, wait)
                    else:
                        res = self.engine.save(self.plan, dst, slot.crcs, self.mode, wait)
                    saved_ok = True
                finally:
                    if streaming:
                        self.engine.set_progress(0)
            else:
                res = self._host_save(slot, zipped)
        except BaseException:
            if streaming:
                slot.progress[4] = STREAM_FAILED
            raise
        finally:
            if releaser is not None:
                # spilled: the rest goes now; failed: what is not in host memory must stay
                released["finish"] = 1.0 if saved_ok else 0.0
                stop_release.set()
                releaser.join()
        res.crc = native().crc32c_combine_tiles_ptr(slot.crcs.ctypes.data, self.plan.ntiles,
                                                     self.plan.tile_bytes, self.plan.total)
        self.saves += 1
        self._write_header(slot, self._header(True, res.crc, metadata, self.codec,
                                              res.wire_bytes, generation))
        if streaming:
            slot.progress[3] = res.wire_bytes
            slot.progress[2] = self.plan.ntiles
            slot.progress[4] = STREAM_COMPLETE
        if releaser is not None:
            res.released_bytes = int(released.get("released_bytes", 0))
        self.last_save = res
        return res

    def _host_save(self, slot: _Slot, zipped: bool) -> TransferResult:
        t0 = time.perf_counter()
        if zipped:
            raw, crcs = host_pack(self.plan)
            blobs, sizes = tpz.encode(raw, self.plan.tile_bytes)
            self.region.array(slot.base + self.stream_offset, len(blobs))[:] = blobs
            slot.csizes[:] = sizes
            wire = len(blobs)
        else:
            stream = self.region.array(slot.base + self.stream_offset, self.plan.total)
            _, crcs = host_pack(self.plan, stream)
            wire = self.plan.total
        slot.crcs[:] = crcs
        return TransferResult(self.plan.total, time.perf_counter() - t0, wire_bytes=wire)

    def save_async(self, metadata: Optional[Dict] = None,
                   codec: Optional[str] = None) -> PendingSave:
        """Checkpoint without stalling the training stream on PCIe.

        The tensors are packed (with tile CRCs) into a snapshot buffer in HBM -- a device-side
        copy at TB/s, ordered on the current stream, which then waits for it, so tensors may
        be updated right after this returns.  A background thread spills the snapshot to the
        host region (TPZ1-encoded when the codec is on) and writes the header; ``result()``
        returns its :class:`TransferResult`.  The snapshot costs ``plan.total`` bytes of HBM
        (allocated on first use).  Host tensors fall back to a synchronous save.  With
        ``slots=2`` the previous checkpoint stays valid for the whole spill.

        ``codec`` overrides the checkpointer's codec for this spill.  A spill next to a
        training loop is a trade: TPZ1 shortens it by ~20 %, but its encode kernels take CU
        time from the loop (a bf16 GEMM loop loses 0.10 s per 32 GB spilled with TPZ1 against
        0.017 s without, ``profiles/async_codec_round3.md``).
        """
        if codec is not None and codec not in ("none", "tpz1"):
            raise ValueError("codec must be 'none' or 'tpz1', not %r" % (codec,))
        self.wait_pending()
        if self.engine is None:
            t0 = time.perf_counter()
            pending = PendingSave(0.0)
            own, self.codec = self.codec, codec or self.codec
            try:
                pending._result = self.save(metadata)
            except BaseException as error:  # surfaced by result()
                pending._error = error
            finally:
                self.codec = own
            pending.stall_s = time.perf_counter() - t0
            pending._done.set()
            return pending
        import torch

        dev = torch.device("cuda", self.device_index)
        if self._snap is None:
            self._snap = torch.empty(self.plan.total, dtype=torch.uint8, device=dev)
            self._snap_crcs = torch.empty(self.plan.ntiles, dtype=torch.int32, device=dev)
        t0 = time.perf_counter()
        self._wait_writers()
        slot, generation = self._target()
        self._invalidate(slot)
        self.engine.snapshot(self.plan, self._snap.data_ptr(), self._snap_crcs.data_ptr(),
                             torch.cuda.current_stream(dev).cuda_stream)
        pending = PendingSave(time.perf_counter() - t0)
        self.saves += 1
        zipped = (codec or self.codec) == "tpz1"

        def spill():
            try:
                res = self.engine.spill(self._snap.data_ptr(), self._snap_crcs.data_ptr(),
                                        self.plan.total,
                                        self.region.addr + slot.base + self.stream_offset,
                                        slot.crcs, slot.csizes, zipped)
                res.crc = native().crc32c_combine_tiles_ptr(
                    slot.crcs.ctypes.data, self.plan.ntiles, self.plan.tile_bytes,
                    self.plan.total)
                self._write_header(slot, self._header(True, res.crc, metadata,
                                                      "tpz1" if zipped else "none",
                                                      res.wire_bytes, generation))
                self.last_save = res
                pending._result = res
            except BaseException as error:  # surfaced by result()
                pending._error = error
            finally:
                pending._done.set()

        pending._thread = threading.Thread(target=spill, name="tpi-spill", daemon=True)
        pending._thread.start()
        self._pending = pending
        return pending

    def rollback(self, strict: bool = True) -> TransferResult:
        """Restore the tensors from the last :meth:`save_async` snapshot still in HBM (device
        to device, CRC-verified) -- e.g. to undo a diverged step without touching PCIe."""
        if self._snap is None:
            raise CheckpointError("no HBM snapshot (save_async was never called)")
        self.wait_pending()
        import torch

        t0 = time.perf_counter()
        bad, first = host_unpack(self.plan, self._snap, self._snap_crcs)
        torch.cuda.current_stream(self.device_index).synchronize()
        res = TransferResult(self.plan.total, time.perf_counter() - t0, 0, bad, first,
                             wire_bytes=0)
        if strict and bad:
            raise CheckpointError("%d corrupt snapshot tile(s), first at %d" % (bad, first))
        return res

    def wait_pending(self) -> None:
        """Block until an asynchronous save in flight has reached host memory."""
        pending, self._pending = self._pending, None
        if pending is not None:
            pending.result()

    def sync(self, metadata: Optional[Dict] = None) -> TransferResult:
        """Incremental save: only tiles whose content changed since the slot being written
        was last synced are packed and spilled (the device-side replacement of the
        reference's 10-second newest-mtime poll + ``rclone sync``, machine-script.sh.tpl:
        118-124).

        A slot's first sync -- and any sync after a full save, async save or load rewrote it
        -- moves every tile; with ``slots=2`` every slot keeps its own tile digests.  Host
        tensors fall back to a full :meth:`save`.
        """
        if self.engine is None:
            res = self.save(metadata)
            res.dirty_tiles = self.plan.ntiles
            return res
        import torch

        self.wait_pending()
        self._wait_writers()
        slot, generation = self._target()
        full = not slot.digests_valid
        self._invalidate(slot)
        if slot.digests is None:
            slot.digests = torch.zeros(self.plan.ntiles, dtype=torch.int64,
                                       device=torch.device("cuda", self.device_index))
        wait = torch.cuda.current_stream(self.device_index).cuda_stream
        res = self.engine.sync(self.plan, self.region.addr + slot.base + self.stream_offset,
                               slot.crcs, full, wait, slot.digests.data_ptr())
        res.crc = native().crc32c_combine_tiles_ptr(slot.crcs.ctypes.data, self.plan.ntiles,
                                                     self.plan.tile_bytes, self.plan.total)
        self.saves += 1
        self._write_header(slot, self._header(True, res.crc, metadata, "none", None, generation))
        slot.digests_valid = True
        self.last_save = res
        return res

    def restore(self, strict: bool = True, stream_timeout: Optional[float] = None,
                generation: Optional[int] = None) -> TransferResult:
        """Unpack + verify the current checkpoint into the bound tensors.  If a preempted
        predecessor is still streaming a newer one into the region, restore that one behind
        its progress (``stream_timeout`` s without progress -> :class:`CheckpointError`;
        default ``TPI_STREAM_TIMEOUT`` or 30).  ``generation`` picks a specific copy (one of
        :meth:`candidates`) instead of the newest."""
        self.wait_pending()
        streaming = self._streaming()
        if streaming is not None and generation in (None, streaming[1].get("generation")):
            if stream_timeout is None:
                stream_timeout = float(os.environ.get("TPI_STREAM_TIMEOUT", "30"))
            return self._restore_streaming(*streaming, strict=strict, timeout=stream_timeout)
        active = self._active()
        if generation is not None:
            active = next(((s, h) for s in self.slots
                           for h in [self._slot_header(s)]
                           if h is not None and h.get("generation") == generation), None)
            if active is None:
                raise CheckpointError("no complete checkpoint of generation %d" % generation)
        if active is None:
            header = self.header()  # raises "no checkpoint" unless an incomplete one is there
            raise CheckpointError("checkpoint incomplete (save was interrupted)")
        slot, header = active
        self._check_compatible(header)
        zipped = header.get("codec", "none") == "tpz1"
        src = self.region.addr + slot.base + self.stream_offset
        if self.engine is not None:
            import torch

            sig = torch.cuda.current_stream(self.device_index).cuda_stream
            if zipped:
                res = self.engine.restore_z(self.plan, src, slot.crcs, slot.csizes, sig)
            else:
                res = self.engine.restore(self.plan, src, slot.crcs, self.mode, sig)
        else:
            t0 = time.perf_counter()
            if zipped:
                nbytes = int(header["stream_bytes"])
                stream, _ = tpz.decode(
                    self.region.array(slot.base + self.stream_offset, nbytes),
                    slot.csizes, self.plan.total, self.plan.tile_bytes)
            else:
                nbytes = self.plan.total
                stream = self.region.array(slot.base + self.stream_offset, self.plan.total)
            bad, first = host_unpack(self.plan, stream, slot.crcs)
            res = TransferResult(self.plan.total, time.perf_counter() - t0, 0, bad, first,
                                 wire_bytes=nbytes)
        res.crc = int(header.get("crc32c", 0))
        self.last_restore = res
        if strict and res.bad_tiles:
            raise CheckpointError("%d corrupt tile(s), first at %d" % (res.bad_tiles,
                                                                      res.first_bad))
        return res

    def _restore_streaming(self, slot: _Slot, header: Dict, strict: bool,
                           timeout: float) -> TransferResult:
        self._check_compatible(header)
        zipped = header.get("codec", "none") == "tpz1"
        prog = slot.progress
        if self.engine is not None:
            import torch

            from ..ops._loader import HipError

            sig = torch.cuda.current_stream(self.device_index).cuda_stream
            try:
                res = self.engine.restore_stream(
                    self.plan, self.region.addr + slot.base + self.stream_offset, slot.crcs,
                    slot.csizes if zipped else None, prog.ctypes.data + 16, timeout, sig)
            except HipError as error:  # stalled / failed writer: no usable checkpoint here
                raise CheckpointError(str(error)) from error
        else:  # host tensors: wait for the whole spill, then the ordinary restore
            last, seen = time.monotonic(), -1
            while int(prog[4]) != STREAM_COMPLETE:
                if int(prog[4]) == STREAM_FAILED:
                    raise CheckpointError("the streamed checkpoint failed in its writer")
                if int(prog[2]) != seen:
                    seen, last = int(prog[2]), time.monotonic()
                elif time.monotonic() - last > timeout:
                    raise CheckpointError("streamed checkpoint stalled (writer gone?)")
                time.sleep(0.001)
            return self.restore(strict)
        res.crc = native().crc32c_combine_tiles_ptr(slot.crcs.ctypes.data, self.plan.ntiles,
                                                     self.plan.tile_bytes, self.plan.total)
        self.last_restore = res
        if strict and res.bad_tiles:
            raise CheckpointError("%d corrupt tile(s), first at %d" % (res.bad_tiles,
                                                                      res.first_bad))
        return res

    # -- progressive materialisation: allocate the state while it streams in -----------------
    @classmethod
    def materialize(cls, path: str, device: Any = None, *, group_bytes: int = 4 << 30,
                    stream_timeout: Optional[float] = None,
                    memory_timeout: Optional[float] = None,
                    **kwargs) -> Tuple["Checkpointer", Dict[str, Any], TransferResult]:
        """Create the tensors a checkpoint region holds and restore them, group by group.

        For a successor whose state does not fit next to its predecessor's on one GPU (a
        170 GB rank on 288 GB of HBM): instead of allocating the whole state up front -- which
        waits until the predecessor has spilled *and* freed all of it -- each group of about
        ``group_bytes`` is allocated as soon as the device has room for it (a background
        thread retries the allocation while the predecessor frees its tensors behind its
        spill, ``save(release_behind=True)``) and restored at once, behind the predecessor's
        streamed save when one is still running.  Allocation, the driver's clearing of the
        freed HBM, the spill and the restore then overlap instead of running one after the
        other.  Tensors come back contiguous, with the saved names, shapes and dtypes; the
        returned checkpointer is bound to them (later saves go to the same region).
        ``device`` may be ``"cpu"`` (host tensors, complete checkpoints only).
        ``memory_timeout`` (default ``TPI_STREAM_TIMEOUT`` or 30 s): give up when no
        allocation has succeeded for that long.  Returns ``(checkpointer, tensors, result)``.
        """
        import torch

        t0 = time.perf_counter()
        layout = _region_layout(path)
        dev = torch.device(device if device is not None else "cuda")
        if dev.type == "cuda" and dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        entries = [TensorEntry.from_json(e) for e in layout["entries"]]
        plan = PackPlan.from_entries(entries, layout["total"], layout["tile_bytes"])
        plan.device = str(dev)
        plan._bound = []
        kwargs.setdefault("codec", layout["codec"])
        t1 = time.perf_counter()
        ck = cls(None, path, tile_bytes=layout["tile_bytes"], slots=layout["slots"], _plan=plan,
                 **kwargs)
        try:
            if ck._entries_digest != layout["entries_sha256"] or ck.size != layout["size"]:
                raise CheckpointError("%s: region layout not reproducible from its entries"
                                      % path)
            t2 = time.perf_counter()
            if ck.engine is not None:  # before the predecessor's freeing makes hipMalloc slow
                ck.engine.reserve(len(entries) + 1, plan.ntiles, layout["codec"] == "tpz1")
                # TPI_MATERIALIZE_H2D=sdma: the restore's host-to-device copies on an SDMA
                # engine of their own (profiles/round4/materialize_170g.md)
                ck.h2d_engine = ck.engine.set_h2d_sdma(
                    os.environ.get("TPI_MATERIALIZE_H2D", "hip") == "sdma")
            ck._setup_times = {"layout": round(t1 - t0, 4), "checkpointer": round(t2 - t1, 4),
                               "reserve": round(time.perf_counter() - t2, 4)}
            tensors, res = ck._materialize(dev, group_bytes, stream_timeout, memory_timeout)
        except BaseException:
            ck.close()
            raise
        return ck, tensors, res

    def _groups(self, group_bytes: int) -> List[Tuple[int, int]]:
        """Entry index ranges ``[lo, hi)`` of about ``group_bytes`` each, in stream order."""
        out, lo, acc = [], 0, 0
        for i, e in enumerate(self.plan.entries):
            acc += e.nbytes
            if acc >= group_bytes or i == len(self.plan.entries) - 1:
                out.append((lo, i + 1))
                lo, acc = i + 1, 0
        return out

    def _sub_plan(self, lo: int, hi: int, tensors: Sequence[Any],
                  lead: Any) -> Tuple[PackPlan, int, int]:
        """(plan, first tile, end tile) of entries ``[lo, hi)``: the tiles that hold them, the
        plan's offsets relative to the first tile.  Neighbouring groups may share a boundary
        tile; each restore scatters only its own tensors from it.  The bytes of the first tile
        before the group's first tensor (the previous group's tail) land in ``lead``, a
        scratch buffer of one tile: the device kernels need a segment at offset 0."""
        tile = self.plan.tile_bytes
        group = self.plan.entries[lo:hi]
        ta = group[0].offset // tile
        tb = min(self.plan.ntiles, -(-(group[-1].offset + group[-1].nbytes) // tile))
        base = ta * tile
        entries = [TensorEntry(e.name, e.dtype, e.shape, e.nbytes, e.offset - base)
                   for e in group]
        named = {e.name: t for e, t in zip(group, tensors)}
        gap = group[0].offset - base
        if gap:
            entries.insert(0, TensorEntry("\0lead", "uint8", (gap,), gap, 0))
            named = dict([("\0lead", lead[:gap])] + list(named.items()))
        sub = PackPlan.from_entries(entries, min(self.plan.total, tb * tile) - base, tile)
        sub.bind(named)
        return sub, ta, tb

    def _materialize(self, dev, group_bytes: int, stream_timeout: Optional[float],
                     memory_timeout: Optional[float]) -> Tuple[Dict[str, Any], TransferResult]:
        import torch

        t_start = time.perf_counter()
        self.wait_pending()
        found = self._streaming()
        streaming = found is not None
        if found is None:
            found = self._active()
        if found is None:
            raise CheckpointError("no checkpoint to materialize in %s" % self.path)
        slot, header = found
        self._check_compatible(header)
        early_fallback = None
        if streaming and self.engine is None:
            streaming = False  # host tensors: wait for the whole spill first
            try:
                self._restore_streaming_wait(slot, stream_timeout)
                header = self._slot_header(slot) or header
            except CheckpointError as error:  # a two-slot region's older copy, if any
                older = self._active()
                if older is None:
                    raise
                slot, header = older
                early_fallback = str(error)
        zipped = header.get("codec", "none") == "tpz1"
        if stream_timeout is None:
            stream_timeout = float(os.environ.get("TPI_STREAM_TIMEOUT", "30"))
        if memory_timeout is None:
            memory_timeout = float(os.environ.get("TPI_STREAM_TIMEOUT", "30"))
        entries = self.plan.entries
        groups = self._groups(max(1, int(group_bytes)))
        ready: "queue.Queue[Any]" = queue.Queue()
        stop = threading.Event()
        waited = [0.0]
        # per group, seconds from the start: [allocation start, allocated, restore start, end]
        trace: List[List[float]] = []

        # torch.empty() holds the GIL while the driver clears just-freed HBM (seconds behind a
        # big spill), which would stall the restoring thread at its next Python step: allocate
        # through _tpi_torch.empty (the same caching-allocator call, GIL released) when built
        try:
            from ..ops._loader import torch_ext

            empty_nogil = torch_ext().empty
        except Exception:  # not built: torch.empty (correct, restores may stall behind it)
            empty_nogil = None
        likes: Dict[str, Any] = {}

        def empty(e: TensorEntry):
            dtype = getattr(torch, e.dtype)
            if empty_nogil is None:
                return torch.empty(e.shape, dtype=dtype, device=dev)
            like = likes.get(e.dtype)
            if like is None:
                like = likes[e.dtype] = torch.empty(0, dtype=dtype, device=dev)
            return empty_nogil(list(e.shape), like)

        restored = [0]  # groups restored so far (the main thread counts)
        # groups that fit in the HBM free right now are allocated at once; the rest -- memory
        # the predecessor has yet to free -- only ALLOC_LOOKAHEAD groups ahead of the restore:
        # by then that memory has long been freed, and its hipMalloc does not block the
        # restore's copies (see the gate below)
        budget = (torch.cuda.mem_get_info(dev)[0] - ALLOC_HEADROOM) if dev.type == "cuda" \
            else float("inf")
        upfront = 0
        for lo, hi in groups:
            size = sum(e.nbytes for e in entries[lo:hi])
            if size > budget:
                break
            budget -= size
            upfront += 1

        lookahead = int(os.environ.get("TPI_ALLOC_LOOKAHEAD", ALLOC_LOOKAHEAD))

        def allocate():  # runs ahead of the restores, as far as the device has room
            try:
                if dev.type == "cuda":
                    torch.cuda.set_device(dev)
                for gi, (lo, hi) in enumerate(groups):
                    while (gi >= upfront and restored[0] + lookahead < gi
                           and not stop.is_set()):
                        stop.wait(0.002)
                    out = []
                    t_group = time.perf_counter()
                    for e in entries[lo:hi]:
                        last = time.monotonic()
                        while True:
                            if stop.is_set():
                                return
                            # ask before allocating: a hipMalloc that has to wait for memory
                            # the predecessor is still freeing blocks for up to a second
                            # inside the HIP runtime, and holds up this process's
                            # hipMemcpyAsync calls -- the restore's -- all that time (HIP API
                            # trace, profiles/round4/materialize_170g.md)
                            if (dev.type == "cuda" and time.monotonic() - last <= memory_timeout
                                    and torch.cuda.mem_get_info(dev)[0]
                                    < e.nbytes + ALLOC_HEADROOM):
                                t = time.monotonic()
                                stop.wait(0.002)
                                waited[0] += time.monotonic() - t
                                continue
                            try:
                                out.append(empty(e))
                                break
                            except RuntimeError as error:  # torch's OOM error included
                                if "out of memory" not in str(error).lower():
                                    raise
                                # the predecessor is still freeing (behind its spill)
                                if time.monotonic() - last > memory_timeout:
                                    raise CheckpointError(
                                        "no room for %s (%.1f GB) within %.0f s" % (
                                            e.name, e.nbytes / 1e9, memory_timeout))
                                t = time.monotonic()
                                stop.wait(0.002)
                                waited[0] += time.monotonic() - t
                    trace.append([round(t_group - t_start, 4),
                                  round(time.perf_counter() - t_start, 4)])
                    ready.put(out)
            except BaseException as error:  # surfaced by the restoring thread
                ready.put(error)

        t_lead = time.perf_counter()
        lead = torch.empty(self.plan.tile_bytes, dtype=torch.uint8, device=dev)
        setup = dict(getattr(self, "_setup_times", {}), lead=round(time.perf_counter() - t_lead, 4),
                     find=round(t_lead - t_start, 4))
        worker = threading.Thread(target=allocate, name="tpi-materialize-alloc", daemon=True)
        worker.start()
        tensors: Dict[str, Any] = {}
        total = TransferResult(self.plan.total, 0.0, wire_bytes=0)
        src = {"slot": slot, "header": header, "zipped": zipped, "streaming": streaming}
        done: List[Tuple[int, int, List[Any]]] = []  # restored groups, for a fallback
        fallback = early_fallback

        def restore_group(lo: int, hi: int, item: List[Any]) -> TransferResult:
            slot, zipped = src["slot"], src["zipped"]
            sub, ta, tb = self._sub_plan(lo, hi, item, lead)
            crcs = slot.crcs[ta:tb]
            csizes = slot.csizes[ta:tb] if zipped else None
            # earlier tiles are in host memory: the previous group waited for them
            start = int(slot.csizes[:ta].sum(dtype=np.uint64)) if zipped \
                else ta * self.plan.tile_bytes
            stream_base = self.region.addr + slot.base + self.stream_offset
            if self.engine is not None:
                sig = torch.cuda.current_stream(dev).cuda_stream
                if src["streaming"]:
                    from ..ops._loader import HipError

                    try:
                        res = self.engine.restore_stream(
                            sub, stream_base + start, crcs, csizes,
                            slot.progress.ctypes.data + 16, stream_timeout, sig, tile_base=ta)
                    except HipError as error:
                        raise CheckpointError(str(error)) from error
                elif zipped:
                    res = self.engine.restore_z(sub, stream_base + start, crcs, csizes, sig)
                else:
                    res = self.engine.restore(sub, stream_base + start, crcs, self.mode, sig)
            else:
                t0 = time.perf_counter()
                if zipped:
                    nbytes = int(csizes.sum(dtype=np.uint64))
                    stream, _ = tpz.decode(self.region.array(
                        slot.base + self.stream_offset + start, nbytes),
                        csizes, sub.total, self.plan.tile_bytes)
                else:
                    nbytes = sub.total
                    stream = self.region.array(slot.base + self.stream_offset + start,
                                               sub.total)
                bad, first = host_unpack(sub, stream, crcs)
                res = TransferResult(sub.total, time.perf_counter() - t0, 0, bad, first,
                                     wire_bytes=nbytes)
            if res.bad_tiles:
                res.first_bad += ta
            return res

        try:
            for gi, (lo, hi) in enumerate(groups):
                item = ready.get()
                if isinstance(item, BaseException):
                    raise item
                t_group = time.perf_counter()
                try:
                    res = restore_group(lo, hi, item)
                except CheckpointError as error:
                    # the predecessor's streamed save failed (or its writer died): fall back
                    # to the complete copy a two-slot region still holds -- every group
                    # again, so the state is one generation throughout
                    older = self._active() if src["streaming"] else None
                    if older is None:
                        raise
                    self._check_compatible(older[1])
                    fallback = str(error)
                    src.update(slot=older[0], header=older[1], streaming=False,
                               zipped=older[1].get("codec", "none") == "tpz1")
                    total = TransferResult(self.plan.total, 0.0, wire_bytes=0)
                    for lo2, hi2, item2 in done:
                        again = restore_group(lo2, hi2, item2)
                        total.chunks += again.chunks
                        total.wire_bytes += again.wire_bytes
                        if again.bad_tiles:
                            total.bad_tiles += again.bad_tiles
                            total.first_bad = again.first_bad if total.first_bad < 0 \
                                else total.first_bad
                    res = restore_group(lo, hi, item)
                total.chunks += res.chunks
                total.wire_bytes += res.wire_bytes
                if res.bad_tiles:
                    total.bad_tiles += res.bad_tiles
                    if total.first_bad < 0:
                        total.first_bad = res.first_bad
                done.append((lo, hi, item))
                for e, t in zip(entries[lo:hi], item):
                    tensors[e.name] = t
                restored[0] = gi + 1
                trace[gi] += [
                    round(t_group - t_start, 4), round(time.perf_counter() - t_start, 4)]
        finally:
            stop.set()
            worker.join()
        slot, header, streaming = src["slot"], src["header"], src["streaming"]
        self.plan.bind(tensors)
        total.seconds = time.perf_counter() - t_start
        total.crc = int(header.get("crc32c", 0)) if not streaming else \
            native().crc32c_combine_tiles_ptr(slot.crcs.ctypes.data, self.plan.ntiles,
                                              self.plan.tile_bytes, self.plan.total)
        self.materialize_stats = {"groups": len(groups), "upfront_groups": upfront,
                                  "alloc_wait_s": round(waited[0], 4),
                                  "streamed": streaming, "trace": trace, "setup": setup,
                                  "fallback": fallback,
                                  "h2d_engine": getattr(self, "h2d_engine", None),
                                  "alloc": "nogil" if empty_nogil is not None else "torch"}
        self.materialized_metadata = header.get("metadata", {})
        self.last_restore = total
        if total.bad_tiles:
            raise CheckpointError("%d corrupt tile(s), first at %d" % (total.bad_tiles,
                                                                      total.first_bad))
        return tensors, total

    def _restore_streaming_wait(self, slot: _Slot, timeout: Optional[float]) -> None:
        """Host path of a streamed checkpoint: wait until its writer completed it."""
        if timeout is None:
            timeout = float(os.environ.get("TPI_STREAM_TIMEOUT", "30"))
        prog = slot.progress
        last, seen = time.monotonic(), -1
        while int(prog[4]) != STREAM_COMPLETE:
            if int(prog[4]) == STREAM_FAILED:
                raise CheckpointError("the streamed checkpoint failed in its writer")
            if int(prog[2]) != seen:
                seen, last = int(prog[2]), time.monotonic()
            elif time.monotonic() - last > timeout:
                raise CheckpointError("streamed checkpoint stalled (writer gone?)")
            time.sleep(0.001)

    # -- HBM-to-HBM hand-off (preemption on the same GPU) --------------------------------------
    def _hbm_manifest_path(self) -> Optional[str]:
        return self.path + ".hbm" if self.path and self.engine is not None else None

    def export_hbm(self, metadata: Optional[Dict] = None) -> Optional[str]:
        """Preempted rank: publish the bound tensors' device allocations next to the spill
        file (``<path>.hbm``), so a successor on the same GPU can copy the state device to
        device (:meth:`restore_hbm`) while this process is still spilling it to host memory.
        The caller must keep the tensors unchanged (and this process alive) until the successor
        has restored -- the preemption handler does (it lingers until ``closed``).

        Allocations travel as HIP IPC handles in the manifest; how those of ``IPC_MAX_ALLOC``
        or more travel depends on ``TPI_HBM_ROUTE`` (:data:`HBM_ROUTES`): relocated into plain
        blocks (default), as dma-buf descriptors, or not at all (CheckpointError, nothing
        written: the successor restores from the host copy).  ``metadata``: that of the save
        this export accompanies; a successor resuming from the HBM gets it even when the host
        copy failed."""
        manifest = self._hbm_manifest_path()
        if manifest is None:
            return None
        import torch

        torch.cuda.synchronize(self.device_index)  # no queued kernel may still write them
        lib = hip()
        route = os.environ.get("TPI_HBM_ROUTE", "auto").strip().lower()
        if route not in HBM_ROUTES:
            raise CheckpointError("TPI_HBM_ROUTE must be one of %s" % (HBM_ROUTES,))
        limit = int(os.environ.get("TPI_IPC_MAX_ALLOC", IPC_MAX_ALLOC))
        sizes: Dict[int, int] = {}  # allocation base -> size
        raw_where: List[Optional[Tuple[int, int]]] = []  # (allocation base, offset) per segment
        base, size = ctypes.c_uint64(0), ctypes.c_uint64(0)
        for seg in self.plan.segs:
            ptr = int(seg["ptr"])
            if int(seg["nbytes"]) == 0 or ptr == 0:
                raw_where.append(None)
                continue
            # one handle per allocation (tensors of one caching-allocator segment share it)
            lib.check(lib.tpi_mem_range(ctypes.c_void_p(ptr), ctypes.byref(base),
                                        ctypes.byref(size)), "tpi_mem_range")
            sizes.setdefault(int(base.value), int(size.value))
            raw_where.append((int(base.value), ptr - int(base.value)))
        big = {key for key, sz in sizes.items() if sz >= limit}
        if big and (route == "ipc" or (route == "dmabuf" and not lib.tpi_dmabuf_available())):
            raise CheckpointError(
                "no HBM hand-off: %d allocation(s) of %.2f GiB or more (the largest %.2f GiB), "
                "and HIP IPC imports of such allocations never return (TPI_IPC_MAX_ALLOC); the "
                "successor restores from the host copy" % (
                    len(big), limit / 2 ** 30, max(sizes[k] for k in big) / 2 ** 30))
        pieces: Dict[str, List[List[int]]] = {}
        if big and route == "auto":
            pieces = self._relocate(raw_where, big)  # segment -> [[block base, 0, n], ...]
        # the allocations the successor maps, in order
        keys: List[int] = []
        index: Dict[int, int] = {}

        def idx(key: int) -> int:
            if key not in index:
                index[key] = len(keys)
                keys.append(key)
            return index[key]

        where: List[Optional[List[int]]] = []
        for si, w in enumerate(raw_where):
            if w is None or str(si) in pieces:
                where.append(None)
            else:
                where.append([idx(w[0]), w[1]])
        for si in pieces:
            pieces[si] = [[idx(p[0]), p[1], p[2]] for p in pieces[si]]
        alloc_sizes = [sizes.get(k) or self._relocated_size[k] for k in keys]
        as_dmabuf = [i for i, k in enumerate(keys) if k in big] if route == "dmabuf" else []
        doc = {"format": "tpi-hbm-2", "pid": os.getpid(),
               "entries_sha256": self._entries_digest, "total": self.plan.total,
               "tile_bytes": self.plan.tile_bytes, "where": where, "pieces": pieces,
               "segs": self.plan.segs.tobytes().hex(), "created": time.time(),
               "metadata": metadata or {}, "allocations": alloc_sizes,
               # the generation the save that follows this export will write
               "generation": self._target()[1]}
        handle = ctypes.create_string_buffer(64)
        offset = ctypes.c_uint64(0)
        ipc: Dict[str, str] = {}
        dmabuf_set = set(as_dmabuf)
        for i, key in enumerate(keys):
            if i in dmabuf_set:
                continue
            lib.check(lib.tpi_ipc_export(ctypes.c_void_p(key), handle, ctypes.byref(offset),
                                         ctypes.byref(size)), "tpi_ipc_export")
            ipc[str(i)] = handle.raw.hex()
        doc["ipc"] = ipc
        if as_dmabuf:
            doc["socket"], doc["dmabuf"] = self._serve_dmabufs(
                [(i, keys[i], alloc_sizes[i]) for i in as_dmabuf])
        bus = ctypes.create_string_buffer(64)
        lib.tpi_device_pci_bus_id(self.device_index, bus, 64)
        doc["device"] = bus.value.decode()
        tmp = manifest + ".tmp"
        with open(tmp, "w") as handle_file:
            json.dump(doc, handle_file)
        os.replace(tmp, manifest)
        return manifest

    def _relocate(self, raw_where: List[Optional[Tuple[int, int]]],
                  big: set) -> Dict[str, List[List[int]]]:
        """Copy every tensor living in one of the ``big`` allocations (HIP IPC cannot open
        them) into plain hipMalloc blocks of at most ``RELOCATE_CHUNK`` bytes, device to
        device; returns, per segment index, its pieces ``[block base, 0, bytes]`` in stream
        order.  The blocks stay allocated until this process exits (the successor maps them).
        Raises CheckpointError when such a tensor is not contiguous or the device has no room
        for the copies -- the successor then restores from the host copy."""
        import torch

        lib = hip()
        todo = [si for si, w in enumerate(raw_where) if w is not None and w[0] in big]
        need = sum(int(self.plan.segs[si]["nbytes"]) for si in todo)
        free, _ = torch.cuda.mem_get_info(self.device_index)
        from ..parallel.placement import device_vram_usage

        usage = device_vram_usage(self.device_index)  # the driver's count (delayed frees)
        if usage is not None:
            free = min(free, usage[1] - usage[0])
        if free < need + (1 << 30):
            raise CheckpointError("no HBM hand-off: relocating %.2f GB out of allocations HIP "
                                  "IPC cannot open needs that much free HBM (%.2f GB free)"
                                  % (need / 1e9, free / 1e9))
        blocks: List[int] = []
        self._relocated_size: Dict[int, int] = getattr(self, "_relocated_size", {})
        self._relocated = getattr(self, "_relocated", [])
        out: Dict[str, List[List[int]]] = {}
        stream = torch.cuda.current_stream(self.device_index).cuda_stream
        ptr = ctypes.c_void_p()
        try:
            for si in todo:
                seg = self.plan.segs[si]
                if int(seg["kind"]) != SEG_CONTIG:
                    raise CheckpointError(
                        "no HBM hand-off: a non-contiguous tensor lives in an allocation HIP "
                        "IPC cannot open")
                nbytes, src = int(seg["nbytes"]), int(seg["ptr"])
                parts = []
                for k in range(0, nbytes, RELOCATE_CHUNK):
                    n = min(RELOCATE_CHUNK, nbytes - k)
                    lib.check(lib.tpi_dev_alloc(n, ctypes.byref(ptr)), "tpi_dev_alloc")
                    blocks.append(ptr.value)
                    lib.check(lib.tpi_d2d(ptr, ctypes.c_void_p(src + k), n, stream), "tpi_d2d")
                    self._relocated_size[ptr.value] = n
                    parts.append([ptr.value, 0, n])
                out[str(si)] = parts
        except BaseException:
            for b in blocks:
                lib.tpi_dev_free(ctypes.c_void_p(b))
            raise
        self._relocated.extend(blocks)
        return out

    def _serve_dmabufs(self, allocs: List[Tuple[int, int, int]]) -> Tuple[str, Dict[str, Any]]:
        """Export every ``(index, base, size)`` allocation as a dma-buf and serve the
        descriptors, in order, to each process of this uid that connects to the returned
        abstract socket name (messages of up to ``FDS_PER_MESSAGE`` descriptors:
        ``{"index", "offsets"}`` + fds, then ``{"end": n}``).  Returns the name and, per
        allocation index, the exported buffer's size and offset (checked against the
        allocation here and again by the importer).  A daemon thread serves as long as this
        process lives."""
        lib = hip()
        fds: List[int] = []
        offsets: List[int] = []
        info: Dict[str, Any] = {}
        fd, off = ctypes.c_int(-1), ctypes.c_uint64(0)
        try:
            for i, key, sz in allocs:
                lib.check(lib.tpi_dmabuf_export(ctypes.c_void_p(key), sz, ctypes.byref(fd),
                                                ctypes.byref(off)), "tpi_dmabuf_export")
                fds.append(fd.value)
                offsets.append(int(off.value))
                buf = os.lseek(fd.value, 0, os.SEEK_END)  # a dma-buf's size
                os.lseek(fd.value, 0, os.SEEK_SET)
                if buf < int(off.value) + sz:
                    raise CheckpointError(
                        "dma-buf export of allocation %d (%d bytes at %#x) gave a %d-byte "
                        "buffer at offset %d" % (i, sz, key, buf, int(off.value)))
                info[str(i)] = [buf, int(off.value)]
        except BaseException:
            for f in fds:
                os.close(f)
            raise
        index = [i for i, _, _ in allocs]
        name = "tpi-hbm-%d-%s" % (os.getpid(), os.urandom(6).hex())
        server = socket.socket(socket.AF_UNIX, socket.SOCK_SEQPACKET)
        server.bind("\0" + name)
        server.listen(4)
        uid = os.getuid()

        def serve() -> None:
            while True:
                try:
                    conn, _ = server.accept()
                except OSError:
                    return
                try:
                    cred = conn.getsockopt(socket.SOL_SOCKET, socket.SO_PEERCRED,
                                           struct.calcsize("3i"))
                    if struct.unpack("3i", cred)[1] != uid:
                        continue  # another user's process: nothing to see
                    for k in range(0, len(fds), FDS_PER_MESSAGE):
                        chunk = fds[k:k + FDS_PER_MESSAGE]
                        msg = json.dumps({"index": index[k:k + len(chunk)],
                                          "offsets": offsets[k:k + len(chunk)]})
                        socket.send_fds(conn, [msg.encode()], chunk)
                    conn.send(json.dumps({"end": len(fds)}).encode())
                except OSError:
                    pass
                finally:
                    conn.close()

        self._dmabuf_server = (server, fds)
        threading.Thread(target=serve, name="tpi-dmabuf-serve", daemon=True).start()
        return name, info

    def _close_dmabuf_server(self) -> None:
        served = getattr(self, "_dmabuf_server", None)
        if served is None:
            return
        self._dmabuf_server = None
        server, fds = served
        try:
            server.shutdown(socket.SHUT_RDWR)
        except OSError:
            pass
        server.close()
        for f in fds:
            try:
                os.close(f)
            except OSError:
                pass

    def _hbm_doc(self) -> Optional[Dict]:
        manifest = self._hbm_manifest_path()
        if manifest is None or not os.path.exists(manifest):
            return None
        try:
            with open(manifest) as f:
                doc = json.load(f)
        except (OSError, ValueError):
            return None
        if (doc.get("format") != "tpi-hbm-2" or doc.get("pid") == os.getpid()
                or doc.get("entries_sha256") != self._entries_digest
                or doc.get("total") != self.plan.total):
            return None
        try:
            os.kill(int(doc["pid"]), 0)  # the exporting process must still hold the memory
        except (OSError, ValueError):
            return None
        bus = ctypes.create_string_buffer(64)
        hip().tpi_device_pci_bus_id(self.device_index, bus, 64)
        if doc.get("device") != bus.value.decode():
            return None  # another GPU: the host region is the way
        return doc

    def hbm_ready(self) -> bool:
        """A live predecessor on this GPU exported its tensors for :meth:`restore_hbm`."""
        return self._hbm_doc() is not None

    def hbm_metadata(self) -> Optional[Dict]:
        """``{"generation", "metadata"}`` of the live predecessor's exported state (None: no
        hand-off)."""
        doc = self._hbm_doc()
        if doc is None:
            return None
        return {"generation": doc.get("generation"), "metadata": dict(doc.get("metadata") or {})}

    # The hand-off claim (``<path>.hbm.claim``, one pid): whoever creates it first owns the
    # exported memory's fate.  A successor claims before it reads the manifest and removes its
    # claim only after every IPC mapping is closed; a predecessor that wants to exit claims it
    # itself, after which no successor can import (it falls back to the host copy).  So the
    # exporter never exits while its memory is imported, whatever the supervisor does.
    def _hbm_claim_path(self) -> Optional[str]:
        manifest = self._hbm_manifest_path()
        return manifest + ".claim" if manifest else None

    def hbm_claim_owner(self) -> Optional[int]:
        """pid holding the hand-off claim (None: unclaimed)."""
        path = self._hbm_claim_path()
        if path is None:
            return None
        try:
            with open(path) as f:
                return int(f.read().strip() or 0)
        except (OSError, ValueError):
            return None

    def claim_hbm(self) -> bool:
        """Take the hand-off claim for this process (a stale claim of a dead process is taken
        over); False when another live process holds it."""
        path = self._hbm_claim_path()
        if path is None:
            return False
        # The claim appears with its pid already in it: the pid goes into a private file that
        # is then hard-linked to the claim path (link fails if the claim exists).  A reader
        # can therefore never see an empty claim and take it for a dead holder's.
        tmp = "%s.%d.tmp" % (path, os.getpid())
        with open(tmp, "w") as f:
            f.write(str(os.getpid()))
        try:
            for _ in range(3):
                try:
                    os.link(tmp, path)
                    return True
                except FileExistsError:
                    owner = self.hbm_claim_owner()
                    if owner == os.getpid():
                        return True
                    if owner is None:
                        continue  # released in between: try again
                    if owner == 0 or _writer_alive(owner):
                        # empty (never produced by this writer; treated as being written) or
                        # a live holder: the claim is taken
                        return False
                    try:  # its holder died: the claim is void
                        os.remove(path)
                    except OSError:
                        pass
            return False
        finally:
            try:
                os.remove(tmp)
            except OSError:
                pass

    def release_hbm_claim(self) -> None:
        """Drop this process's claim (after its IPC mappings are closed)."""
        if self.hbm_claim_owner() == os.getpid():
            try:
                os.remove(self._hbm_claim_path())
            except OSError:
                pass

    def restore_hbm(self, strict: bool = True) -> TransferResult:
        """Copy the state of a preempted predecessor on the same GPU straight from its HBM
        (its allocations mapped here over dma-buf, or HIP IPC for an ``ipc`` export; one
        fused copy pass + a read-back verify, every tile's digest checked) into the bound
        tensors."""
        if not self.claim_hbm():
            raise CheckpointError("the HBM hand-off is claimed by another process (withdrawn "
                                  "by its exporter, or taken by another successor)")
        doc = self._hbm_doc()
        if doc is None:
            self.release_hbm_claim()
            raise CheckpointError("no HBM hand-off from a live predecessor on this GPU")
        import torch

        lib = hip()
        n = len(doc["allocations"])
        ipc = {int(i): h for i, h in (doc.get("ipc") or {}).items()}
        sizes = [int(x) for x in doc["allocations"]]
        bases: List[Optional[int]] = [None] * n   # each allocation's base in this process
        mapped: List[Optional[int]] = [None] * n  # what to unmap / close
        via_dmabuf = [False] * n
        t0 = time.perf_counter()
        try:
            limit = float(os.environ.get("TPI_IPC_OPEN_TIMEOUT", "10"))
        except ValueError:
            limit = 10.0

        def open_ipc(i: int) -> None:
            base = ctypes.c_void_p()
            lib.check(lib.tpi_ipc_open(bytes.fromhex(ipc[i]), self.device_index,
                                       ctypes.byref(base)), "tpi_ipc_open")
            bases[i] = mapped[i] = base.value

        def open_dmabufs() -> None:
            # the predecessor's server sends the descriptors in batches; each is checked
            # (size), mapped here and closed at once (the mapping keeps its own reference)
            sock = socket.socket(socket.AF_UNIX, socket.SOCK_SEQPACKET)
            sock.settimeout(limit)
            ptr, size = ctypes.c_void_p(), ctypes.c_uint64(0)
            want = doc.get("dmabuf") or {}
            got = 0
            with sock:
                sock.connect("\0" + doc["socket"])
                while True:
                    msg, fds, _, _ = socket.recv_fds(sock, 1 << 16, FDS_PER_MESSAGE)
                    try:
                        if not msg:
                            raise CheckpointError("the predecessor closed the hand-off socket")
                        head = json.loads(msg)
                        if "end" in head:
                            if head["end"] != len(want) or got != len(want):
                                raise CheckpointError("hand-off socket sent %s of %d "
                                                      "dma-bufs" % (head["end"], len(want)))
                            return
                        if len(fds) != len(head["index"]):
                            raise CheckpointError("hand-off message lost descriptors")
                        for k, fd in enumerate(fds):
                            i = int(head["index"][k])
                            off = int(head["offsets"][k])
                            buf = os.lseek(fd, 0, os.SEEK_END)
                            if buf < off + sizes[i] or [buf, off] != want.get(str(i)):
                                raise CheckpointError(
                                    "dma-buf for allocation %d is %d bytes at offset %d; the "
                                    "exporter announced %s for %d bytes" % (
                                        i, buf, off, want.get(str(i)), sizes[i]))
                            lib.check(lib.tpi_dmabuf_import(self.device_index, fd,
                                                            ctypes.byref(ptr),
                                                            ctypes.byref(size)),
                                      "tpi_dmabuf_import")
                            mapped[i] = ptr.value
                            via_dmabuf[i] = True
                            if int(size.value) < off + sizes[i]:
                                # never let a kernel read past what was mapped
                                raise CheckpointError(
                                    "dma-buf %d maps %d bytes, the allocation needs %d" % (
                                        i, int(size.value), off + sizes[i]))
                            bases[i] = ptr.value + off
                            got += 1
                    finally:
                        for fd in fds:
                            os.close(fd)

        def close_one(i: int) -> None:
            if mapped[i] is not None:
                if via_dmabuf[i]:
                    lib.tpi_dmabuf_unmap(ctypes.c_void_p(mapped[i]))
                else:
                    lib.tpi_ipc_close(ctypes.c_void_p(mapped[i]))
                mapped[i] = bases[i] = None

        def each(fn) -> None:
            # one mapping per predecessor allocation (a model's state is hundreds of them);
            # opens and closes are independent driver calls, so 8 threads overlap them
            if n > 8:
                from concurrent.futures import ThreadPoolExecutor

                with ThreadPoolExecutor(8) as pool:
                    list(pool.map(fn, range(n)))
            else:
                for i in range(n):
                    fn(i)

        def close_all() -> None:
            t1 = time.perf_counter()
            each(close_one)
            self.hbm_close_s = time.perf_counter() - t1
            self.release_hbm_claim()  # nothing of the predecessor is mapped any more

        def open_all() -> None:
            # Bounded: an import that never returns (hipIpcOpenMemHandle on an allocation of
            # 2 GiB or more spins forever, profiles/round5/ipc_cause.md) must not strand this
            # successor holding the claim while its predecessor waits on it -- past
            # TPI_IPC_OPEN_TIMEOUT the HBM route is given up (the caller restores from the
            # host copy).  The openers are daemon threads: one stuck in the driver cannot hold
            # up this process's exit.  IPC handles and dma-bufs are opened side by side.
            todo = sorted(ipc)
            lock = threading.Lock()
            errors: List[BaseException] = []

            def worker() -> None:
                while True:
                    with lock:
                        if not todo or errors:
                            return
                        i = todo.pop()
                    try:
                        open_ipc(i)
                    except BaseException as error:  # re-raised by the caller
                        with lock:
                            errors.append(error)
                        return

            def receiver() -> None:
                try:
                    open_dmabufs()
                except BaseException as error:
                    with lock:
                        errors.append(error)

            workers = [threading.Thread(target=worker, name="tpi-ipc-open", daemon=True)
                       for _ in range(min(8, len(todo)))]
            if doc.get("socket"):
                workers.append(threading.Thread(target=receiver, name="tpi-dmabuf-open",
                                                daemon=True))
            for w in workers:
                w.start()
            deadline = time.monotonic() + limit
            for w in workers:
                w.join(max(0.0, deadline - time.monotonic()))
            if errors:
                raise errors[0]
            if any(w.is_alive() for w in workers):
                with lock:
                    todo.clear()
                    errors.append(CheckpointError("timed out"))
                raise CheckpointError(
                    "HIP IPC import of the predecessor's HBM did not return within %.1f s "
                    "(TPI_IPC_OPEN_TIMEOUT); restoring from the host copy" % limit)
            if any(b is None for b in bases):
                raise CheckpointError("the HBM hand-off left allocations unmapped")

        try:
            open_all()
            self.hbm_open_s = time.perf_counter() - t0
            src = np.frombuffer(bytes.fromhex(doc["segs"]), dtype=self.plan.segs.dtype).copy()
            if len(src) != len(self.plan.segs):
                raise CheckpointError("HBM hand-off describes a different tensor set")
            owner = np.full(len(src), -1, dtype=np.int64)  # mapped allocation of each segment
            for i, w in enumerate(doc["where"]):
                src[i]["ptr"] = 0 if w is None else bases[w[0]] + w[1]
                owner[i] = -1 if w is None else w[0]
            dst = self.plan.segs
            if doc.get("pieces"):
                src, dst, owner = _split_relocated(src, self.plan.segs, doc["pieces"], bases,
                                                   owner)
            # never launch a copy that could touch memory outside what is mapped: every source
            # segment inside its mapped allocation, every destination inside its own
            _check_copy_ranges(src, owner, bases, sizes, dst, lib)
            try:  # diagnostic for the journal
                self.hbm_free_before_copy = torch.cuda.mem_get_info(self.device_index)[0]
            except Exception:
                self.hbm_free_before_copy = 0
            sig = torch.cuda.current_stream(self.device_index).cuda_stream
            res = self.engine.copy_segments(src, self.plan, sig, dst)  # synchronous: copy done
        except BaseException:
            close_all()
            raise
        # Unmapping the predecessor's allocations (~0.03 s per 100 GB) is not on the restore's
        # critical path: the copy has completed, so it runs behind the caller ("restored" goes
        # out at once); close() / the next hand-off wait for it.
        self.hbm_close_s = 0.0
        self._hbm_closer = threading.Thread(target=close_all, name="tpi-ipc-close", daemon=True)
        self._hbm_closer.start()
        self.last_restore = res
        if strict and res.bad_tiles:
            raise CheckpointError("%d tile(s) differ after the HBM hand-off" % res.bad_tiles)
        try:
            os.remove(self._hbm_manifest_path())
        except OSError:
            pass
        return res

    def _check_compatible(self, header: Dict) -> None:
        if (header["total"] != self.plan.total or header["tile_bytes"] != self.plan.tile_bytes
                or header.get("stream_offset") != self.stream_offset
                or header.get("crc_offset") != self.crc_offset
                or header.get("entries_sha256") != self._entries_digest):
            raise CheckpointError("checkpoint layout does not match the bound tensors")

    def persist(self, path: str) -> str:
        """Write the current checkpoint (header, CRCs, stream: one slot) to ``path``
        atomically.  ``path`` may name a file on another node (``ssh://host/dir/file``,
        ``host:/dir/file``: an off-node ``storage.container``, :mod:`..storage.remote`); the
        file is written locally first, then moved there."""
        from ..storage import remote

        if remote.is_remote(path):
            tmp = _local_scratch(path)
            try:
                self.persist(tmp)
                remote.store(tmp, path)
            finally:
                if os.path.exists(tmp):
                    os.remove(tmp)
            return path
        self.wait_pending()
        active = self._active()
        if active is None:
            raise CheckpointError("nothing saved yet")
        slot, header = active
        tmp = path + ".tpi-partial"
        # parallel pwrite of the slot (native, GIL released) + fsync, then an atomic rename
        native().write_file_ptr(tmp, self.region.addr + slot.base,
                                self.stream_offset + int(header["stream_bytes"]),
                                FILE_THREADS, True)
        os.replace(tmp, path)
        return path

    def load(self, path: str) -> TransferResult:
        """Read a persisted checkpoint file into the region (the slot a save would write, so
        a bad file leaves the current checkpoint intact with ``slots=2``) and restore it.

        The stream section is read by parallel native readers in chunks that are published
        like a streamed save's (progress block), so the device restore runs behind the file
        read instead of after it.  ``path`` may name a file on another node (see
        :meth:`persist`): it is fetched first."""
        from ..storage import remote

        if remote.is_remote(path):
            tmp = remote.fetch(path, os.path.dirname(_local_scratch(path)))
            try:
                return self.load(tmp)
            finally:
                os.remove(tmp)
        self.wait_pending()
        self._wait_writers()
        slot, generation = self._target()
        with open(path, "rb") as f:
            head = np.frombuffer(f.read(PREAMBLE + self.header_cap), np.uint8)
            header = self.read_header(head)
            self._check_compatible(header)
            if not header.get("complete"):
                raise CheckpointError("%s holds an incomplete checkpoint" % path)
            size = os.fstat(f.fileno()).st_size
        stream_bytes = int(header["stream_bytes"])
        end = self.stream_offset + stream_bytes
        if size < end:
            raise CheckpointError("%s is truncated (%d of %d bytes)" % (path, size, end))
        self._invalidate(slot)
        # entries + CRCs + blob sizes first (small), then the stream, streamed
        native().read_stream_ptr(path, self.region.addr + slot.base + self.entries_offset,
                                 self.entries_offset, self.stream_offset - self.entries_offset,
                                 FILE_THREADS, 64 << 20, 0, 0, 0)
        if header.get("codec", "none") == "tpz1":
            tile_ends = np.cumsum(slot.csizes.astype(np.uint64), dtype=np.uint64)
            if len(tile_ends) and int(tile_ends[-1]) != stream_bytes:
                raise CheckpointError("%s: blob sizes do not add up to the stream" % path)
        else:
            tile_ends = np.minimum(np.arange(1, self.plan.ntiles + 1, dtype=np.uint64)
                                   * np.uint64(self.plan.tile_bytes), np.uint64(self.plan.total))
        header["generation"] = generation  # newest once complete; written last, like a save
        prog = slot.progress
        prog[1], prog[2], prog[3], prog[5] = generation, 0, 0, os.getpid()
        prog[4] = STREAM_RUNNING
        prog[0] = PROGRESS_MAGIC
        self._write_header(slot, dict(header, complete=False, streaming=True))
        failure: list = []

        def read():
            try:
                native().read_stream_ptr(path, self.region.addr + slot.base + self.stream_offset,
                                         self.stream_offset, stream_bytes, FILE_THREADS,
                                         LOAD_CHUNK, prog.ctypes.data + 16,
                                         tile_ends.ctypes.data, len(tile_ends))
                self._write_header(slot, header)
                prog[4] = STREAM_COMPLETE
            except BaseException as error:  # the restore sees FAILED and raises
                failure.append(error)
                prog[4] = STREAM_FAILED

        reader = threading.Thread(target=read, name="tpi-load", daemon=True)
        reader.start()
        try:
            res = self.restore()
        finally:
            reader.join()
        if failure:
            raise CheckpointError("loading %s failed: %s" % (path, failure[0]))
        return res

    def release_device(self) -> int:
        """A preempted rank after its save: free the HBM this checkpointer and its bound
        tensors hold -- engine staging chunks, the async snapshot, and the storages of every
        bound tensor (which the model shares: they are unusable afterwards) -- keeping the
        host region (and its pinning) for the successor.  Returns the bytes released."""
        freed = 0
        self._snap = self._snap_crcs = None
        for slot in self.slots:
            slot.digests = None
        if self.engine is not None:
            self.engine.close()
            self.engine = None
        for t in getattr(self.plan, "_bound", []):
            if getattr(t, "is_cuda", False):
                storage = t.untyped_storage()
                freed += storage.nbytes()
                storage.resize_(0)
        freed += self._free_relocated()
        return freed

    def _free_relocated(self) -> int:
        """Free the blocks an HBM export relocated tensors into (:meth:`_relocate`); only once
        no successor maps them any more (the hand-off protocol has ended)."""
        blocks = getattr(self, "_relocated", None)
        if not blocks:
            return 0
        self._relocated = []
        lib = hip()
        freed = 0
        for b in blocks:
            lib.tpi_dev_free(ctypes.c_void_p(b))
            freed += self._relocated_size.pop(b, 0)
        return freed

    def wait_hbm_close(self) -> None:
        closer = getattr(self, "_hbm_closer", None)
        if closer is not None:
            closer.join()
            self._hbm_closer = None

    def watch(self, fn, name: str) -> threading.Thread:
        """Run ``fn`` on a daemon thread that :meth:`close` joins before unmapping the
        region (``fn`` may poll the region through :meth:`wait_stream`)."""
        thread = threading.Thread(target=fn, name=name, daemon=True)
        self._watchers.append(thread)
        thread.start()
        return thread

    @property
    def closing(self) -> bool:
        return self._closing.is_set()

    def close(self) -> None:
        self._closing.set()
        for thread in self._watchers:
            if thread is not threading.current_thread():
                thread.join()
        self._watchers = []
        self.wait_hbm_close()
        try:
            self.wait_pending()
        except CheckpointError:
            pass
        self._snap = self._snap_crcs = None
        for slot in getattr(self, "slots", []):
            slot.digests = None
        if self.engine is not None:
            self.engine.close()
            self.engine = None
        if self.region is not None:
            self.slots = []
            self.region.close()
            self.region = None
        self._close_dmabuf_server()
        self._free_relocated()
        if self.plan is not None and hasattr(self.plan, "unbind"):
            self.plan.unbind()  # the tensors' HBM can go with the caller's references

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def _seg_extent(seg) -> Tuple[int, int]:
    """``[lo, hi)`` of the memory a segment descriptor touches (strided views: from their
    lowest to their highest element)."""
    ptr, nbytes = int(seg["ptr"]), int(seg["nbytes"])
    if int(seg["kind"]) == SEG_CONTIG or nbytes == 0:
        return ptr, ptr + nbytes
    elem = int(seg["elem"])
    neg = pos = 0
    for d in range(int(seg["ndim"])):
        span = (int(seg["sizes"][d]) - 1) * int(seg["strides"][d]) * elem
        if span < 0:
            neg += span
        else:
            pos += span
    return ptr + neg, ptr + pos + elem


def _check_copy_ranges(src: np.ndarray, owner: np.ndarray, bases: List[Optional[int]],
                       sizes: List[int], dst: np.ndarray, lib) -> None:
    """Host-side bounds check before the hand-off's copy kernel: each source segment must lie
    inside the predecessor allocation it was mapped from (``owner``), each destination segment
    inside the device allocation holding it in this process.  A descriptor that fails raises
    CheckpointError (the caller restores from the host copy) instead of faulting the GPU."""
    base, size = ctypes.c_uint64(0), ctypes.c_uint64(0)
    for i in range(len(src)):
        if int(src[i]["nbytes"]) == 0:
            continue
        a = int(owner[i])
        lo, hi = _seg_extent(src[i])
        if a < 0 or bases[a] is None or lo < bases[a] or hi > bases[a] + sizes[a]:
            raise CheckpointError(
                "HBM hand-off: source segment %d [%#x, %#x) lies outside its mapped allocation "
                "%d [%s, +%d)" % (i, lo, hi, a, None if a < 0 else bases[a],
                                  -1 if a < 0 else sizes[a]))
        lo, hi = _seg_extent(dst[i])
        if lib.tpi_mem_range(ctypes.c_void_p(int(dst[i]["ptr"])), ctypes.byref(base),
                             ctypes.byref(size)) != 0:
            raise CheckpointError("HBM hand-off: destination segment %d is not device memory"
                                  % i)
        if lo < int(base.value) or hi > int(base.value) + int(size.value):
            raise CheckpointError(
                "HBM hand-off: destination segment %d [%#x, %#x) lies outside its allocation "
                "[%#x, +%d)" % (i, lo, hi, int(base.value), int(size.value)))


def _split_relocated(src: np.ndarray, dst: np.ndarray, pieces: Dict[str, List[List[int]]],
                     bases: List[Optional[int]], owner: np.ndarray
                     ) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Source and destination descriptors for an HBM hand-off whose exporter relocated some
    tensors into blocks (:meth:`Checkpointer._relocate`): each such segment becomes one
    contiguous segment per block, the destination split at the same stream offsets.  Both
    stay sorted by stream offset, so the copy and its verification see the same stream.
    ``owner`` (mapped allocation per segment) is expanded alongside."""
    out_src, out_dst, out_owner = [], [], []
    for i in range(len(src)):
        parts = pieces.get(str(i))
        if not parts:
            out_src.append(src[i:i + 1])
            out_dst.append(dst[i:i + 1])
            out_owner.append(int(owner[i]))
            continue
        if int(dst[i]["kind"]) != SEG_CONTIG:
            raise CheckpointError("HBM hand-off: a relocated tensor is not contiguous here")
        if sum(int(p[2]) for p in parts) != int(src[i]["nbytes"]):
            raise CheckpointError("HBM hand-off: relocated pieces do not cover tensor %d" % i)
        done = 0
        for alloc, off, n in parts:
            s_part = src[i:i + 1].copy()
            d_part = dst[i:i + 1].copy()
            for part, ptr in ((s_part, bases[alloc] + off), (d_part, int(dst[i]["ptr"]) + done)):
                part["ptr"] = ptr
                part["off"] = int(src[i]["off"]) + done
                part["nbytes"] = n
                part["kind"], part["ndim"] = SEG_CONTIG, 0
            out_src.append(s_part)
            out_dst.append(d_part)
            out_owner.append(int(alloc))
            done += n
    return np.concatenate(out_src), np.concatenate(out_dst), np.array(out_owner, np.int64)


def _region_layout(path: str) -> Dict[str, Any]:
    """What :meth:`Checkpointer.materialize` needs from a region file without its tensors:
    the entries (and their blob's digest), total, tile size, codec, slot count and size.
    Reads the first slot's preamble, or the second slot's (at half the file) when a save in
    progress has cleared the first."""
    size = os.path.getsize(path)
    with open(path, "rb") as f:
        for base in (0, size // 2):
            f.seek(base)
            pre = f.read(PREAMBLE)
            if pre[:8] != MAGIC:
                continue
            n, entries_offset, entries_len = struct.unpack("<QQQ", pre[8:32])
            header = json.loads(f.read(n))
            f.seek(base + entries_offset)
            blob = f.read(entries_len)
            slot_end = _layout(Checkpointer.HEADER_RESERVE, entries_len, header["ntiles"],
                               header["total"], header["tile_bytes"])[4]
            slot_bytes = align_up(slot_end, 4096)
            slots = 2 if size >= 2 * slot_bytes else 1
            if base and slots != 2:
                continue
            if size < slot_end:  # a persisted file holds one slot, cut after its stream
                raise CheckpointError("%s is a persisted checkpoint, not a spill region: "
                                      "restore it with Checkpointer.load()" % path)
            return {"entries": json.loads(blob),
                    "entries_sha256": hashlib.sha256(blob).hexdigest(),
                    "total": header["total"], "tile_bytes": header["tile_bytes"],
                    "codec": header.get("codec", "none"), "slots": slots,
                    "size": slot_bytes * slots if slots > 1 else slot_end}
    raise CheckpointError("%s holds no checkpoint header" % path)


def describe_checkpoint(path: str, entries: bool = True) -> Dict:
    """Header of a persisted checkpoint file (no tensors needed), with its tensor entries
    unless ``entries=False``."""
    with open(path, "rb") as f:
        pre = f.read(PREAMBLE)
        if pre[:8] != MAGIC:
            raise CheckpointError("%s is not a checkpoint" % path)
        n, entries_offset, entries_len = struct.unpack("<QQQ", pre[8:32])
        header = json.loads(f.read(n))
        if entries:
            f.seek(entries_offset)
            header["entries"] = json.loads(f.read(entries_len))
        return header


def verify_checkpoint(path: str) -> Dict:
    """Integrity check of a persisted checkpoint without its tensors: decode the stream (if
    encoded) and compare every tile's CRC32C with the recorded one (host, native code)."""
    header = describe_checkpoint(path, entries=False)
    if not header.get("complete"):
        return {"complete": False, "bad_tiles": None, "first_bad": None}
    ntiles, tile, total = header["ntiles"], header["tile_bytes"], header["total"]
    data = np.memmap(path, dtype=np.uint8, mode="r")
    crcs = np.array(data[header["crc_offset"]:header["crc_offset"] + 4 * ntiles].view(np.uint32))
    start = header["stream_offset"]
    stream = data[start:start + int(header["stream_bytes"])]
    first_malformed = -1
    if header.get("codec", "none") == "tpz1":
        sizes = np.array(data[header["csize_offset"]:header["csize_offset"] + 4 * ntiles]
                         .view(np.uint32))
        stream, first_malformed = tpz.decode(np.ascontiguousarray(stream), sizes, total, tile)
    from ..ops.hashing import crc32c_tiles

    actual = crc32c_tiles(np.ascontiguousarray(stream), tile_bytes=tile)
    bad = np.nonzero(actual != crcs)[0]
    return {"complete": True, "codec": header.get("codec", "none"), "tiles": ntiles,
            "bad_tiles": int(len(bad)), "first_bad": int(bad[0]) if len(bad) else -1,
            "first_malformed_blob": int(first_malformed),
            "crc32c": native().crc32c_combine_tiles_ptr(crcs.ctypes.data, ntiles, tile, total)
            == header.get("crc32c")}
