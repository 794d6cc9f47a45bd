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
import struct
import threading
import time
from typing import Any, Dict, List, Mapping, Optional, Sequence, Tuple, Union

import numpy as np

from ..ops import codec as tpz
from ..ops import hip, native
from ..ops.packing import PackPlan, align_up
from ..ops.packing import pack as host_pack, unpack as host_unpack
from . import host
from .base import (MAGIC, PREAMBLE, PROGRESS_MAGIC, STREAM_COMPLETE,  # noqa: F401
                   STREAM_FAILED, STREAM_RUNNING, CheckpointError, TransferResult,
                   _writer_alive)
from .handoff import (FDS_PER_MESSAGE, HBM_ROUTES, IPC_MAX_ALLOC, RELOCATE_CHUNK,  # noqa: F401
                      HbmHandoff)  # (the constants: re-exported, tests read them here)
from .engine import (MODES, DeviceEngine, _engine_pool, _take_engine,  # noqa: F401
                     prewarm_engine)
from .host import HostRegion
from .materialize import ALLOC_HEADROOM, ALLOC_LOOKAHEAD, Materializer  # noqa: F401
from .persist import FILE_THREADS, LOAD_CHUNK, Persistence, _local_scratch  # noqa: F401

CODECS = ("none", "tpz1")


def _layout(header_cap: int, entries_len: int, ntiles: int, total: int, tile_bytes: int):
    entries_offset = align_up(PREAMBLE + header_cap, 4096)
    crc_offset = align_up(entries_offset + entries_len, 4096)
    csize_offset = crc_offset + 4 * ntiles
    stream_offset = align_up(csize_offset + 4 * ntiles, 4096)
    capacity = max(total, tpz.bound(total, tile_bytes))
    return entries_offset, crc_offset, csize_offset, stream_offset, stream_offset + capacity


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


def region_total(path: str) -> Optional[int]:
    """Bytes of device state the checkpoint region file ``path`` describes (its header's
    ``total``), None when there is no readable header.  Reads the file only (no mapping)."""
    try:
        with open(path, "rb") as f:
            head = f.read(PREAMBLE + Checkpointer.HEADER_RESERVE)
        return int(Checkpointer.read_header(np.frombuffer(head, np.uint8))["total"])
    except (OSError, ValueError, KeyError, CheckpointError):
        return None


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


class Checkpointer(HbmHandoff, Materializer, Persistence):
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

    def _check_compatible(self, header: Dict) -> None:
        if (header["total"] != self.plan.total or header["tile_bytes"] != self.plan.tile_bytes
                or header.get("stream_offset") != self.stream_offset
                or header.get("crc_offset") != self.crc_offset
                or header.get("entries_sha256") != self._entries_digest):
            raise CheckpointError("checkpoint layout does not match the bound tensors")

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
