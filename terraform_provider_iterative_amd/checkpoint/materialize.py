"""Progressive materialisation of a checkpoint region: the state is allocated group by group
while it streams in (the :class:`~.checkpointer.Checkpointer` mixin behind
``Checkpointer.materialize``).

For a successor whose state does not fit next to its predecessor's on one GPU (a 170 GB rank
on 288 GB of HBM), allocation, the driver's clearing of the freed HBM, the predecessor's spill
and the restore overlap instead of running one after the other
(``profiles/round4/materialize_170g.md``).  Reference: the replacement machine restores the
bucket's ``data/`` before the task runs again (``task/common/machine/machine-script.sh.tpl:89``).
"""
from __future__ import annotations

import os
import queue
import threading
import time
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

from ..ops import codec as tpz
from ..ops import native
from ..ops.packing import PackPlan, TensorEntry
from ..ops.packing import unpack as host_unpack
from .base import STREAM_COMPLETE, STREAM_FAILED, CheckpointError, TransferResult

ALLOC_HEADROOM = 512 << 20  # materialize(): free HBM beyond a tensor's size before allocating it
ALLOC_LOOKAHEAD = 3  # materialize(): groups allocated ahead of the restore once HBM runs short


class Materializer:
    """The materialisation half of :class:`~.checkpointer.Checkpointer` (a mixin: it uses the
    checkpointer's plan, engine, slots and streaming restore)."""

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
        from .checkpointer import _region_layout

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

