"""HBM-resident workdir for rank processes.

``stage_workdir`` turns the task's working directory into one device buffer:

1. the root rank walks the tree with the rclone-compatible filters (native walker),
2. optionally (``TPI_STAGE_ZERO_COPY=1``) DMAs large page-cache resident files (>= 64 MiB,
   not on tmpfs) straight from their pages: 1 GiB windows are
   mapped read-only with MAP_POPULATE and registered for DMA (~13 ms per GiB, measured on
   MI355X: 57 GB/s H2D from such a mapping, ``scripts/exp/zerocopy_stage.py``), copies and
   the next registration overlap; everything else goes through the native loader
   (``runtime/stage.py`` ``Loader``: pread workers into a NUMA-local pinned ring, H2D of
   chunk k overlapping the reads of chunk k+1; 51 GB/s for 10 GB on MI355X),
3. fans the buffer out to every rank over xGMI with the RCCL task communicator
   (:class:`..parallel.comm.TaskComm`, the runtime stager's own data plane),
4. optionally verifies the copy with the device shard-hash kernel on every rank.

Each file is then a zero-copy ``uint8`` view (``StagedWorkdir.tensor(path)``); the digests
give the change detection that replaces the reference's 10-second ``find -printf %T@`` poll
(``machine-script.sh.tpl:118-124``): re-hash on device, spill only dirty shards.
"""
from __future__ import annotations

import ctypes
import logging
import os
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

from ..ops import native, shard_hash
from ..storage.transfer import make_filter, transfer_rules

log = logging.getLogger("tpi.workdir")

ALIGN = 4096
FANOUT_METHODS = ("sharded", "broadcast", "independent")
ZERO_COPY_MIN = 64 << 20  # files at least this large are DMA'd from their page-cache pages


@dataclass
class FileEntry:
    path: str
    offset: int
    size: int
    mtime_ns: int = 0


@dataclass
class StagedWorkdir:
    root: str
    files: List[FileEntry]
    buffer: object  # 1-D uint8 tensor
    stats: Dict[str, float] = field(default_factory=dict)

    def tensor(self, path: str):
        for f in self.files:
            if f.path == path:
                return self.buffer[f.offset:f.offset + f.size]
        raise KeyError(path)

    def digest(self, shard_bytes: int = 1 << 20):
        """Per-shard digests as an int64 tensor on the buffer's device."""
        import torch

        out = shard_hash(self.buffer, shard_bytes=shard_bytes)
        if isinstance(out, torch.Tensor):
            return out
        return torch.from_numpy(out.view("int64").copy())

    def write_back(self, directory: str, paths: Optional[List[str]] = None,
                   ranges: Optional[List[Tuple[int, int]]] = None, threads: int = 16) -> int:
        """Write files (all, ``paths``, or only the image ``ranges`` they overlap) from the
        buffer back to ``directory``: only those bytes leave the device (native loader,
        pinned ring), not the whole buffer.  Returns the bytes written."""
        from .stage import Loader

        wanted = [f for f in self.files if paths is None or f.path in paths]
        for f in wanted:
            dst = os.path.join(directory, f.path)
            if not os.path.exists(dst) or os.path.getsize(dst) != f.size:
                os.makedirs(os.path.dirname(dst), exist_ok=True)
                with open(dst, "ab") as handle:
                    handle.truncate(f.size)
        if ranges is None:
            ranges = [(f.offset, f.offset + f.size) for f in wanted if f.size]
        entries = [(f.path, f.offset, f.size) for f in wanted]
        if not ranges or not entries:
            return 0
        device = self.buffer.device.index if self.buffer.device.type == "cuda" else -1
        with Loader(device, chunk_bytes=64 << 20, threads=threads) as loader:
            return loader.store(directory, entries, sorted(ranges),
                                self.buffer.data_ptr())["bytes"]

    def sync(self, directory: str, shard_bytes: int = 1 << 20) -> Dict[str, float]:
        """Write back only the shards whose digest changed since the last sync (or since
        staging) -- the device-side replacement of the reference's 10-second newest-mtime
        poll + ``rclone sync`` (machine-script.sh.tpl:118-124)."""
        import numpy as np

        t0 = time.perf_counter()
        digests = self.digest(shard_bytes)
        cur = digests.cpu().numpy() if hasattr(digests, "cpu") else np.asarray(digests)
        base = self.stats.get("_digests")
        if base is None or len(base) != len(cur):
            dirty = np.arange(len(cur))
        else:
            dirty = np.nonzero(cur != base)[0]
        ranges: List[Tuple[int, int]] = []
        total = int(self.buffer.numel())
        for i in dirty.tolist():
            lo, hi = i * shard_bytes, min(total, (i + 1) * shard_bytes)
            if ranges and ranges[-1][1] == lo:
                ranges[-1] = (ranges[-1][0], hi)
            else:
                ranges.append((lo, hi))
        written = self.write_back(directory, ranges=ranges) if ranges else 0
        self.stats["_digests"] = cur
        return {"dirty_shards": int(len(dirty)), "bytes": written,
                "seconds": time.perf_counter() - t0}


def manifest(root: str, exclude: Optional[List[str]] = None) -> Tuple[List[FileEntry], int]:
    entries = native().walk(root, make_filter(transfer_rules(exclude)))
    files, off = [], 0
    for rel, size, mtime, _mode, is_dir in entries:
        if is_dir:
            continue
        files.append(FileEntry(rel, off, size, mtime))
        off += (size + ALIGN - 1) // ALIGN * ALIGN
    return files, off


def _pieces_for(root: str, files: List[FileEntry], lo: int, hi: int):
    """(path, file_off, len, dst_off-relative-to-lo) pieces covering [lo, hi)."""
    pieces = []
    for f in files:
        a, b = max(lo, f.offset), min(hi, f.offset + f.size)
        if a < b:
            pieces.append((os.path.join(root, f.path), a - f.offset, b - a, a - lo))
    return pieces


def _runs(files: List[FileEntry], small: List[bool], total: int) -> List[Tuple[int, int]]:
    """Buffer ranges [lo, hi) covering maximal sequences of consecutive small files (with
    their alignment padding), so the bounce path never writes over a zero-copy file."""
    runs: List[Tuple[int, int]] = []
    start = None
    for i, f in enumerate(files):
        end = files[i + 1].offset if i + 1 < len(files) else total
        if small[i]:
            if start is None:
                start = f.offset
            if i + 1 == len(files) or not small[i + 1]:
                runs.append((start, end))
                start = None
    return runs


def _zero_copy(root: str, files: List[FileEntry], buffer, stream, window: int,
               inflight: int = 3) -> float:
    """H2D straight from the page cache: each window of a large file is mapped read-only
    (MAP_POPULATE), registered for DMA and copied on ``stream``; windows are unregistered
    once their copy completed, ``inflight`` of them overlap.  Returns the host-side seconds."""
    import mmap

    import torch

    from ..ops import hip

    lib = hip()
    page = mmap.ALLOCATIONGRANULARITY
    pending: List[tuple] = []
    host_s = 0.0

    def retire(entry):
        ev, m, addr = entry
        ev.synchronize()
        lib.tpi_host_unregister(ctypes.c_void_p(addr))
        m.close()

    for f in files:
        fd = os.open(os.path.join(root, f.path), os.O_RDONLY)
        try:
            for pos in range(0, f.size, window):
                n = min(window, f.size - pos)
                t = time.perf_counter()
                base = pos // page * page
                span = pos - base + n
                m = mmap.mmap(fd, span, mmap.MAP_SHARED | getattr(mmap, "MAP_POPULATE", 0),
                              mmap.PROT_READ, offset=base)
                addr = _address(m)
                lib.check(lib.tpi_host_register_ro(ctypes.c_void_p(addr), span),
                          "hipHostRegister(read-only)")
                lib.check(lib.tpi_h2d_async(ctypes.c_void_p(buffer.data_ptr() + f.offset + pos),
                                            ctypes.c_void_p(addr + pos - base), n,
                                            stream.cuda_stream), "hipMemcpyAsync")
                ev = torch.cuda.Event()
                ev.record(stream)
                pending.append((ev, m, addr))
                host_s += time.perf_counter() - t
                if len(pending) >= inflight:
                    retire(pending.pop(0))
        finally:
            os.close(fd)
    for entry in pending:
        retire(entry)
    return host_s


def _zero_copy_ok(root: str, f: FileEntry, zero_copy_min: int) -> bool:
    """Opt-in (``TPI_STAGE_ZERO_COPY=1``); large, page-cache resident and not on tmpfs.

    Measured on MI355X: freshly written 1 GB files stage at 39-50 GB/s this way against 23-37
    through the bounce buffers (``scripts/exp/stage_modes.py``), but the task's data files
    written by the push (``copy_file_range``) stage at 12 GB/s against 27-28 -- so the bounce
    path stays the default.  A file read from disk would fault in single-threaded under
    MAP_POPULATE, and shmem pages pin for DMA several times slower than the bounce copy."""
    if f.size < zero_copy_min or os.environ.get("TPI_STAGE_ZERO_COPY", "0") != "1":
        return False
    resident, size, tmpfs = native().resident_bytes(os.path.join(root, f.path))
    return not tmpfs and resident >= 0 and resident >= 0.9 * size


def _address(m) -> int:
    """Address of a (read-only) mmap's first byte."""
    import numpy as np

    return int(np.frombuffer(m, dtype=np.uint8).ctypes.data)


def _numa(device_index: int) -> int:
    from ..ops import hip

    node = ctypes.c_int(-1)
    hip().tpi_device_numa_node(device_index, ctypes.byref(node))
    return node.value


def load_into(root: str, files: List[FileEntry], total: int, buffer,
              chunk_bytes: int = 256 << 20, threads: int = 16,
              zero_copy_min: int = ZERO_COPY_MIN) -> Dict[str, float]:
    """Fill ``buffer`` (device or host uint8 tensor of ``total`` bytes) from the files.

    On the device, files of at least ``zero_copy_min`` bytes are DMA'd straight from their
    page-cache pages (:func:`_zero_copy`, opt-in); the rest go through the native loader's
    pinned ring (:class:`.stage.Loader`), the reads of chunk k+1 overlapping the DMA of k.
    """
    import torch

    t0 = time.perf_counter()
    read_s = 0.0
    if buffer.device.type != "cuda":
        for lo in range(0, total, chunk_bytes):
            hi = min(total, lo + chunk_bytes)
            t = time.perf_counter()
            native().read_pieces(_pieces_for(root, files, lo, hi), buffer.data_ptr() + lo, threads)
            read_s += time.perf_counter() - t
        return {"seconds": time.perf_counter() - t0, "read_s": read_s, "bytes": total}
    stream = torch.cuda.Stream(buffer.device)
    # the copies must land after whatever the caller queued on ``buffer`` (its allocation /
    # fill on the current stream)
    stream.wait_stream(torch.cuda.current_stream(buffer.device))
    small = [not _zero_copy_ok(root, f, zero_copy_min) for f in files]
    big = [f for f, s in zip(files, small) if not s]
    zc_s = 0.0
    if big:
        with torch.cuda.stream(stream):
            buffer.zero_()  # alignment padding between zero-copied files (digests need zeros)
        try:
            zc_s = _zero_copy(root, big, buffer, stream, window=max(chunk_bytes, 1 << 30))
        except Exception as error:  # e.g. a file system without mmap: bounce everything
            log.warning("zero-copy staging unavailable (%s); using bounce buffers", error)
            small = [True] * len(files)
    runs = _runs(files, small, total)
    if runs:
        # everything else through the native loader (csrc/hip/stage.hip): NUMA-local pinned
        # ring, pread workers filling chunk k+1 while chunk k is in flight H2D
        from .stage import Loader

        stream.synchronize()  # the loader's copy stream is not ordered after torch's streams
        entries = [(f.path, f.offset, f.size) for f in files]
        with Loader(buffer.device.index, chunk_bytes=min(chunk_bytes, 64 << 20), nbuf=4,
                    threads=threads, numa_node=_numa(buffer.device.index)) as loader:
            for run_lo, run_hi in runs:
                read_s += loader.load(root, entries, run_lo, run_hi,
                                      buffer.data_ptr())["read_ms"] / 1e3
    stream.synchronize()
    return {"seconds": time.perf_counter() - t0, "read_s": read_s, "zero_copy_host_s": zc_s,
            "zero_copy_files": len(big), "bytes": total}


def stage_workdir(root: Optional[str] = None, device=None, exclude: Optional[List[str]] = None,
                  group=None, src: int = 0, method: str = "auto", verify: bool = True,
                  chunk_bytes: int = 256 << 20, threads: int = 16,
                  zero_copy_min: int = ZERO_COPY_MIN) -> StagedWorkdir:
    """Stage ``root`` (default ``$TPI_DATA_DIRECTORY`` or cwd) into HBM on every rank.

    The library path for scripts that stage themselves (``TPI_STAGE=off`` tasks, or no
    runtime stager); it uses the stager's own data plane -- the native loader and the RCCL
    task communicator (:class:`..parallel.comm.TaskComm`) -- with ``torch.distributed`` only
    carrying the file list and the digests:

    * ``sharded`` (``auto`` on GPUs): rank i loads the i-th 1/N of the image over its own
      PCIe link, then one in-place all-gather over xGMI;
    * ``broadcast``: rank ``src`` loads everything, then an RCCL broadcast;
    * ``independent`` (``auto`` on CPUs): every rank loads its own copy -- the reference's
      pattern, each machine running its own ``rclone copy`` (``machine-script.sh.tpl:89``).
    """
    import torch

    root = root or os.environ.get("TPI_DATA_DIRECTORY") or os.getcwd()
    distributed = False
    try:
        import torch.distributed as dist

        distributed = dist.is_available() and dist.is_initialized()
    except ImportError:  # pragma: no cover
        dist = None
    rank = dist.get_rank(group) if distributed else 0
    world = dist.get_world_size(group) if distributed else 1
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
            else torch.device("cpu")
    device = torch.device(device)
    on_gpu = device.type == "cuda"
    if method == "auto":
        method = "sharded" if on_gpu else "independent"
    if method not in FANOUT_METHODS:
        raise ValueError("method must be one of %s" % (FANOUT_METHODS,))
    if not on_gpu:
        method = "independent"  # host images: every rank reads the node's files itself
    if rank == src:
        files, size = manifest(root, exclude)
        meta = [[(f.path, f.offset, f.size, f.mtime_ns) for f in files], size]
    else:
        meta = [None, None]
    if world > 1:
        dist.broadcast_object_list(meta, src=src, group=group)
    files = [FileEntry(*m) for m in meta[0]]
    size = int(meta[1])
    # the sharded all-gather needs equal shards: pad the image to a multiple of world pages
    quantum = ALIGN * max(1, world)
    total = (size + quantum - 1) // quantum * quantum if world > 1 and on_gpu else size
    alloc = torch.zeros if not on_gpu or method == "sharded" else torch.empty
    buffer = alloc(total, dtype=torch.uint8, device=device)
    stats: Dict[str, float] = {"bytes": total, "files": len(files), "method": method}  # type: ignore
    t0 = time.perf_counter()
    if world == 1 or method == "independent":
        load = load_into(root, files, total, buffer, chunk_bytes, threads, zero_copy_min)
        stats["read_s"] = load["read_s"]
        stats["zero_copy_files"] = load.get("zero_copy_files", 0)
    else:
        from ..parallel.comm import TaskComm
        from .stage import Loader

        entries = [(f.path, f.offset, f.size) for f in files]
        torch.cuda.current_stream(device).synchronize()  # the zeroed buffer, before the DMA
        comm = TaskComm.from_group(group, device=device.index)
        try:
            with Loader(device.index, chunk_bytes=min(chunk_bytes, 64 << 20), nbuf=4,
                        threads=threads, numa_node=_numa(device.index)) as loader:
                if method == "sharded":
                    shard = total // world
                    lo, hi = rank * shard, min(size, (rank + 1) * shard)
                    if lo < hi:
                        stats["read_s"] = loader.load(root, entries, lo, hi,
                                                      buffer.data_ptr())["read_ms"] / 1e3
                    stats["load_s"] = time.perf_counter() - t0
                    comm.allgather_inplace(buffer, shard)
                else:
                    if rank == src:
                        stats["read_s"] = loader.load(root, entries, 0, size,
                                                      buffer.data_ptr())["read_ms"] / 1e3
                    stats["load_s"] = time.perf_counter() - t0
                    comm.broadcast(buffer, total, root=src)
        finally:
            comm.close()
    stats["stage_s"] = time.perf_counter() - t0
    staged = StagedWorkdir(root, files, buffer, stats)
    if total:  # baseline of sync(): what was staged
        base = staged.digest()
        stats["_digests"] = base.cpu().numpy() if hasattr(base, "cpu") else base
    if verify and world > 1 and total:
        mine = staged.digest()
        ref = mine.clone()
        dist.broadcast(ref, src=src, group=group)
        stats["verified"] = bool(torch.equal(mine, ref))  # type: ignore[assignment]
    return staged
