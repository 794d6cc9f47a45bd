"""Host memory regions for checkpoint spills.

A region is one mapping holding ``[preamble | tile CRCs | packed stream]``.  Anonymous regions
model "host DRAM"; file-backed ones (``/dev/shm/...`` or a file in the task's storage root)
outlive the rank process, which is what lets a preempted rank's successor restore from
host memory.  For device checkpoints the region is NUMA-bound to the GPU's socket, populated
with parallel first touch and registered with HIP once (``hipHostRegister``), so every later
save/restore is a pure DMA pipeline.
"""
from __future__ import annotations

import ctypes
import mmap
import os
import threading
from typing import Dict, Optional, Tuple

import numpy as np

from ..ops import hip


PIN_WINDOW = 1 << 30  # progressive pinning: registration granule


class HostRegion:
    """``progressive=True`` (device regions): map without populating and pin in the
    background, window by window (``tpi_host_pin_start``); the engine's copies wait for their
    window, so a restore streams while the rest of the region is still being pinned."""

    def __init__(self, size: int, path: Optional[str] = None, *, device: bool = False,
                 numa_node: int = -1, populate: bool = True, _mapped=None,
                 progressive: bool = False, window: int = PIN_WINDOW, threads: int = 8):
        self.size = size
        self.path = path
        self.device = device
        self.registered = False
        self._mmap = None
        self.pinner = None
        self.window = 0
        if _mapped is not None:  # adopted from early_prefetch(): python mmap, registered
            self._mmap, self.addr = _mapped
            self.registered = True
        elif device and progressive:
            lib = hip()
            enc = path.encode() if path else None
            ptr = lib.tpi_host_map(enc, size, numa_node, 0)
            if not ptr:
                raise MemoryError("tpi_host_map(%d bytes) failed: %s" % (size, lib.error()))
            self.addr = int(ptr)
            self.pinner = lib.tpi_host_pin_start(ctypes.c_void_p(self.addr), size, window,
                                                 threads)
            self.window = int(lib.tpi_host_pin_window(self.pinner))
            self.registered = True
        elif device:
            lib = hip()
            enc = path.encode() if path else None
            ptr = lib.tpi_host_map(enc, size, numa_node, 1 if populate else 0)
            if not ptr:
                raise MemoryError("tpi_host_map(%d bytes) failed: %s" % (size, lib.error()))
            self.addr = int(ptr)
            lib.check(lib.tpi_host_register(ctypes.c_void_p(self.addr), size), "hipHostRegister")
            self.registered = True
        else:
            if path:
                fd = os.open(path, os.O_RDWR | os.O_CREAT, 0o600)
                try:
                    if os.fstat(fd).st_size < size:
                        os.ftruncate(fd, size)
                    self._mmap = mmap.mmap(fd, size)
                finally:
                    os.close(fd)
            else:
                self._mmap = mmap.mmap(-1, size)
            buf = (ctypes.c_char * size).from_buffer(self._mmap)
            self.addr = ctypes.addressof(buf)
            del buf
        _announce(self.addr, size, path)

    def array(self, offset: int = 0, length: Optional[int] = None, dtype=np.uint8) -> np.ndarray:
        """numpy view of ``[offset, offset + length)``."""
        length = self.size - offset if length is None else length
        itemsize = np.dtype(dtype).itemsize
        buf = (ctypes.c_char * length).from_address(self.addr + offset)
        arr = np.frombuffer(buf, dtype=np.uint8, count=length)
        return arr.view(dtype) if itemsize > 1 else arr

    def close(self, timings: Optional[Dict[str, float]] = None) -> None:
        """Unregister (unpin) and unmap; ``timings`` receives the seconds of each phase
        (``unregister``, ``unmap``)."""
        if self.addr is None:
            return
        import time

        t0 = time.perf_counter()
        if self.device and self._mmap is not None:  # early-prefetched mapping
            if self.registered:
                hip().tpi_host_unregister(ctypes.c_void_p(self.addr))
            t1 = time.perf_counter()
            try:
                self._mmap.close()
            except BufferError:
                pass
        elif self.device:
            lib = hip()
            if self.pinner:  # unregisters every pinned window
                lib.tpi_host_pin_release(self.pinner)
                self.pinner = None
            elif self.registered:
                lib.tpi_host_unregister(ctypes.c_void_p(self.addr))
            t1 = time.perf_counter()
            lib.tpi_host_unmap(ctypes.c_void_p(self.addr), self.size)
        else:
            t1 = t0
            if self._mmap is not None:
                try:
                    self._mmap.close()
                except BufferError:  # outstanding numpy views; the mapping dies with them
                    pass
        if timings is not None:
            timings["unregister"] = t1 - t0
            timings["unmap"] = time.perf_counter() - t1
        self.addr = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass


def _announce(addr: int, size: int, path: Optional[str]) -> None:
    """Record a checkpoint region in the task's region list (``TPI_REGIONS_FILE``, set by
    the supervisor): its memory-limit check leaves these mappings out of a rank's host memory
    -- a spill region mirrors device state, it is not the rank's working set (a legacy alias
    like ``m+t4`` allows 16 GB per rank, less than one GPU's checkpoint).  One ``O_APPEND``
    line ``<pid> <start hex> <end hex> <path or ->``."""
    registry = os.environ.get("TPI_REGIONS_FILE")
    if not registry or not addr:
        return
    line = "%d %x %x %s\n" % (os.getpid(), addr, addr + size, os.path.abspath(path) if path
                              else "-")
    try:
        fd = os.open(registry, os.O_WRONLY | os.O_CREAT | os.O_APPEND, 0o644)
        try:
            os.write(fd, line.encode())
        finally:
            os.close(fd)
    except OSError:
        pass


def numa_placement(addr: int, size: int) -> Optional[Dict[str, object]]:
    """Where the kernel put the pages of the mapping ``[addr, addr + size)``: bytes per NUMA
    node and the page size, from ``/proc/self/numa_maps`` (None when unreadable).  The regions
    are bound MPOL_PREFERRED to the GPU's socket, so a node short of free memory spills the
    rest to the other socket, whose pages then cross the inter-socket link on every copy."""
    try:
        with open("/proc/self/numa_maps") as f:
            lines = f.readlines()
    except OSError:
        return None
    out: Dict[str, object] = {}
    nodes: Dict[str, int] = {}
    page_kb = 4
    for line in lines:
        fields = line.split()
        try:
            start = int(fields[0], 16)
        except (IndexError, ValueError):
            continue
        if not (addr <= start < addr + size) or len(fields) < 2:
            continue
        out.setdefault("policy", fields[1])  # e.g. "prefer:0", "default"
        counts = {}
        for f in fields[2:]:
            key, _, value = f.partition("=")
            if key == "kernelpagesize_kB":
                page_kb = int(value)
            elif key.startswith("N") and key[1:].isdigit():
                counts[key] = int(value)
        for key, pages in counts.items():  # the page size comes last on the line
            nodes[key] = nodes.get(key, 0) + pages * page_kb * 1024
    if not nodes:
        return None
    out["bytes_per_node"] = nodes
    out["page_kB"] = page_kb
    return out


# path -> (thread, result box) of regions being mapped + registered in the background
_prefetched: Dict[str, Tuple[threading.Thread, dict]] = {}
_prefetch_lock = threading.Lock()


def prefetch(path: str, device_index: Optional[int] = None, numa: bool = True,
             window: int = PIN_WINDOW, cancel: Optional[threading.Event] = None) -> bool:
    """Start mapping and pinning an existing spill file in the background.

    A respawned rank calls this right after ``import torch``: the region is mapped at once and
    pinned progressively (``HostRegion(progressive=True)``: read-faulted and registered 1 GiB
    window by window in native threads), so the restore of the next
    :class:`~.checkpointer.Checkpointer` on ``path`` -- which adopts the region -- starts on
    the first pinned window instead of waiting ~2 s for all 100 GB
    (``profiles/preempt_e2e_100g_round1.md``).  Returns False when there is nothing to prefetch.
    """
    if not path or not os.path.exists(path):
        return False
    size = os.path.getsize(path)
    if size == 0:
        return False
    with _prefetch_lock:
        if path in _prefetched:
            return True
        if cancel is not None and cancel.is_set():  # the owner moved on (see watch_prefetch)
            return False
        node = -1
        if numa:
            import torch

            dev = torch.cuda.current_device() if device_index is None else device_index
            value = ctypes.c_int(-1)
            if hip().tpi_device_numa_node(dev, ctypes.byref(value)) == 0:
                node = value.value
        box: dict = {}
        try:
            box["region"] = HostRegion(size, path, device=True, numa_node=node,
                                       progressive=True, window=window)
            if os.path.exists(path + ".hbm") and box["region"].pinner:
                # a live predecessor exported its HBM: the successor will copy from there, and
                # registering 100 GB of host pages (GPU page-table updates) under its IPC
                # imports slowed them 5-20x (profiles/round5/r5ad/).  Held until the hand-off
                # is done (Checkpointer.restore_hbm) or a copy needs the region.
                hip().tpi_host_pin_hold(box["region"].pinner, 1)
        except Exception as error:  # surfaced as "not adopted"; the caller maps itself
            box["error"] = error
        _prefetched[path] = (None, box)
    return True


def watch_prefetch(path: str, cancel: threading.Event, poll: float = 0.2) -> threading.Thread:
    """:func:`prefetch` ``path`` as soon as it exists.  A hot standby starts with its rank,
    before the rank has created its spill file; mapping and pinning the file well before any
    preemption leaves the successor's restore nothing to wait for but the data.  Stops when
    ``cancel`` is set."""
    def run():
        while not cancel.is_set():
            try:
                ready = os.path.getsize(path) > 0
            except OSError:
                ready = False
            if ready:
                prefetch(path, cancel=cancel)
                return
            cancel.wait(poll)

    thread = threading.Thread(target=run, name="tpi-watch-prefetch", daemon=True)
    thread.start()
    return thread


def wait_pinned(path: str, timeout: float = 600.0, cancel: Optional[threading.Event] = None,
                poll: float = 0.01) -> Optional[float]:
    """Seconds until the prefetched region of ``path`` is mapped and pinned whole (None: no
    prefetch of ``path``, it failed, ``timeout`` passed or ``cancel`` was set).  A hot standby
    pins a 170 GB spill in a few seconds; until then its restore waits window by window."""
    import time

    t0 = time.monotonic()
    with _prefetch_lock:
        entry = _prefetched.get(path)
    if entry is None:
        return None
    thread, box = entry
    if thread is not None:  # early_prefetch(): registered whole when its thread is done
        thread.join(timeout)
    region = box.get("region")
    if region is None:
        return None
    pinner = region.pinner
    if pinner:
        lib = hip()
        lib.tpi_host_pin_hold(pinner, 0)  # someone waits for it: no longer held
        while lib.tpi_host_pin_ready(pinner) < region.size:
            if (cancel is not None and cancel.is_set()) or time.monotonic() - t0 > timeout:
                return None
            time.sleep(poll)
    return time.monotonic() - t0


def adopt(path: str, size: int) -> Optional[HostRegion]:
    """The prefetched region of ``path`` if it has exactly ``size`` bytes (waits for it)."""
    with _prefetch_lock:
        entry = _prefetched.pop(path, None)
    if entry is None:
        return None
    thread, box = entry
    if thread is not None:
        thread.join()
    region = box.get("region")
    if region is not None and region.size != size:
        region.close()
        region = None
    return region


def _torch_hip_library() -> str:
    """Path of the HIP runtime torch loads (found without importing torch)."""
    import importlib.util

    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.origin:
        raise ImportError("torch not found")
    return os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")


def early_prefetch(path: str) -> bool:
    """:func:`prefetch` that may run BEFORE ``import torch``.

    A background thread maps the spill file (MAP_POPULATE) and registers it with torch's own
    HIP runtime library (loaded by path, so torch later binds to the same one), overlapping
    the ~1.5 s of ``import torch`` of a respawned rank.  The next Checkpointer on ``path``
    adopts the region.
    """
    if not path or not os.path.exists(path):
        return False
    size = os.path.getsize(path)
    if size == 0:
        return False
    with _prefetch_lock:
        if path in _prefetched:
            return True
        box: dict = {}

        def work():
            try:
                fd = os.open(path, os.O_RDWR)
                try:
                    mm = mmap.mmap(fd, size, mmap.MAP_SHARED | getattr(mmap, "MAP_POPULATE", 0),
                                   mmap.PROT_READ | mmap.PROT_WRITE)
                finally:
                    os.close(fd)
                buf = (ctypes.c_char * size).from_buffer(mm)
                addr = ctypes.addressof(buf)
                del buf
                lib = ctypes.CDLL(_torch_hip_library(), mode=ctypes.RTLD_GLOBAL)
                lib.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
                rc = lib.hipHostRegister(ctypes.c_void_p(addr), size, 0x2 | 0x1)  # mapped|portable
                if rc != 0:
                    mm.close()
                    raise OSError("hipHostRegister failed (%d)" % rc)
                box["region"] = HostRegion(size, path, device=True, _mapped=(mm, addr))
            except Exception as error:  # surfaced as "not adopted"; the caller maps itself
                box["error"] = error

        thread = threading.Thread(target=work, name="tpi-early-prefetch", daemon=True)
        thread.start()
        _prefetched[path] = (thread, box)
    return True
