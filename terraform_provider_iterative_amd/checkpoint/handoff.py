"""The same-GPU HBM hand-off of a preempted rank's state (the "hot" recovery path).

Reference: a reclaimed spot VM is replaced and the new one restores the bucket's ``data/``
prefix before the task runs again (``task/common/machine/machine-script.sh.tpl:89``); the group
scales to 0 right after the task exits (``:10-15,51``).  Here a preempted rank (the
*predecessor*) and its successor on the same GPU hand the state over device to device:

* :meth:`HbmHandoff.export_hbm` (predecessor): one manifest next to the spill file
  (``<spill>.hbm``) with a HIP IPC handle per allocation holding the state; tensors of
  allocations HIP IPC cannot open (2 GiB or more) are first relocated into 1 GiB blocks
  (:data:`HBM_ROUTES`, ``profiles/round5/ipc_cause.md``);
* :meth:`HbmHandoff.restore_hbm` (successor): claims the hand-off, maps every allocation
  (bounded by ``TPI_IPC_OPEN_TIMEOUT``), checks every copy descriptor on the host, copies with
  the fused copy + read-back kernels (``csrc/hip/kernels.hip`` ``k_stream_hash``), and unmaps
  behind the restore;
* the claim file (``<spill>.hbm.claim``, created atomically with its pid) decides who owns the
  exported memory's fate, so the predecessor never exits while its memory is mapped elsewhere.

The full state machine, with the supervisor's side, is the "Hand-off modes" table of
``docs/ARCHITECTURE.md``.
"""
from __future__ import annotations

import ctypes
import json
import os
import socket
import struct
import threading
import time
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from ..ops import hip
from ..ops.packing import SEG_CONTIG
from .base import CheckpointError, TransferResult, _writer_alive

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


class HbmHandoff:
    """The hand-off half of :class:`~.checkpointer.Checkpointer` (a mixin: it uses the
    checkpointer's ``path``, ``engine``, ``plan``, ``device_index`` and digests)."""

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
        try:
            return self._publish_hbm(manifest, lib, route, sizes, raw_where, big, pieces,
                                     metadata)
        except BaseException:
            # nothing was published: the relocated copies would otherwise stay allocated
            # through the whole save and the successor's allocation
            self._free_relocated()
            raise

    def _publish_hbm(self, manifest: str, lib, route: str, sizes: Dict[int, int],
                     raw_where: List[Optional[Tuple[int, int]]], big: set,
                     pieces: Dict[str, List[List[int]]], metadata: Optional[Dict]) -> str:
        """The second half of :meth:`export_hbm`: IPC handles (and dma-bufs) of every
        allocation, then the manifest, written atomically."""
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
        offset, size = ctypes.c_uint64(0), ctypes.c_uint64(0)
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
        """See :meth:`_restore_hbm`; the host region's pinning, held while the hand-off runs
        (:func:`host.prefetch`), resumes when it ends, however it ends."""
        try:
            return self._restore_hbm(strict)
        finally:
            region = getattr(self, "region", None)
            if region is not None and getattr(region, "pinner", None):
                hip().tpi_host_pin_hold(region.pinner, 0)

    def _restore_hbm(self, strict: bool = True) -> TransferResult:
        """Copy the state of a preempted predecessor on the same GPU straight from its HBM
        (its allocations mapped here over dma-buf, or HIP IPC for an ``ipc`` export; one
        fused copy pass + a read-back verify, every tile's digest checked) into the bound
        tensors."""
        t_entry = time.perf_counter()
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
        phases = {"claim": t0 - t_entry}  # seconds per step, for the journal
        self.hbm_phases = phases
        try:
            limit = float(os.environ.get("TPI_IPC_OPEN_TIMEOUT", "10"))
        except ValueError:
            limit = 10.0

        # Set (under ``gate``) once the hand-off has been given up or closed: an opener thread
        # that returns from the driver after that closes its new mapping at once instead of
        # recording it -- nothing would ever unmap it, and the predecessor has been told it may
        # exit.
        gate = threading.Lock()
        given_up = [False]

        def open_ipc(i: int) -> None:
            base = ctypes.c_void_p()
            lib.check(lib.tpi_ipc_open(bytes.fromhex(ipc[i]), self.device_index,
                                       ctypes.byref(base)), "tpi_ipc_open")
            with gate:
                if not given_up[0]:
                    bases[i] = mapped[i] = base.value
                    return
            lib.tpi_ipc_close(base)

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
                            with gate:
                                late = given_up[0]
                                if not late:
                                    mapped[i] = ptr.value
                                    via_dmabuf[i] = True
                            if late:
                                lib.tpi_dmabuf_unmap(ptr)
                                raise CheckpointError("the hand-off was given up")
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
            with gate:
                given_up[0] = True  # from now on late openers close their own mappings
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

            try:  # TPI_IPC_OPEN_THREADS: concurrent imports (driver calls)
                nthreads = max(1, int(os.environ.get("TPI_IPC_OPEN_THREADS", "8")))
            except ValueError:
                nthreads = 8
            workers = [threading.Thread(target=worker, name="tpi-ipc-open", daemon=True)
                       for _ in range(min(nthreads, len(todo)))]
            if doc.get("socket"):
                workers.append(threading.Thread(target=receiver, name="tpi-dmabuf-open",
                                                daemon=True))
            for w in workers:
                w.start()
            deadline = time.monotonic() + limit
            try:  # meanwhile: this process's destinations (the plan's segments), checked once
                key = self.plan.segs.tobytes()
                if getattr(self, "_dst_checked", None) != key:
                    _check_destinations(self.plan.segs, lib)
                    self._dst_checked = key
            except BaseException as error:
                with lock:
                    todo.clear()
                    errors.append(error)
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
            self.hbm_open_s = phases["open"] = time.perf_counter() - t0
            t1 = time.perf_counter()
            src = np.frombuffer(bytes.fromhex(doc["segs"]), dtype=self.plan.segs.dtype).copy()
            if len(src) != len(self.plan.segs):
                raise CheckpointError("HBM hand-off describes a different tensor set")
            # each segment's mapped allocation and offset in it, as arrays (-1: none)
            where = doc["where"]
            owner = np.array([-1 if w is None else int(w[0]) for w in where], dtype=np.int64)
            offs = np.array([0 if w is None else int(w[1]) for w in where], dtype=np.uint64)
            if len(owner) != len(src):
                raise CheckpointError("HBM hand-off: %d locations for %d segments"
                                      % (len(owner), len(src)))
            base_of = np.array([0 if b is None else b for b in bases] + [0], dtype=np.uint64)
            src["ptr"] = np.where(owner < 0, np.uint64(0),
                                  base_of[np.where(owner < 0, len(bases), owner)] + offs)
            dst = self.plan.segs
            if doc.get("pieces"):
                src, dst, owner = _split_relocated(src, self.plan.segs, doc["pieces"], bases,
                                                   owner)
            # never launch a copy that could touch memory outside what is mapped: every source
            # segment inside its mapped allocation, every destination inside its own
            # (relocated pieces split contiguous destination segments of the plan, whose
            # bounds open_all checked: they need no second look)
            _check_copy_ranges(src, owner, bases, sizes, None, lib)
            t2 = time.perf_counter()
            phases["plan"] = t2 - t1
            try:  # diagnostic for the journal
                self.hbm_free_before_copy = torch.cuda.mem_get_info(self.device_index)[0]
            except Exception:
                self.hbm_free_before_copy = 0
            sig = torch.cuda.current_stream(self.device_index).cuda_stream
            t3 = time.perf_counter()
            phases["meminfo"] = t3 - t2
            try:
                res = self.engine.copy_segments(src, self.plan, sig, dst)  # synchronous
            except BaseException as error:
                self.hbm_fault_dump = _dump_copy_plan(self._hbm_manifest_path(), src, dst,
                                                      owner, bases, sizes, doc, error,
                                                      self.device_index,
                                                      getattr(self, "hbm_device_state", None))
                raise
            phases["copy"] = time.perf_counter() - t3
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


def _dump_copy_plan(manifest: str, src: np.ndarray, dst: np.ndarray, owner: np.ndarray,
                    bases: List[Optional[int]], sizes: List[int], doc: Dict,
                    error: BaseException, device_index: int = 0,
                    device_state: Optional[Dict] = None) -> Optional[str]:
    """Evidence of a failed hand-off copy (``<manifest>.fault.json``): every source and
    destination descriptor the kernel was given, each source's mapped allocation
    ``[base, base + size)``, the relocation pieces, and what the driver held on the device --
    so a fault can be tied to an address instead of to timing."""
    path = (manifest or "/tmp/tpi-hbm") + ".fault.%d.json" % os.getpid()
    try:
        from ..parallel.placement import device_vram_usage

        def segs(a: np.ndarray) -> List[List[int]]:
            return [[int(x["ptr"]), int(x["nbytes"]), int(x["kind"]), int(x["off"])] for x in a]

        usage = None
        try:
            usage = device_vram_usage(device_index)
        except Exception:
            pass
        at_fault = None
        if device_state and device_state.get("pci"):  # sysfs: readable after the fault too
            from ..parallel.placement import orphaned_vram

            at_fault = orphaned_vram(device_state["pci"])
        with open(path, "w") as f:
            json.dump({"error": str(error), "time": time.time(), "predecessor": doc.get("pid"),
                       "src": segs(src), "dst": segs(dst), "owner": [int(o) for o in owner],
                       "mapped": [[None if b is None else int(b), int(n)]
                                  for b, n in zip(bases, sizes)],
                       "pieces": doc.get("pieces"), "vram_used_total": usage,
                       "device_before_copy": device_state, "device_at_fault": at_fault}, f)
        return path
    except Exception:
        return None


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
                       sizes: List[int], dst: Optional[np.ndarray], lib) -> None:
    """Host-side bounds check before the hand-off's copy kernel: each source segment must lie
    inside the predecessor allocation it was mapped from (``owner``), each destination segment
    inside the device allocation holding it in this process (``dst`` None: checked already,
    :func:`_check_destinations`).  A descriptor that fails raises CheckpointError (the caller
    restores from the host copy) instead of faulting the GPU."""
    live = src["nbytes"] != 0
    contig = live & (src["kind"] == SEG_CONTIG)
    if np.any(owner[live] < 0):
        i = int(np.flatnonzero(live & (owner < 0))[0])
        raise CheckpointError("HBM hand-off: source segment %d has no mapped allocation" % i)
    if any(bases[int(a)] is None for a in np.unique(owner[live])):
        raise CheckpointError("HBM hand-off: a source segment's allocation is not mapped")
    # contiguous segments (nearly all): one vector comparison against their allocations
    base_of = np.array([0 if b is None else b for b in bases] + [0], dtype=np.uint64)
    size_of = np.array(list(sizes) + [0], dtype=np.uint64)
    own = np.where(owner < 0, len(bases), owner)
    lo = src["ptr"].astype(np.uint64)
    hi = lo + src["nbytes"].astype(np.uint64)
    bad = contig & ((lo < base_of[own]) | (hi > base_of[own] + size_of[own]))
    for i in list(np.flatnonzero(bad)) + list(np.flatnonzero(live & ~contig)):
        a = int(owner[i])
        lo_i, hi_i = _seg_extent(src[i])
        if lo_i < bases[a] or hi_i > bases[a] + sizes[a]:
            raise CheckpointError(
                "HBM hand-off: source segment %d [%#x, %#x) lies outside its mapped allocation "
                "%d [%#x, +%d)" % (i, lo_i, hi_i, a, bases[a], sizes[a]))
    if dst is not None:
        _check_destinations(dst, lib)


def _check_destinations(dst: np.ndarray, lib) -> None:
    """Every destination segment inside the device allocation that holds it (one driver
    query per allocation: segments are sorted, consecutive ones often share one)."""
    base, size = ctypes.c_uint64(0), ctypes.c_uint64(0)
    known: Tuple[int, int] = (1, 0)  # [lo, hi) of the last allocation looked up
    for i in range(len(dst)):
        if int(dst[i]["nbytes"]) == 0:
            continue
        lo, hi = _seg_extent(dst[i])
        if not (known[0] <= lo and hi <= known[1]):
            if lib.tpi_mem_range(ctypes.c_void_p(int(dst[i]["ptr"])), ctypes.byref(base),
                                 ctypes.byref(size)) != 0:
                raise CheckpointError("HBM hand-off: destination segment %d is not device "
                                      "memory" % i)
            known = (int(base.value), int(base.value) + int(size.value))
        if lo < known[0] or hi > known[1]:
            raise CheckpointError(
                "HBM hand-off: destination segment %d [%#x, %#x) lies outside its allocation "
                "[%#x, +%d)" % (i, lo, hi, known[0], known[1] - known[0]))


def _split_relocated(src: np.ndarray, dst: np.ndarray, pieces: Dict[str, List[List[int]]],
                     bases: List[Optional[int]], owner: np.ndarray
                     ) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Source and destination descriptors for an HBM hand-off whose exporter relocated some
    tensors into blocks (:meth:`Checkpointer._relocate`): each such segment becomes one
    contiguous segment per block, the destination split at the same stream offsets.  Both
    stay sorted by stream offset, so the copy and its verification see the same stream.
    ``owner`` (mapped allocation per segment) is expanded alongside.  The segments between
    relocated ones are carried over as whole slices."""
    out_src, out_dst, out_owner = [], [], []
    prev = 0
    for i in sorted(int(k) for k in pieces):
        parts = pieces[str(i)]
        if not parts:
            continue
        out_src.append(src[prev:i])
        out_dst.append(dst[prev:i])
        out_owner.append(owner[prev:i])
        prev = i + 1
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
            out_owner.append(np.array([alloc], np.int64))
            done += n
    out_src.append(src[prev:])
    out_dst.append(dst[prev:])
    out_owner.append(owner[prev:])
    return (np.concatenate(out_src), np.concatenate(out_dst),
            np.concatenate(out_owner).astype(np.int64))


class _SpillOffer(HbmHandoff):
    """The claim protocol of the HBM offer next to a spill file, without a checkpointer (a
    successor deciding before it has allocated anything)."""

    def __init__(self, spill: str):
        self._spill = spill

    def _hbm_manifest_path(self) -> Optional[str]:
        return self._spill + ".hbm"


def decline_hbm_handoff(spill: str) -> bool:
    """Successor side: withdraw the predecessor's HBM offer next to ``spill`` -- claim it, then
    remove the manifest and the claim -- because this process cannot make room for its own copy
    of the state next to the exported one.  The predecessor, waiting for a claimer
    (``preemption._await_successor``), sees "successor closed" at once and exits, which gives
    its HBM back; the successor restores from the host copy.  False: no offer, or another
    process holds it."""
    offer = _SpillOffer(spill)
    manifest = offer._hbm_manifest_path()
    if not os.path.exists(manifest) or not offer.claim_hbm():
        return False
    try:
        os.remove(manifest)  # first: the claim's removal then reads as "closed"
    except OSError:
        pass
    offer.release_hbm_claim()
    return True
