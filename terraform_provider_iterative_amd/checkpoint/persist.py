"""Persisting a checkpoint to a file (local, or an off-node container) and loading it back:
the :class:`~.checkpointer.Checkpointer` mixin behind ``persist`` / ``load``.

The file is one slot of the region layout (``checkpointer`` module docstring).  Reference:
the task's final copy of its data to the bucket and the restore from it
(``task/common/machine/machine-script.sh.tpl:89,118-124``).
"""
from __future__ import annotations

import ctypes
import os
import tempfile
import threading

import numpy as np

from ..ops import native
from .base import (PREAMBLE, PROGRESS_MAGIC, STREAM_COMPLETE, STREAM_FAILED, STREAM_RUNNING,
                   CheckpointError, TransferResult)

FILE_THREADS = 16        # persist / load: native pwrite/pread threads
LOAD_CHUNK = 256 << 20   # load: bytes read (and published to the restore) per step


def _local_scratch(remote_path: str) -> str:
    """Where a checkpoint bound for (or fetched from) another node is staged on this one:
    ``TPI_PERSIST_TMPDIR``, else the task directory, else the temp directory."""
    base = (os.environ.get("TPI_PERSIST_TMPDIR") or os.environ.get("TPI_TASK_DIRECTORY")
            or tempfile.gettempdir())
    return os.path.join(base, ".tpi-persist-%d-%s" % (os.getpid(),
                                                     os.path.basename(remote_path) or "ckpt"))


class Persistence:
    """The file half of :class:`~.checkpointer.Checkpointer` (a mixin)."""

    def persist(self, path: str) -> str:
        """Write the current checkpoint (header, CRCs, stream: one slot) to ``path``
        atomically.  ``path`` may name a file on another node or in a bucket (``ssh://host/dir/
        file``, ``host:/dir/file``, ``s3://``/``gs://``/``az://bucket/key``: an off-node
        ``storage.container``, :mod:`..storage.remote`); the slot then goes there straight
        from the host region, with no local temporary file."""
        from ..storage import remote

        self.wait_pending()
        active = self._active()
        if active is None:
            raise CheckpointError("nothing saved yet")
        slot, header = active
        if remote.is_remote(path):
            nbytes = self.stream_offset + int(header["stream_bytes"])
            view = memoryview((ctypes.c_char * nbytes).from_address(
                self.region.addr + slot.base)).cast("B")
            remote.store_bytes(view, path)
            return path
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
        :meth:`persist`): an object in a bucket is read in place by ranged requests, streamed
        the same way; a file on an SSH node is fetched first."""
        from ..storage import remote

        obj = None
        if remote.is_remote(path):
            obj = remote.object_source(path)
            if obj is None:
                tmp = remote.fetch(path, os.path.dirname(_local_scratch(path)))
                try:
                    return self.load(tmp)
                finally:
                    os.remove(tmp)
        self.wait_pending()
        self._wait_writers()
        slot, generation = self._target()
        if obj is None:
            with open(path, "rb") as f:
                head = np.frombuffer(f.read(PREAMBLE + self.header_cap), np.uint8)
                size = os.fstat(f.fileno()).st_size
        else:
            size = obj[0].size(obj[1])
            if size is None:
                raise CheckpointError("no checkpoint at %s" % path)
            head = np.frombuffer(obj[0].read(obj[1], 0, min(size, PREAMBLE + self.header_cap)),
                                 np.uint8)
        header = self.read_header(head)
        self._check_compatible(header)
        if not header.get("complete"):
            raise CheckpointError("%s holds an incomplete checkpoint" % path)
        stream_bytes = int(header["stream_bytes"])
        end = self.stream_offset + stream_bytes
        if size < end:
            raise CheckpointError("%s is truncated (%d of %d bytes)" % (path, size, end))
        self._invalidate(slot)
        # entries + CRCs + blob sizes first (small), then the stream, streamed
        if obj is None:
            native().read_stream_ptr(path, self.region.addr + slot.base + self.entries_offset,
                                     self.entries_offset,
                                     self.stream_offset - self.entries_offset,
                                     FILE_THREADS, 64 << 20, 0, 0, 0)
        else:
            obj[0].read_into(obj[1], self.region.addr + slot.base + self.entries_offset,
                             self.entries_offset, self.stream_offset - self.entries_offset)
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

        def publish(done: int) -> None:  # as read_stream's words: bytes, then whole tiles
            prog[3] = done
            prog[2] = int(np.searchsorted(tile_ends, np.uint64(done), side="right"))

        def read():
            try:
                if obj is None:
                    native().read_stream_ptr(path,
                                             self.region.addr + slot.base + self.stream_offset,
                                             self.stream_offset, stream_bytes, FILE_THREADS,
                                             LOAD_CHUNK, prog.ctypes.data + 16,
                                             tile_ends.ctypes.data, len(tile_ends))
                else:
                    obj[0].read_into(obj[1], self.region.addr + slot.base + self.stream_offset,
                                     self.stream_offset, stream_bytes, publish)
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
