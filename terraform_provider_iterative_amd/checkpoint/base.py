"""Types the checkpoint modules share: the error, a transfer's result, and whether the
process that publishes a streamed save is still alive."""
from __future__ import annotations

import os
import struct
from dataclasses import dataclass

# The region / file format (``checkpointer`` module docstring): magic and preamble, and the
# streamed save's progress block (magic, then state 1 streaming / 2 complete / 3 failed).
MAGIC = b"TPICKPT2"
PREAMBLE = 32
PROGRESS_MAGIC = struct.unpack("<Q", b"TPIPROG1")[0]
STREAM_RUNNING, STREAM_COMPLETE, STREAM_FAILED = 1, 2, 3


class CheckpointError(RuntimeError):
    pass




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
    device_seconds: float = -1.0  # device time of the kernels alone (HBM hand-off copy)

    def __post_init__(self):
        if self.wire_bytes < 0:
            self.wire_bytes = self.bytes

    @property
    def gbps(self) -> float:
        return self.bytes / self.seconds / 1e9 if self.seconds > 0 else float("inf")


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
