"""The task communicator: RCCL over xGMI between the ranks of one task.

The reference has no collective layer -- "distribution" means every machine pulling the same
bucket prefix (``machine-script.sh.tpl:89``).  A task on the ``mi355x`` backend gets one RCCL
communicator over its ranks (``csrc/hip/stage.hip``, linked against the RCCL that ships with
torch), independent of whatever ``torch.distributed`` group the user script may build:

* the id comes from ``ncclGetUniqueId`` on rank 0 and reaches the other ranks through the
  task's state directory (``supervisor/comm-<generation>.id``, written atomically; the
  generation is ``TPI_RESTART_COUNT``, equal across a gang-respawned group), or through an
  existing ``torch.distributed`` group when there is one (:meth:`TaskComm.from_group`);
* the collectives the runtime needs for workdir fan-out: in-place all-gather (sharded
  staging, every xGMI link busy) and broadcast (the ring baseline).
"""
from __future__ import annotations

import ctypes
import json
import os
import time
from typing import Optional

from ..ops import hip

ID_BYTES = 128


class CommError(RuntimeError):
    pass


def unique_id() -> bytes:
    lib = hip()
    buf = ctypes.create_string_buffer(ID_BYTES)
    lib.check(lib.tpi_comm_unique_id(buf), "ncclGetUniqueId")
    return buf.raw


def _ptr(t) -> int:
    return t.data_ptr() if hasattr(t, "data_ptr") else int(t)


class TaskComm:
    """One rank's handle on the task communicator."""

    def __init__(self, uid: bytes, world: int, rank: int, device: int):
        if len(uid) != ID_BYTES:
            raise CommError("communicator id must be %d bytes" % ID_BYTES)
        self.lib = hip()
        self.world, self.rank, self.device = world, rank, device
        handle = self.lib.tpi_comm_init_rank(uid, world, rank, device)
        if not handle:
            raise CommError("ncclCommInitRank failed: %s" % self.lib.error())
        self.handle = handle

    # -- construction -------------------------------------------------------------------------
    @classmethod
    def from_state_dir(cls, state_dir: Optional[str] = None, rank: Optional[int] = None,
                       world: Optional[int] = None, device: Optional[int] = None,
                       timeout: float = 120.0) -> "TaskComm":
        """Inside a task: rank 0 publishes the id in ``state_dir`` (default the task's
        ``supervisor/``), the others wait for it."""
        env = os.environ
        state_dir = state_dir or os.path.join(env["TPI_TASK_DIRECTORY"], "supervisor")
        rank = int(env.get("RANK", "0")) if rank is None else rank
        world = int(env.get("WORLD_SIZE", "1")) if world is None else world
        if device is None:
            mine = env.get("TPI_RANK_GPUS", "")
            device = int(mine.split(",")[0]) if mine else 0
        path = os.path.join(state_dir, "comm-%s.id" % env.get("TPI_RESTART_COUNT", "0"))
        if rank == 0:
            uid = unique_id()
            tmp = "%s.tmp.%d" % (path, os.getpid())
            with open(tmp, "w") as handle:
                json.dump({"id": uid.hex(), "world": world, "time": time.time()}, handle)
            os.replace(tmp, path)
        else:
            deadline = time.time() + timeout
            while True:
                try:
                    with open(path) as handle:
                        uid = bytes.fromhex(json.load(handle)["id"])
                    break
                except (OSError, ValueError, KeyError):
                    if time.time() > deadline:
                        raise CommError("no communicator id at %s after %.0f s" % (path, timeout))
                    time.sleep(0.005)
        return cls(uid, world, rank, device)

    @classmethod
    def from_group(cls, group=None, device: Optional[int] = None) -> "TaskComm":
        """Share the id through an initialised ``torch.distributed`` group."""
        import torch
        import torch.distributed as dist

        rank, world = dist.get_rank(group), dist.get_world_size(group)
        box = [unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0, group=group)
        if device is None:
            device = torch.cuda.current_device()
        return cls(box[0], world, rank, device)

    # -- collectives ----------------------------------------------------------------------------
    def allgather_inplace(self, buf, shard_bytes: int, sync: bool = True) -> None:
        """Every rank's shard ``buf[rank*shard_bytes : (rank+1)*shard_bytes]`` to every rank."""
        comms = (ctypes.c_void_p * 1)(self.handle)
        bufs = (ctypes.c_void_p * 1)(_ptr(buf))
        self.lib.check(self.lib.tpi_comm_allgather_inplace(comms, 1, bufs, shard_bytes,
                                                           1 if sync else 0), "all-gather")

    def broadcast(self, buf, nbytes: int, root: int = 0, sync: bool = True) -> None:
        comms = (ctypes.c_void_p * 1)(self.handle)
        bufs = (ctypes.c_void_p * 1)(_ptr(buf))
        self.lib.check(self.lib.tpi_comm_broadcast(comms, 1, bufs, nbytes, root,
                                                   1 if sync else 0), "broadcast")

    def synchronize(self) -> None:
        comms = (ctypes.c_void_p * 1)(self.handle)
        self.lib.check(self.lib.tpi_comm_sync(comms, 1), "comm sync")

    def close(self) -> None:
        if self.handle:
            self.lib.tpi_comm_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
