"""Which step boundary do the ranks of a job checkpoint at?

A preempted gang must save the *same* step on every rank, or its successors resume from
mismatched states (weights of step k on one rank, k+1 on another).  The reference never faces
this -- its recovery restores the last 10 s workdir sync and leaves consistency to the user
script (``machine-script.sh.tpl:89,118-124``; ``README.md:88-101``) -- so the protocol here is
new.  Every rank calls the step-boundary hook (:func:`.preemption.step`) at the same points of
its loop; at each call it learns whether this boundary is a preemption and/or a periodic save
point.  Three implementations, chosen once at the first boundary:

``ShmAgreement``        ranks on one host (the node runtime's case): one cache line per rank
                        in a shared mapping (``csrc/native/ctl.cpp``).  Per step: one store,
                        two loads -- no collective, no host/device sync.  A preempted rank
                        proposes its own boundary, or the one after the furthest peer's;
                        every rank saves at that boundary.
``CollectiveAgreement`` ranks on several hosts: one 2-int all-reduce per boundary
                        (``max`` of the preempt flags, ``min`` of the periodic due flags).
``LocalAgreement``      a single process: its own flag decides.
"""
from __future__ import annotations

import mmap
import os
import socket
import sys
import uuid
from typing import Optional, Tuple

from ..ops import native


def _host_identity() -> str:
    try:
        with open("/proc/sys/kernel/random/boot_id") as f:
            boot = f.read().strip()
    except OSError:
        boot = ""
    return "%s/%s" % (socket.gethostname(), boot)


def _dist():
    """``torch.distributed`` when a multi-rank default group is up, else None."""
    dist = sys.modules.get("torch.distributed")
    if dist is None or not dist.is_available() or not dist.is_initialized():
        return None
    return dist if dist.get_world_size() > 1 else None


class LocalAgreement:
    kind = "local"

    def __init__(self):
        self.ordinal = 0

    def arrive(self, preempt: bool, due: bool) -> Tuple[bool, bool]:
        """(save for preemption here, take a periodic checkpoint here)."""
        self.ordinal += 1
        return preempt, due

    def close(self) -> None:
        pass


class ShmAgreement:
    """Ranks of one host: the control block of ``csrc/native/ctl.h`` in a shared mapping.

    Rank 0 creates the block in ``/dev/shm`` and broadcasts its name; once every rank has
    mapped it, the file is unlinked, so nothing outlives the job."""

    kind = "shm"

    def __init__(self, dist, shm_dir: str = "/dev/shm"):
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.ordinal = 0
        lib = native()
        size = int(lib.ctl_bytes(self.world))
        name = [None]
        if self.rank == 0:
            path = os.path.join(shm_dir, "tpi-ctl-%s" % uuid.uuid4().hex)
            fd = os.open(path, os.O_RDWR | os.O_CREAT | os.O_EXCL, 0o600)
            os.ftruncate(fd, size)
            self._map = mmap.mmap(fd, size)
            os.close(fd)
            self._addr = _address(self._map)
            lib.ctl_init(self._addr, self.world)
            name[0] = path
        dist.broadcast_object_list(name, src=0)
        if self.rank != 0:
            fd = os.open(name[0], os.O_RDWR)
            self._map = mmap.mmap(fd, size)
            os.close(fd)
            self._addr = _address(self._map)
        mapped = [None] * self.world
        dist.all_gather_object(mapped, bool(lib.ctl_valid(self._addr, self.world)))
        if self.rank == 0:
            os.unlink(name[0])
        if not all(mapped):
            raise RuntimeError("step-boundary control block not visible on every rank")
        self.preempt_target = 0
        self.proposed = False
        self._lib = lib

    def arrive(self, preempt: bool, due: bool) -> Tuple[bool, bool]:
        self.ordinal += 1
        pre, per = self._lib.ctl_arrive(self._addr, self.rank, self.ordinal)
        if preempt and not pre:
            pre = self._lib.ctl_propose_preempt(self._addr, self.world, self.rank)
        self.proposed = False
        if due and self.rank == 0:  # one clock decides the periodic cadence
            proposed = self._lib.ctl_propose_periodic(self._addr, self.world, self.rank)
            self.proposed = bool(proposed)
            per = proposed or per
        if pre and self.ordinal > pre:  # cannot happen by the protocol; never skip a save
            pre = self.ordinal
        self.preempt_target = pre
        return bool(pre) and self.ordinal >= pre, bool(per) and self.ordinal == per

    def close(self) -> None:
        pass  # the mapping is released with the process (a save may still be running)


class CollectiveAgreement:
    """Ranks on several hosts: a blocking 2-int all-reduce per boundary."""

    kind = "collective"

    def __init__(self, dist):
        import torch

        self.dist = dist
        self.ordinal = 0
        self.device = torch.device("cpu")
        if dist.get_backend() == "nccl":
            self.device = torch.device("cuda", torch.cuda.current_device())

    def arrive(self, preempt: bool, due: bool) -> Tuple[bool, bool]:
        import torch

        self.ordinal += 1
        flags = torch.tensor([-1 if preempt else 0, 1 if due else 0], dtype=torch.int32,
                             device=self.device)
        self.dist.all_reduce(flags, op=self.dist.ReduceOp.MIN)
        pre, per = flags.tolist()
        return pre < 0, per > 0

    def close(self) -> None:
        pass


def _address(buf: mmap.mmap) -> int:
    import ctypes

    return ctypes.addressof(ctypes.c_char.from_buffer(buf))


def create(mode: Optional[str] = None):
    """The agreement for this process (collective calls when a multi-rank group is up: call
    it on every rank at the same point).  ``TPI_AGREEMENT`` = ``shm`` / ``collective`` /
    ``local`` overrides the choice."""
    mode = mode or os.environ.get("TPI_AGREEMENT", "auto")
    dist = _dist()
    if dist is None or mode == "local":
        return LocalAgreement()
    if mode == "collective":
        return CollectiveAgreement(dist)
    hosts = [None] * dist.get_world_size()
    dist.all_gather_object(hosts, _host_identity())
    if len(set(hosts)) == 1 and os.path.isdir("/dev/shm"):
        return ShmAgreement(dist)
    return CollectiveAgreement(dist)
