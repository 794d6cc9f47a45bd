"""GPU inventory and placement leases for the ``mi355x`` provider.

The reference asks a cloud for machines (ASG/MIG/VMSS capacity = ``parallelism``); here the
"machine" is a set of GPUs of this node.  Concurrent tasks get disjoint GPU sets through
lease files under ``<state_root>/placement`` guarded by ``flock``; a lease names its task and
is released by the task's supervisor when it exits (the scaling group going to 0).  Stale
leases (task gone, supervisor dead) are reclaimed on the next allocation.

Inventory comes from the KFD topology in sysfs (no HIP initialisation, so the CLI stays
cheap and never touches the GPU): every node with a non-zero ``gfx_target_version`` is a
GPU, numbered like HIP does, filtered by ``ROCR_VISIBLE_DEVICES``/``HIP_VISIBLE_DEVICES``.
``TPI_MI355X_GPUS=0,1,...`` overrides it (tests and CPU-only rehearsals use it).
"""
from __future__ import annotations

import fcntl
import json
import os
import time
from contextlib import contextmanager
from typing import Dict, Iterator, List, Optional

from ..utils.record import field, record

KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"


@record
class GPU:
    index: int                 # HIP device index on this node
    gfx: str = ""              # e.g. "gfx950"
    numa_node: int = -1
    pci: str = ""
    cus: int = 0
    cpus: List[int] = field(default_factory=list)  # NUMA-local CPU cores

    def to_json(self) -> dict:
        return {"index": self.index, "gfx": self.gfx, "numa_node": self.numa_node,
                "pci": self.pci, "cus": self.cus}


def _read(path: str) -> str:
    try:
        with open(path) as handle:
            return handle.read()
    except OSError:
        return ""


def _cpulist(spec: str) -> List[int]:
    cpus: List[int] = []
    for part in spec.strip().split(","):
        if not part:
            continue
        lo, _, hi = part.partition("-")
        cpus.extend(range(int(lo), int(hi or lo) + 1))
    return cpus


def _gfx_name(version: int) -> str:
    major, minor, step = version // 10000, (version // 100) % 100, version % 100
    return "gfx%d%d%x" % (major, minor, step)


def _visible_filter(gpus: List[GPU], environ) -> List[GPU]:
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        value = environ.get(var)
        if value:
            keep = [int(x) for x in value.split(",") if x.strip().isdigit()]
            gpus = [gpus[i] for i in keep if i < len(gpus)]
            for new_index, gpu in enumerate(gpus):
                gpu.index = new_index
    return gpus


def discover(environ=None) -> List[GPU]:
    """GPUs of this node (see module docstring)."""
    environ = os.environ if environ is None else environ
    override = environ.get("TPI_MI355X_GPUS")
    if override is not None:
        return [GPU(index=int(x), gfx="gfx950") for x in override.split(",") if x.strip()]
    gpus: List[GPU] = []
    try:
        nodes = sorted(os.listdir(KFD_NODES), key=lambda n: int(n) if n.isdigit() else 1 << 30)
    except OSError:
        return gpus
    for node in nodes:
        props = {}
        for line in _read(os.path.join(KFD_NODES, node, "properties")).splitlines():
            key, _, value = line.partition(" ")
            props[key] = value.strip()
        version = int(props.get("gfx_target_version", "0") or 0)
        if not version:
            continue
        minor = props.get("drm_render_minor")
        if minor and os.path.exists("/dev/dri") and \
                not os.access("/dev/dri/renderD%s" % minor, os.R_OK | os.W_OK):
            continue  # not ours (container/cgroup); ROCr would not enumerate it either
        gpu = GPU(index=len(gpus), gfx=_gfx_name(version),
                  cus=int(props.get("simd_count", "0") or 0) // 4)
        if minor:
            dev = "/sys/class/drm/renderD%s/device" % minor
            numa = _read(os.path.join(dev, "numa_node")).strip()
            gpu.numa_node = int(numa) if numa.lstrip("-").isdigit() else -1
            gpu.pci = os.path.basename(os.path.realpath(dev))
            if gpu.numa_node >= 0:
                gpu.cpus = _cpulist(_read("/sys/devices/system/node/node%d/cpulist"
                                          % gpu.numa_node))
        gpus.append(gpu)
    return _visible_filter(gpus, environ)


class PlacementError(RuntimeError):
    pass


class Placement:
    """Lease-file allocator over the node's GPUs."""

    LEASE_GRACE = 120.0  # a lease without a live supervisor yet is kept this long

    def __init__(self, state_root: str, gpus: Optional[List[GPU]] = None):
        self.root = os.path.join(state_root, "placement")
        os.makedirs(self.root, exist_ok=True)
        self.gpus = discover() if gpus is None else gpus

    def lease_path(self, index: int) -> str:
        return os.path.join(self.root, "gpu-%d.lease" % index)

    @contextmanager
    def _locked(self) -> Iterator[None]:
        fd = os.open(os.path.join(self.root, "placement.lock"), os.O_RDWR | os.O_CREAT, 0o644)
        try:
            fcntl.flock(fd, fcntl.LOCK_EX)
            yield
        finally:
            fcntl.flock(fd, fcntl.LOCK_UN)
            os.close(fd)

    def _read_lease(self, index: int) -> Optional[dict]:
        raw = _read(self.lease_path(index))
        if not raw:
            return None
        try:
            return json.loads(raw)
        except ValueError:
            return {"task": "?", "created": 0}

    @staticmethod
    def _alive(lease: dict) -> bool:
        task_dir = lease.get("task_dir")
        if task_dir and not os.path.isdir(task_dir):
            return False
        state = _read(os.path.join(task_dir or "", "supervisor", "state.json"))
        if state:
            try:
                data = json.loads(state)
            except ValueError:
                data = {}
            if data.get("phase") == "stopped":
                return False
            pid = int(data.get("pid", 0) or 0)
            if pid and _pid_alive(pid):
                return True
        created = float(lease.get("created", 0))
        return time.time() - created < Placement.LEASE_GRACE

    def leases(self) -> Dict[int, dict]:
        out = {}
        for gpu in self.gpus:
            lease = self._read_lease(gpu.index)
            if lease is not None:
                out[gpu.index] = lease
        return out

    def free(self) -> List[GPU]:
        with self._locked():
            return self._free_locked()

    def _free_locked(self) -> List[GPU]:
        free = []
        for gpu in self.gpus:
            lease = self._read_lease(gpu.index)
            if lease is not None and self._alive(lease):
                continue
            if lease is not None:  # stale
                try:
                    os.unlink(self.lease_path(gpu.index))
                except FileNotFoundError:
                    pass
            free.append(gpu)
        return free

    def held_by(self, task_id: str) -> List[GPU]:
        return [g for g in self.gpus if (self._read_lease(g.index) or {}).get("task") == task_id]

    def allocate(self, task_id: str, count: int, task_dir: str = "",
                 prefer_numa: bool = True) -> List[GPU]:
        """Lease ``count`` GPUs for ``task_id`` (idempotent: returns existing leases)."""
        if count <= 0:
            return []
        if count > len(self.gpus):
            raise PlacementError("task needs %d GPUs; this node has %d" % (count, len(self.gpus)))
        with self._locked():
            held = self.held_by(task_id)
            if len(held) >= count:
                return held[:count]
            free = [g for g in self._free_locked() if g not in held]
            need = count - len(held)
            if len(free) < need:
                busy = sorted({l.get("task", "?") for l in self.leases().values()})
                raise PlacementError("not enough free GPUs: need %d, free %d (held by %s)"
                                     % (need, len(free), ", ".join(busy) or "-"))
            chosen = self._choose(free, need, prefer_numa)
            now = time.time()
            for gpu in chosen:
                tmp = self.lease_path(gpu.index) + ".tmp"
                with open(tmp, "w") as handle:
                    json.dump({"task": task_id, "task_dir": task_dir, "created": now,
                               "creator_pid": os.getpid(), "gpu": gpu.index}, handle)
                os.replace(tmp, self.lease_path(gpu.index))
            return sorted(held + chosen, key=lambda g: g.index)

    @staticmethod
    def _choose(free: List[GPU], need: int, prefer_numa: bool) -> List[GPU]:
        """Prefer GPUs of one NUMA node (host-memory locality for spills), then contiguous
        indices (fewest distinct sockets)."""
        if prefer_numa:
            by_node: Dict[int, List[GPU]] = {}
            for gpu in free:
                by_node.setdefault(gpu.numa_node, []).append(gpu)
            fitting = [g for g in by_node.values() if len(g) >= need]
            if fitting:
                best = min(fitting, key=len)  # tightest fit keeps big blocks for big tasks
                return sorted(best, key=lambda g: g.index)[:need]
        return sorted(free, key=lambda g: g.index)[:need]

    def release(self, task_id: str) -> int:
        with self._locked():
            n = 0
            for gpu in self.held_by(task_id):
                try:
                    os.unlink(self.lease_path(gpu.index))
                    n += 1
                except FileNotFoundError:
                    pass
            return n


def numa_cpus(node: int) -> List[int]:
    """CPU cores of NUMA node ``node`` (empty when unknown)."""
    if node is None or node < 0:
        return []
    return _cpulist(_read("/sys/devices/system/node/node%d/cpulist" % node))


def pin_to_numa(node: int) -> Optional[List[int]]:
    """Restrict this process to the cores of NUMA node ``node`` that it may already use
    (``TPI_NUMA_PIN=0`` disables).  Returns the new affinity, or None if nothing changed."""
    if os.environ.get("TPI_NUMA_PIN", "1") == "0" or not hasattr(os, "sched_setaffinity"):
        return None
    cpus = set(numa_cpus(node)) & set(os.sched_getaffinity(0))
    if not cpus:
        return None
    os.sched_setaffinity(0, cpus)
    return sorted(cpus)


def pin_to_device_numa(device_index: int) -> Optional[List[int]]:
    """:func:`pin_to_numa` for the socket of HIP device ``device_index`` (resolved through
    its PCI bus id, so it agrees with HIP's numbering under any visible-device mask)."""
    import ctypes

    from ..ops import hip

    lib = hip(required=False)
    if lib is None:
        return None
    node = ctypes.c_int(-1)
    if lib.tpi_device_numa_node(device_index, ctypes.byref(node)) != 0:
        return None
    return pin_to_numa(node.value)


def _pid_alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        return True
    stat = _read("/proc/%d/stat" % pid)
    if stat:
        state = stat.rsplit(")", 1)[-1].split()
        if state and state[0] in ("Z", "X"):
            return False
    return True


pid_alive = _pid_alive
