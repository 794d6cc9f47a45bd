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
from typing import Dict, Iterator, List, Optional, Tuple

from ..utils.record import field, record

KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"


def _kfd(sub: str) -> str:
    """A path under KFD's sysfs tree (``TPI_SYSFS_KFD`` replaces ``/sys/class/kfd/kfd``: tests
    fake the topology and the per-process accounting)."""
    root = os.environ.get("TPI_SYSFS_KFD")
    return os.path.join(root, sub) if root else os.path.join("/sys/class/kfd/kfd", sub)
DRAIN_MAX_AGE = 600.0     # s: an older drain marker is ignored
DRAIN_STEP = 64 << 20     # a fall of at least this much counts as memory coming back


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
    if override is not None:  # "0,1,..." or "0=<pci bus id>,..." (tests: a fake sysfs)
        out = []
        for item in (x.strip() for x in override.split(",")):
            if item:
                index, _, pci = item.partition("=")
                out.append(GPU(index=int(index), gfx="gfx950", pci=pci))
        return out
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
    """The request can never be placed on this node (more GPUs than it has, ...)."""


class PlacementBusy(PlacementError):
    """The node could run the request, but not now: the task waits in the queue."""


def node_cpus(environ=None) -> List[int]:
    """Cores tasks may be given: ``TPI_NODE_CPUS`` (``0-15,32-47``) or this process's
    affinity mask (a container's cpuset, not the host's core count)."""
    environ = os.environ if environ is None else environ
    spec = environ.get("TPI_NODE_CPUS")
    if spec:
        return _cpulist(spec)
    if hasattr(os, "sched_getaffinity"):
        return sorted(os.sched_getaffinity(0))
    return list(range(os.cpu_count() or 1))


def node_memory_mb(environ=None) -> int:
    """Host memory tasks may reserve: ``TPI_NODE_MEMORY_MB``, else ``TPI_MEMORY_FRACTION``
    (default 0.9) of MemTotal."""
    environ = os.environ if environ is None else environ
    if environ.get("TPI_NODE_MEMORY_MB"):
        return int(float(environ["TPI_NODE_MEMORY_MB"]))
    total_kb = 0
    for line in _read("/proc/meminfo").splitlines():
        if line.startswith("MemTotal:"):
            total_kb = int(line.split()[1])
    fraction = float(environ.get("TPI_MEMORY_FRACTION", "0.9"))
    return int(total_kb / 1024 * fraction)


@record
class Request:
    """What a task asks the node for: ``parallelism`` ranks, each with ``gpus_per_rank`` GPUs,
    ``cpus_per_rank`` cores and ``memory_mb_per_rank`` of host memory (the machine type is
    per machine, and a rank is a machine: ``resource_job.go:107-140`` gives each of the Job's
    ``parallelism`` pods the machine's limits).  ``spot``: reclaimable capacity."""
    task: str
    parallelism: int = 1
    gpus_per_rank: int = 0
    cpus_per_rank: int = 0
    memory_mb_per_rank: int = 0
    spot: bool = False
    task_dir: str = ""
    gpu_filter: Optional[List[int]] = None  # region "gpus=" / "numa=" selectors
    numa: Optional[int] = None


@record
class Allocation:
    task: str
    gpus: List[int] = field(default_factory=list)
    rank_cpus: List[List[int]] = field(default_factory=list)
    memory_mb: int = 0                      # whole task
    memory_mb_per_rank: int = 0
    spot: bool = False
    notes: List[str] = field(default_factory=list)  # clamped requests etc.

    def to_json(self) -> dict:
        return {"task": self.task, "gpus": list(self.gpus),
                "rank_cpus": [list(c) for c in self.rank_cpus], "memory_mb": self.memory_mb,
                "memory_mb_per_rank": self.memory_mb_per_rank, "spot": self.spot,
                "notes": list(self.notes)}


class Placement:
    """Lease-file allocator over the node's GPUs."""

    LEASE_GRACE = 120.0  # a lease without a live supervisor yet is kept this long

    def __init__(self, state_root: str, gpus: Optional[List[GPU]] = None):
        self.root = os.path.join(state_root, "placement")
        os.makedirs(self.root, exist_ok=True)
        self.gpus = discover() if gpus is None else gpus

    def lease_path(self, index: int) -> str:
        return os.path.join(self.root, "gpu-%d.lease" % index)

    def drain_path(self, index: int) -> str:
        """The released lease of the GPU's previous holder (renamed by its supervisor or by
        :meth:`release`), until the next holder has seen the driver take its memory back."""
        return os.path.join(self.root, "gpu-%d.drain" % index)

    def _drain_marker(self, index: int) -> Optional[dict]:
        raw = _read(self.drain_path(index))
        if not raw:
            return None
        try:
            marker = json.loads(raw)
        except ValueError:
            return None
        try:  # a marker nobody consumed for this long says nothing about the GPU now
            if time.time() - os.path.getmtime(self.drain_path(index)) > DRAIN_MAX_AGE:
                return None
        except OSError:
            return None
        return marker

    def settle_gpus(self, indices: List[int], timeout: Optional[float] = None,
                    poll: float = 0.02) -> List[dict]:
        """Before a task's ranks start on GPUs ``indices``: wait until the amdgpu driver has
        taken the previous holders' device memory back, bounded by ``timeout``
        (``TPI_GPU_DRAIN_TIMEOUT``, default 30 s).  Returns one record per GPU that had
        something to wait for (for the task's journal: ``gpu-drain``).  Reference: the
        reference's replacement machine is a fresh VM (``task/aws/resources/
        resource_auto_scaling_group.go:51-106``) that inherits nothing of its predecessor;
        here a GPU changes hands on one node, so its start waits for what the last holder left.

        Why: a process's HBM is not free when it exits, nor when it frees it -- the driver
        wipes freed VRAM and releases it seconds later (200 GB: ~5 s; a 100 GB buffer as one
        step at the end of its wipe), while the HIP runtime of the next process already
        reports it free.  A task that fills the device on top of it over-commits VRAM, and the
        driver then evicts buffers -- including ones another process maps over HIP IPC --
        under running kernels; the round-5/6 hand-off faults came on exactly such runs
        (``profiles/round5/ipc_cause.md``, ``profiles/round6/``).

        A GPU is settled when both hold:
        * orphaned memory -- the driver's ``mem_info_vram_used`` minus what live processes
          hold by KFD's per-process accounting -- is at most ``ORPHAN_LIMIT`` (or this GPU's
          learned idle floor + 2 GiB), or has stopped falling for ``ORPHAN_FLAT_S`` -- longer
          for a big count, :func:`flat_window` -- (then it is no drain: a level up to
          ``ORPHAN_FLOOR_MAX`` is remembered as the GPU's floor);
        * with a drain marker (the previous holder's released lease): the driver's count is
          back to that holder's reservation count (``vram_baseline``) + ``max(1 GiB, 1 %)``.
        Without KFD's accounting, a count that keeps falling is waited for until it has not
        fallen for :func:`flat_window`.  The GPU's lease then records the settled count as its
        own baseline.  GPUs without a readable counter (no sysfs, fake inventories) are not
        waited for."""
        if timeout is None:
            try:
                timeout = float(os.environ.get("TPI_GPU_DRAIN_TIMEOUT", "30"))
            except ValueError:
                timeout = 30.0
        by_index = {g.index: g for g in self.gpus}
        todo = []
        for index in indices:
            gpu = by_index.get(index)
            if gpu is None or not gpu.pci:
                continue
            gid = kfd_gpu_id(gpu.pci)
            state = orphaned_vram(gpu.pci, gid)
            if state is None:
                continue
            marker = self._drain_marker(index)
            total = state["total"]
            baseline = None if marker is None else marker.get("vram_baseline")
            floor = self._orphan_floor(index)
            item = {"gpu": index, "pci": gpu.pci, "gid": gid, "start": state, "now": state,
                    "previous": (marker or {}).get("task"),
                    "target": None if baseline is None else
                    int(baseline) + max(1 << 30, total // 100),
                    "limit": max(ORPHAN_LIMIT, (floor or 0) + (2 << 30)),
                    "low": state["orphaned"] if state["orphaned"] is not None else state["used"],
                    "last_drop": None, "done": False, "flat": False}
            todo.append(item)
        t0 = time.monotonic()
        while todo:
            now = time.monotonic()
            pending = 0
            for item in todo:
                if item["done"]:
                    continue
                st = item["now"]
                level = st["orphaned"] if st["orphaned"] is not None else None
                quiet = now - (item["last_drop"] if item["last_drop"] is not None else t0)
                flat = quiet >= flat_window(st["orphaned"] if st["orphaned"] is not None
                                            else st["used"])
                if level is not None:
                    drained = level <= item["limit"] or flat
                else:  # no per-process accounting: a falling count is a drain
                    drained = flat or (item["target"] is None and
                                       st["used"] <= max(ORPHAN_LIMIT, st["total"] // 33))
                back = item["target"] is None or st["used"] <= item["target"]
                if drained and (back or flat):
                    item["done"], item["waited"] = True, now - t0
                    item["flat"] = flat and not (level is not None and level <= item["limit"])
                pending += not item["done"]
            if not pending or now - t0 >= timeout:
                break
            time.sleep(poll)
            for item in todo:
                if item["done"]:
                    continue
                st = orphaned_vram(item["pci"], item["gid"])
                if st is None:
                    item["done"], item["waited"] = True, time.monotonic() - t0
                    continue
                prev, item["now"] = item["now"], st
                level = st["orphaned"] if st["orphaned"] is not None else st["used"]
                if level < item["low"] - DRAIN_STEP:
                    item["low"] = level
                    item["last_drop"] = time.monotonic()
                # memory still moving -- exiting processes' memory turning orphaned (the
                # orphaned count rises), or the driver's count falling -- is no idle level
                moved = abs(st["used"] - prev["used"]) > DRAIN_STEP or (
                    st["orphaned"] is not None and prev["orphaned"] is not None
                    and st["orphaned"] > prev["orphaned"] + DRAIN_STEP)
                if moved:
                    item["last_drop"] = time.monotonic()
                    item["low"] = min(item["low"], level)
        waited = time.monotonic() - t0
        out = []
        for item in todo:
            start, now = item["start"], item["now"]
            orphan0 = start["orphaned"]
            busy = (orphan0 is not None and orphan0 > item["limit"]) or (
                orphan0 is None and start["used"] > max(ORPHAN_LIMIT, start["total"] // 33))
            if item["previous"] is not None or item["target"] is not None or busy:
                out.append({"gpu": item["gpu"], "previous": item["previous"],
                            "waited_s": round(item.get("waited", waited), 3),
                            "used_gb_at_start": round(start["used"] / 1e9, 2),
                            "used_gb": round(now["used"] / 1e9, 2),
                            "orphaned_gb_at_start": None if orphan0 is None else
                            round(orphan0 / 1e9, 2),
                            "orphaned_gb": None if now["orphaned"] is None else
                            round(now["orphaned"] / 1e9, 2),
                            "target_gb": None if item["target"] is None else
                            round(item["target"] / 1e9, 2),
                            "floor": item["flat"],
                            "timed_out": not item["done"]})
            if item["flat"] and now["orphaned"] is not None and now["orphaned"] <= ORPHAN_FLOOR_MAX:
                # a level above ORPHAN_FLOOR_MAX is no driver's own memory (a stuck or leaked
                # buffer): not learned, so the next start looks again
                self._set_orphan_floor(item["gpu"], now["orphaned"])
            try:
                os.unlink(self.drain_path(item["gpu"]))
            except FileNotFoundError:
                pass
            self._rebase_lease(item["gpu"], now["used"])
        return out

    def _orphan_floor(self, index: int) -> Optional[int]:
        """Orphaned VRAM this GPU was seen to carry without draining (its idle level)."""
        raw = _read(os.path.join(self.root, "gpu-%d.floor" % index)).strip()
        return int(raw) if raw.isdigit() else None

    def _set_orphan_floor(self, index: int, value: int) -> None:
        path = os.path.join(self.root, "gpu-%d.floor" % index)
        tmp = path + ".tmp"
        with open(tmp, "w") as handle:
            handle.write(str(int(value)))
        os.replace(tmp, path)

    def _rebase_lease(self, index: int, used: int) -> None:
        """The settled driver count becomes the lease's baseline (nothing of its holder runs
        on the GPU yet)."""
        with self._locked():
            lease = self._read_lease(index)
            if not lease or lease.get("task") == "?":
                return
            lease["vram_baseline"] = int(used)
            tmp = self.lease_path(index) + ".tmp"
            with open(tmp, "w") as handle:
                json.dump(lease, handle)
            os.replace(tmp, self.lease_path(index))

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
            for gpu in chosen:
                self._write_lease(gpu, {"task": task_id, "task_dir": task_dir})
            return sorted(held + chosen, key=lambda g: g.index)

    def _write_lease(self, gpu: GPU, lease: dict) -> None:
        """A GPU's lease, with the driver's VRAM count of a GPU nobody holds
        (``vram_baseline``): what the driver must be back to before the next holder starts
        (:meth:`settle_gpus`).  A drain marker still pending carries the baseline over (the
        previous holder's memory is not back yet, so the count now would include it)."""
        lease = dict(lease, created=time.time(), creator_pid=os.getpid(), gpu=gpu.index)
        marker = self._drain_marker(gpu.index)
        if marker is not None and marker.get("vram_baseline") is not None:
            lease["vram_baseline"] = marker["vram_baseline"]
        else:
            usage = vram_usage(gpu.pci) if gpu.pci else None
            if usage is not None:
                lease["vram_baseline"] = usage[0]
        tmp = self.lease_path(gpu.index) + ".tmp"
        with open(tmp, "w") as handle:
            json.dump(lease, handle)
        os.replace(tmp, self.lease_path(gpu.index))

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
                try:  # the lease becomes the GPU's drain marker (see settle_gpus)
                    os.replace(self.lease_path(gpu.index), self.drain_path(gpu.index))
                    n += 1
                except FileNotFoundError:
                    pass
            for path in (self.alloc_path(task_id), self.queue_path(task_id)):
                try:
                    os.unlink(path)
                except FileNotFoundError:
                    pass
            return n

    # -- whole-machine reservations: GPUs + cores + host memory, a queue, spot preemption ----
    #
    # The reference's scaling group keeps ``desired = parallelism`` until the cloud has the
    # capacity (resource_auto_scaling_group.go:51-106,188-199), and its consumers show the
    # task as ``queued`` meanwhile (cmd/leo/read/read.go:164-176).  On one node the capacity
    # is this node's GPUs, cores and DRAM: a task that does not fit waits in a queue (on-demand
    # before spot, then first come first served), and an on-demand task may reclaim the
    # resources of ``spot >= 0`` tasks, which are checkpointed and re-queued.

    def alloc_path(self, task_id: str) -> str:
        return os.path.join(self.root, "tasks", task_id + ".json")

    def queue_path(self, task_id: str) -> str:
        return os.path.join(self.root, "queue", task_id + ".json")

    def _load_dir(self, sub: str) -> Dict[str, dict]:
        out: Dict[str, dict] = {}
        base = os.path.join(self.root, sub)
        try:
            names = os.listdir(base)
        except OSError:
            return out
        for name in names:
            if not name.endswith(".json"):
                continue
            try:
                out[name[:-5]] = json.loads(_read(os.path.join(base, name)) or "null") or {}
            except ValueError:
                continue
        return out

    def allocations(self) -> Dict[str, dict]:
        """Live reservations by task id (stale ones -- task gone, supervisor dead past the
        grace period -- are dropped)."""
        out = {}
        for task, alloc in self._load_dir("tasks").items():
            if self._alive(alloc):
                out[task] = alloc
            else:
                try:
                    os.unlink(self.alloc_path(task))
                except FileNotFoundError:
                    pass
        return out

    def queue(self) -> List[dict]:
        """Live queue entries, in service order: on-demand before spot, then FIFO."""
        live = []
        for task, entry in self._load_dir("queue").items():
            pid = int(entry.get("waiter_pid", 0) or 0)
            fresh = time.time() - float(entry.get("enqueued", 0)) < self.LEASE_GRACE
            if (pid and _pid_alive(pid)) or (not pid and fresh):
                live.append(entry)
            else:
                try:
                    os.unlink(self.queue_path(task))
                except FileNotFoundError:
                    pass
        return sorted(live, key=lambda e: (int(e.get("priority", 1)), e.get("enqueued", 0)))

    def enqueue(self, req: "Request", waiter_pid: int = 0, reason: str = "") -> dict:
        with self._locked():
            old = _read(self.queue_path(req.task))
            entry = json.loads(old) if old else {}
            entry.update({"task": req.task, "task_dir": req.task_dir, "request": _req_json(req),
                          "priority": 1 if req.spot else 0, "reason": reason})
            entry.setdefault("enqueued", time.time())
            if waiter_pid:
                entry["waiter_pid"] = waiter_pid
            os.makedirs(os.path.dirname(self.queue_path(req.task)), exist_ok=True)
            tmp = self.queue_path(req.task) + ".tmp"
            with open(tmp, "w") as handle:
                json.dump(entry, handle)
            os.replace(tmp, self.queue_path(req.task))
            return entry

    def dequeue(self, task_id: str) -> None:
        with self._locked():
            try:
                os.unlink(self.queue_path(task_id))
            except FileNotFoundError:
                pass

    def position(self, task_id: str) -> int:
        """0-based place of ``task_id`` in the queue, -1 if not queued."""
        for i, entry in enumerate(self.queue()):
            if entry.get("task") == task_id:
                return i
        return -1

    def reserve(self, req: "Request") -> "Allocation":
        """Reserve GPUs, cores and memory for every rank of ``req`` atomically.

        Idempotent (an existing reservation is returned).  Raises :class:`PlacementError` when
        the node can never hold the request and :class:`PlacementBusy` when it cannot right
        now -- including when a task queued ahead of it is waiting for the same node."""
        with self._locked():
            existing = self._load_dir("tasks").get(req.task)
            if existing and existing.get("gpus") is not None:
                return _alloc_from(existing)
            pool = self._pool(req)
            need = req.gpus_per_rank * req.parallelism
            if need > len(pool):
                raise PlacementError("task needs %d GPUs; %d match on this node"
                                     % (need, len(pool)))
            ahead = self._ahead(req)
            if ahead:
                raise PlacementBusy("queued behind %s" % ", ".join(ahead[:3]))
            allocs = self.allocations()
            free = [g for g in self._free_locked() if g in pool]
            if len(free) < need:
                raise PlacementBusy("not enough free GPUs: need %d, free %d (held by %s)" % (
                    need, len(free), ", ".join(sorted(allocs)) or "-"))
            chosen = sorted(self._choose(free, need, True), key=lambda g: g.index)
            alloc = Allocation(task=req.task, gpus=[g.index for g in chosen], spot=req.spot)
            self._reserve_cpus(req, chosen, allocs, alloc)
            self._reserve_memory(req, allocs, alloc)
            now = time.time()
            for gpu in chosen:
                self._write_lease(gpu, {"task": req.task, "task_dir": req.task_dir,
                                        "spot": req.spot})
            record = dict(alloc.to_json(), task_dir=req.task_dir, created=now,
                          creator_pid=os.getpid())
            os.makedirs(os.path.dirname(self.alloc_path(req.task)), exist_ok=True)
            tmp = self.alloc_path(req.task) + ".tmp"
            with open(tmp, "w") as handle:
                json.dump(record, handle)
            os.replace(tmp, self.alloc_path(req.task))
            try:
                os.unlink(self.queue_path(req.task))
            except FileNotFoundError:
                pass
            return alloc

    def _pool(self, req: "Request") -> List[GPU]:
        pool = list(self.gpus)
        if req.gpu_filter is not None:
            pool = [g for g in pool if g.index in req.gpu_filter]
        if req.numa is not None:
            pool = [g for g in pool if g.numa_node == req.numa]
        return pool

    def _ahead(self, req: "Request") -> List[str]:
        """Queued tasks that must be served before ``req``."""
        mine = None
        entries = self.queue()
        for entry in entries:
            if entry.get("task") == req.task:
                mine = (int(entry.get("priority", 1)), entry.get("enqueued", 0))
        if mine is None:  # not queued yet: behind everyone of its priority or better
            mine = (1 if req.spot else 0, float("inf"))
        return [e["task"] for e in entries if e.get("task") != req.task and
                (int(e.get("priority", 1)), e.get("enqueued", 0)) < mine]

    def _reserve_cpus(self, req: "Request", gpus: List[GPU], allocs: Dict[str, dict],
                      alloc: "Allocation") -> None:
        if req.cpus_per_rank <= 0:
            alloc.rank_cpus = [[] for _ in range(req.parallelism)]
            return
        cores = node_cpus()
        per = min(req.cpus_per_rank, max(1, len(cores) // req.parallelism))
        if per < req.cpus_per_rank:
            alloc.notes.append("cpus clamped to %d per rank (node has %d cores)"
                               % (per, len(cores)))
        used = {c for a in allocs.values() for cs in a.get("rank_cpus") or [] for c in cs}
        free = [c for c in cores if c not in used]
        if len(free) < per * req.parallelism:
            raise PlacementBusy("not enough free cores: need %d x %d, free %d"
                                % (req.parallelism, per, len(free)))
        taken: set = set()
        out = []
        for r in range(req.parallelism):
            mine = gpus[r * req.gpus_per_rank:(r + 1) * req.gpus_per_rank]
            local = {c for g in mine for c in g.cpus}
            # the cores of the socket the rank's GPUs hang off first, then any
            order = [c for c in free if c in local and c not in taken] + \
                    [c for c in free if c not in local and c not in taken]
            pick = sorted(order[:per])
            taken.update(pick)
            out.append(pick)
        alloc.rank_cpus = out

    def _reserve_memory(self, req: "Request", allocs: Dict[str, dict],
                        alloc: "Allocation") -> None:
        if req.memory_mb_per_rank <= 0:
            return
        budget = node_memory_mb()
        per = min(req.memory_mb_per_rank, max(1, budget // req.parallelism))
        if per < req.memory_mb_per_rank:
            alloc.notes.append("memory clamped to %d MB per rank (node budget %d MB)"
                               % (per, budget))
        used = sum(int(a.get("memory_mb", 0) or 0) for a in allocs.values())
        if used + per * req.parallelism > budget:
            raise PlacementBusy("not enough host memory: need %d MB, free %d of %d MB"
                                % (per * req.parallelism, budget - used, budget))
        alloc.memory_mb_per_rank = per
        alloc.memory_mb = per * req.parallelism

    def victims(self, req: "Request") -> List[dict]:
        """Spot reservations an on-demand ``req`` would reclaim to fit now: the fewest tasks
        (largest first) whose GPUs, cores and memory, added to what is free, cover it."""
        if req.spot:
            return []
        with self._locked():
            allocs = self.allocations()
            pool = self._pool(req)
            free_gpus = {g.index for g in self._free_locked() if g in pool}
            need_gpus = req.gpus_per_rank * req.parallelism
            cores = node_cpus()
            used_cores = {c for a in allocs.values() for cs in a.get("rank_cpus") or []
                          for c in cs}
            per_cpu = min(req.cpus_per_rank, max(1, len(cores) // req.parallelism)) \
                if req.cpus_per_rank > 0 else 0
            free_cores = len(set(cores) - used_cores)
            budget = node_memory_mb()
            per_mem = min(req.memory_mb_per_rank, max(1, budget // req.parallelism)) \
                if req.memory_mb_per_rank > 0 else 0
            free_mem = budget - sum(int(a.get("memory_mb", 0) or 0) for a in allocs.values())
            spot = [a for a in allocs.values() if a.get("spot") and not a.get("requeueing")]
            spot.sort(key=lambda a: (-len(a.get("gpus") or []), -int(a.get("memory_mb", 0))))
            chosen: List[dict] = []

            def fits() -> bool:
                return (len(free_gpus) >= need_gpus and free_cores >= per_cpu * req.parallelism
                        and free_mem >= per_mem * req.parallelism)

            for a in spot:
                if fits():
                    break
                chosen.append(a)
                free_gpus.update(g for g in a.get("gpus") or [] if any(p.index == g for p in pool))
                free_cores += sum(len(cs) for cs in a.get("rank_cpus") or [])
                free_mem += int(a.get("memory_mb", 0) or 0)
            return chosen if chosen and fits() else []

    def mark_requeueing(self, task_id: str) -> None:
        """A reclaimed spot task keeps its reservation until its ranks are down."""
        with self._locked():
            raw = _read(self.alloc_path(task_id))
            if not raw:
                return
            alloc = json.loads(raw)
            alloc["requeueing"] = time.time()
            tmp = self.alloc_path(task_id) + ".tmp"
            with open(tmp, "w") as handle:
                json.dump(alloc, handle)
            os.replace(tmp, self.alloc_path(task_id))


def _req_json(req: "Request") -> dict:
    return {"task": req.task, "parallelism": req.parallelism,
            "gpus_per_rank": req.gpus_per_rank, "cpus_per_rank": req.cpus_per_rank,
            "memory_mb_per_rank": req.memory_mb_per_rank, "spot": req.spot,
            "task_dir": req.task_dir, "gpu_filter": req.gpu_filter, "numa": req.numa}


def _alloc_from(data: dict) -> "Allocation":
    return Allocation(task=data.get("task", ""), gpus=list(data.get("gpus") or []),
                      rank_cpus=[list(c) for c in data.get("rank_cpus") or []],
                      memory_mb=int(data.get("memory_mb", 0) or 0),
                      memory_mb_per_rank=int(data.get("memory_mb_per_rank", 0) or 0),
                      spot=bool(data.get("spot")), notes=list(data.get("notes") or []))


def region_placement_report(entries: List[dict], tolerance: float = 0.10):
    """Host-region NUMA placement of a job's ranks against their GPUs' sockets.

    ``entries``: one per rank, ``{"rank", "gpu_numa", "bytes_per_node": {"N0": bytes, ...},
    "wire_bytes_per_step"}`` (``gpu_numa`` -1: unknown, not checked).  Every rank's spill and
    restore cross the host memory its region lives in; a region on the other socket puts that
    traffic on the inter-socket link as well (at 8 ranks, ~0.74 TB/s of host-DRAM traffic over
    two sockets).  Returns ``(report, problems)``: the report adds the host-DRAM bytes each
    NUMA node moves per step (save into + restore out of the regions on it), ``problems``
    names every rank with more than ``tolerance`` of its region off its GPU's node."""
    traffic: Dict[str, float] = {}
    problems: List[str] = []
    for e in entries:
        per_node = {k: int(v) for k, v in (e.get("bytes_per_node") or {}).items()}
        total = sum(per_node.values())
        wire = float(e.get("wire_bytes_per_step") or 0)
        for node, nbytes in per_node.items():
            if total:
                traffic[node] = traffic.get(node, 0.0) + wire * nbytes / total
        gpu = e.get("gpu_numa")
        if gpu is None or int(gpu) < 0 or not total:
            continue
        remote = total - per_node.get("N%d" % int(gpu), 0)
        if remote > tolerance * total:
            problems.append("rank %s: %.1f of its %.1f GB host region on %s, but its GPU is on "
                            "NUMA node %d" % (e.get("rank"), remote / 1e9, total / 1e9,
                                              ",".join(sorted(n for n in per_node
                                                              if n != "N%d" % int(gpu))),
                                              int(gpu)))
    report = {"ranks": entries,
              "host_dram_bytes_per_step": {k: int(v) for k, v in sorted(traffic.items())}}
    return report, problems


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


def vram_usage(pci: str) -> Optional[Tuple[int, int]]:
    """``(used, total)`` bytes of a GPU's device memory from the amdgpu driver's sysfs
    counters (no GPU context needed: readable while other processes still hold the device),
    None when unreadable.  ``pci``: the GPU's bus id (:attr:`GPU.pci`)."""
    base = os.path.join(os.environ.get("TPI_SYSFS_PCI", "/sys/bus/pci/devices"), pci)
    used, total = _read(base + "/mem_info_vram_used").strip(), \
        _read(base + "/mem_info_vram_total").strip()
    if not (used.isdigit() and total.isdigit()):
        return None
    return int(used), int(total)


ORPHAN_LIMIT = 4 << 30  # orphaned VRAM (held by no live process) a GPU may carry when idle
ORPHAN_FLAT_S = 3.0     # an orphan count that has not fallen for this long is no drain ...
WIPE_RATE_MIN = 20e9    # ... unless it is big: the driver wipes freed VRAM at ~35 GB/s and
#                         gives a buffer back in one step at the end of its wipe, so a 150 GB
#                         buffer shows no fall for ~4.3 s (profiles/round6/r6f: a 3 s window
#                         took it for an idle level)


def flat_window(level: int) -> float:
    """Seconds without a fall after which ``level`` bytes of orphaned VRAM are taken for no
    drain: ``ORPHAN_FLAT_S``, or as long as the driver's wipe of that much memory can take."""
    return max(ORPHAN_FLAT_S, level / WIPE_RATE_MIN)
ORPHAN_FLOOR_MAX = 16 << 30  # the most a learned idle level may be


def kfd_gpu_id(pci: str) -> Optional[int]:
    """KFD's ``gpu_id`` of the GPU at PCI bus id ``pci`` (``0000:d9:00.0``): the topology node
    whose ``domain``/``location_id`` match it.  None when the topology is unreadable."""
    try:
        dom, bus, devfn = pci.split(":")
        dev, fn = devfn.split(".")
        loc = (int(bus, 16) << 8) | (int(dev, 16) << 3) | int(fn, 16)
        domain = int(dom, 16)
        nodes = os.listdir(_kfd("topology/nodes"))
    except (ValueError, OSError):
        return None
    for node in nodes:
        props = {}
        for line in _read(os.path.join(_kfd("topology/nodes"), node, "properties")).splitlines():
            key, _, value = line.partition(" ")
            props[key] = value.strip()
        if props.get("location_id") == str(loc) and props.get("domain", "0") == str(domain):
            gid = _read(os.path.join(_kfd("topology/nodes"), node, "gpu_id")).strip()
            return int(gid) if gid.isdigit() and int(gid) else None
    return None


def live_vram(gpu_id: Optional[int]) -> Optional[int]:
    """Bytes of a GPU's memory that live processes hold, by KFD's per-process accounting
    (``/sys/class/kfd/kfd/proc/<pid>/vram_<gpu_id>``; a process's count drops when it frees,
    before the driver has wiped and released the memory).  None when unreadable."""
    if gpu_id is None:
        return None
    try:
        pids = os.listdir(_kfd("proc"))
    except OSError:
        return None
    total, seen = 0, False
    for pid in pids:
        raw = _read(os.path.join(_kfd("proc"), pid, "vram_%d" % gpu_id)).strip()
        if raw.isdigit():
            total += int(raw)
            seen = True
    return total if seen or not pids else None


def orphaned_vram(pci: str, gpu_id: Optional[int] = None) -> Optional[Dict[str, int]]:
    """``{"used", "total", "live", "orphaned"}`` of a GPU: device memory the driver counts as
    used that no live process holds -- memory of exited processes and frees the driver is still
    wiping (plus the driver's own few GB).  ``live``/``orphaned`` are None without KFD's
    per-process accounting."""
    usage = vram_usage(pci) if pci else None
    if usage is None:
        return None
    live = live_vram(gpu_id if gpu_id is not None else kfd_gpu_id(pci))
    return {"used": usage[0], "total": usage[1], "live": live,
            "orphaned": None if live is None else max(0, usage[0] - live)}


def device_vram_usage(device_index: int) -> Optional[Tuple[int, int]]:
    """:func:`vram_usage` of HIP device ``device_index`` (found through its PCI bus id)."""
    import ctypes

    from ..ops import hip

    lib = hip(required=False)
    if lib is None:
        return None
    bus = ctypes.create_string_buffer(64)
    if lib.tpi_device_pci_bus_id(device_index, bus, 64) != 0:
        return None
    return vram_usage(bus.value.decode().lower())


def wait_vram_drained(pci: str, fraction: float = 0.03, timeout: float = 120.0) -> Dict:
    """Block until at most ``fraction`` of a GPU's memory is in use (processes of an earlier
    task may still be tearing down, their HBM not yet back), or ``timeout``; returns what was
    seen: ``{"used_gb_at_start", "waited_s", "used_gb"}`` (empty when sysfs is unreadable).
    Back-to-back measurements start from an empty device this way."""
    import time

    first = vram_usage(pci) if pci else None
    if first is None:
        return {}
    t0 = time.monotonic()
    now = first
    while now is not None and now[0] > fraction * now[1] and time.monotonic() - t0 < timeout:
        time.sleep(0.1)
        now = vram_usage(pci)
    return {"used_gb_at_start": round(first[0] / 1e9, 2),
            "waited_s": round(time.monotonic() - t0, 2),
            "used_gb": round((now or first)[0] / 1e9, 2)}


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
