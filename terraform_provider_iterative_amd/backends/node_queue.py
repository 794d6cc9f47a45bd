"""Placement and the node queue of a node task (a :class:`~.node.NodeTask` mixin): reserving
the machine(s) on this node, queueing when they are busy, reclaiming spot capacity for an
on-demand task, the detached waiter that starts a queued task, and the drain of a GPU handed
over from its previous holder before the task's ranks start on it.

Reference: the scaling group keeps ``desired = parallelism`` until the cloud has capacity
(``task/aws/resources/resource_auto_scaling_group.go:51-106,188-199``) and its consumers show
the task as queued meanwhile (``cmd/leo/read/read.go:164-176``).
"""
from __future__ import annotations

import logging
import os
import signal
import subprocess
import sys
import time
from typing import Dict, List, Optional

from ..models.cloud import PROVIDER_MI355X, parse_region_selectors
from ..parallel.placement import (Allocation, Placement, PlacementBusy, PlacementError,
                                  Request)
from .nodeio import _now, _write_json, control_socket

log = logging.getLogger("tpi")
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class Queued(Exception):
    """Placement could not reserve the machine now: the task waits in the node queue."""


class NodeQueue:
    """The placement half of :class:`~.node.NodeTask`."""

    def _request(self) -> Optional[Request]:
        d = self._definition()
        machine = self._machine()
        gpus = machine.gpus if self.provider == PROVIDER_MI355X else 0
        reserve = self.resource_mode() == "reserve"
        if not gpus and not reserve:
            return None
        selectors = parse_region_selectors(self.cloud.region)
        return Request(task=self.id, parallelism=d["parallelism"], gpus_per_rank=gpus,
                       cpus_per_rank=machine.cpus if reserve else 0,
                       memory_mb_per_rank=machine.memory_mb if reserve else 0,
                       spot=self.spot(), task_dir=self.root,
                       gpu_filter=_index_list(selectors["gpus"]) if "gpus" in selectors else None,
                       numa=int(selectors["numa"]) if "numa" in selectors else None)

    def _place(self) -> None:
        """Reserve the task's machine(s) on this node; raises :class:`Queued` when they are
        busy (``TPI_PLACEMENT_QUEUE=0``: fail instead, the pre-queue behaviour)."""
        definition = self._definition()
        req = self._request()
        if req is None:
            definition["gpus"] = []
            _write_json(self.task_file, definition)
            return
        placement = self.placement
        try:
            alloc = placement.reserve(req)
        except PlacementBusy as busy:
            if self._knob("TPI_PLACEMENT_QUEUE", "1") == "0":
                raise PlacementError("%s: %s" % (self.id, busy)) from None
            placement.enqueue(req, reason=str(busy))
            self._event("queued", str(busy), "spot" if req.spot else "on-demand",
                        "position %d" % placement.position(self.id))
            self._reclaim(placement, req)
            raise Queued(str(busy)) from None
        except PlacementError as error:
            raise PlacementError("%s: %s" % (self.id, error)) from None
        self._apply(definition, alloc, placement)

    def _apply(self, definition: Dict, alloc: Allocation, placement: Placement) -> None:
        by_index = {g.index: g for g in placement.gpus}
        definition["gpus"] = list(alloc.gpus)
        definition["gpu_info"] = [by_index[g].to_json() for g in alloc.gpus if g in by_index]
        definition["allocation"] = alloc.to_json()
        _write_json(self.task_file, definition)
        desc = ["gpus " + (",".join(str(g) for g in alloc.gpus) or "-")]
        if any(alloc.rank_cpus):
            desc.append("cpus " + " | ".join(_ranges(c) for c in alloc.rank_cpus))
        if alloc.memory_mb:
            desc.append("memory %d MB" % alloc.memory_mb)
        if alloc.spot:
            desc.append("spot")
        self._event("placed", *(desc + alloc.notes))

    def _reclaim(self, placement: Placement, req: Request) -> List[str]:
        """On-demand task that does not fit: requeue the spot tasks whose resources make it
        fit (they checkpoint, release and wait for capacity again)."""
        if req.spot or placement.position(self.id) != 0:
            return []
        out = []
        for victim in placement.victims(req):
            task_dir = victim.get("task_dir") or ""
            reply = control_socket(os.path.join(task_dir, "supervisor"),
                                   "requeue reclaimed by %s" % self.id)
            if reply and reply.get("ok"):
                placement.mark_requeueing(victim["task"])
                self._event("reclaim", "spot task %s" % victim["task"],
                            "gpus " + ",".join(str(g) for g in victim.get("gpus") or []))
                out.append(victim["task"])
        return out

    # -- the node queue -----------------------------------------------------------------------
    def _waiter_argv(self) -> List[str]:
        code = ("import sys; sys.path.insert(0, %r); "
                "from terraform_provider_iterative_amd.parallel.scheduler import main; "
                "sys.exit(main([%r]))" % (ROOT, self.root))
        return [sys.executable, "-c", code]

    def _spawn_waiter(self) -> int:
        """Start the detached process that waits for this task's turn, then starts it."""
        logfile = open(os.path.join(self.sup_dir, "queue.log"), "ab")
        try:
            proc = subprocess.Popen(self._waiter_argv(), stdin=subprocess.DEVNULL,
                                    stdout=logfile, stderr=logfile, close_fds=True,
                                    cwd=self.root, start_new_session=True)
        finally:
            logfile.close()
        self._write_queue_state(proc.pid)
        return proc.pid

    def _write_queue_state(self, pid: int, phase: str = "queued") -> None:
        state = self._state()
        _write_json(os.path.join(self.sup_dir, "state.json"), {
            "pid": pid, "task_id": self.id, "phase": phase, "running": 0, "ranks": [],
            "restarts": int(state.get("restarts", 0) or 0), "heartbeat": _now()})

    def run_queued(self, poll: float = 0.1) -> int:
        """The waiter (:mod:`..parallel.scheduler`): hold this task's place in the queue until
        its machine can be reserved, reclaiming spot capacity when it is the on-demand head,
        then start the supervisor.  SIGTERM (``leo stop`` / ``delete``) leaves the queue."""
        stopping: List[bool] = []
        signal.signal(signal.SIGTERM, lambda *_: stopping.append(True))
        if os.path.exists(self._stop_marker()):
            stopping.append(True)
        else:
            self._write_queue_state(os.getpid())
        placement = self.placement
        req = self._request()
        requeued = self._was_running()
        if req is None:  # nothing to wait for
            self.start(restart_base=self._restarts() + requeued, force=True)
            return 0
        placement.enqueue(req, waiter_pid=os.getpid(),
                          reason="requeued" if requeued else "busy")
        if requeued:  # a reclaimed spot task: back in the queue, resumes when placed again
            self._event("queued", "requeued", "spot" if req.spot else "on-demand",
                        "position %d" % placement.position(self.id))
        t0 = _now()
        while not stopping:
            if os.path.exists(self._stop_marker()):
                break
            try:
                alloc = placement.reserve(req)
            except PlacementBusy:
                if not req.spot:
                    self._reclaim(placement, req)
                time.sleep(poll)
                continue
            except PlacementError as error:
                placement.dequeue(self.id)
                self._event("placement-failed", str(error))
                self._write_queue_state(0, "stopped")
                return 1
            self._event("dequeued", "waited %.3f s" % (_now() - t0))
            self._apply(self._definition(), alloc, placement)
            self.start(restart_base=self._restarts() + requeued, force=True)
            return 0
        placement.dequeue(self.id)
        self._event("stop-requested", "queued task left the queue")
        self._write_queue_state(0, "stopped")
        return 0

    def _restarts(self) -> int:
        return int(self._state().get("restarts", 0) or 0)

    def _was_running(self) -> bool:
        return any(e.code == "rank-start" for e in self.events())

    def _settle_gpus(self, spec: Dict) -> None:
        """A GPU handed over from another holder is used only once the driver has its memory
        back (:meth:`Placement.settle_gpus`); each wait is journalled (``gpu-drain``)."""
        gpus = [int(g) for g in str(spec["env"].get("TPI_VISIBLE_GPUS", "")).split(",") if g]
        if not gpus:
            return
        for rec in self.placement.settle_gpus(gpus):
            desc = ["gpu %d" % rec["gpu"], "waited %.3f s" % rec["waited_s"],
                    "VRAM in use %.1f -> %.1f GB" % (rec["used_gb_at_start"], rec["used_gb"])]
            if rec["orphaned_gb_at_start"] is not None:
                desc.append("held by no process %.1f -> %.1f GB" % (
                    rec["orphaned_gb_at_start"], rec["orphaned_gb"]))
            if rec["floor"]:
                desc.append("stopped falling: taken as the GPU's idle level")
            if rec["previous"]:
                desc.append("previous holder %s" % rec["previous"])
            if rec["target_gb"] is not None:
                desc.append("target %.1f GB" % rec["target_gb"])
            if rec["timed_out"]:
                desc.append("timed out (TPI_GPU_DRAIN_TIMEOUT): starting anyway")
            self._event("gpu-drain", *desc)


def _ranges(cpus: List[int]) -> str:
    """``[0,1,2,5]`` -> ``"0-2,5"``."""
    out, start, prev = [], None, None
    for c in sorted(cpus):
        if start is None:
            start = prev = c
        elif c == prev + 1:
            prev = c
        else:
            out.append(str(start) if start == prev else "%d-%d" % (start, prev))
            start = prev = c
    if start is not None:
        out.append(str(start) if start == prev else "%d-%d" % (start, prev))
    return ",".join(out) or "-"


def _index_list(spec: str) -> List[int]:
    out: List[int] = []
    for part in spec.replace("|", ":").replace(";", ":").split(":"):
        if not part:
            continue
        lo, _, hi = part.partition("-")
        out.extend(range(int(lo), int(hi or lo) + 1))
    return out
