"""Node-local task backends: ``local`` (CPU) and ``mi355x`` (1-8 GPUs of this node).

One task = one directory ``<state_root>/<provider>/<task id>/``:

* ``data/``        the task's storage and working directory (the reference's bucket
                   ``data/`` prefix; with ``storage.container`` the container directory)
* ``reports/``     ``task-<machine uuid>`` logs and ``status-<uuid>`` reports
* ``supervisor/``  ``spec.json``, ``script``, ``state.json``, ``events.jsonl``, log
* ``task.json``    the task definition (what the cloud backends keep in cloud resources)

Create mirrors the reference's step lists (``task/aws/task.go:135-196``,
``task/k8s/task.go:129-176``): validate, create storage, place, push the workdir, start.
Start launches the native supervisor (``csrc/supervisor/supervisor.cpp``), which plays the
scaling group + machine script; Stop sends it SIGTERM (scale to zero).
"""
from __future__ import annotations

import json
import logging
import os
import signal
import subprocess
import sys
import time
from typing import Dict, List, Optional

from .. import _build
from ..models.cloud import PROVIDER_LOCAL, PROVIDER_MI355X, Cloud
from ..models.machine_types import MachineType, parse_node_machine
from ..models.values import (STATUS_RUNNING, Event, NotFoundError, NotImplementedErr,
                             RemoteStorage, Task as TaskSpec, new_status)
from ..parallel.placement import Placement, node_cpus, pid_alive
from ..storage import remote as remote_storage
from ..storage import transfer as storage
from ..utils.identifier import Identifier, parse_identifier
from ..utils.steps import Step, StepTiming, run_steps
from .base import Task
from .node_queue import NodeQueue, Queued  # noqa: F401
from .node_storage import NodeStorage
from .nodeio import _now, _read_json, _write_json, control_socket  # noqa: F401

log = logging.getLogger("tpi")

# Host environment a rank inherits besides the task's own variables (the systemd unit of
# the reference starts from a clean environment + EnvironmentFile, tpl:45-59).
PASSTHROUGH_EXACT = ("PATH", "HOME", "USER", "LOGNAME", "LANG", "TZ", "TMPDIR",
                     "LD_LIBRARY_PATH", "PYTHONPATH", "OMP_NUM_THREADS", "MAX_JOBS",
                     "TPI_SSH_COMMAND")  # the transport to an off-node storage.container
PASSTHROUGH_PREFIXES = ("LC_", "HSA_", "HIP_", "ROCR_", "ROCM_", "NCCL_", "RCCL_", "GPU_",
                        "AMD_", "MIOPEN_", "TORCH_", "PYTORCH_")

DEFAULT_MASTER_PORT_BASE = 29500
HBM_MB_PER_GPU = 288 * 1024  # MI355X: 288 GiB of HBM3E per GPU
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def node_address() -> str:
    import socket

    try:
        with socket.socket(socket.AF_INET, socket.SOCK_DGRAM) as s:
            s.connect(("10.255.255.255", 1))
            return s.getsockname()[0]
    except OSError:
        return "127.0.0.1"


def shebang_python(script: str):
    """``(interpreter, flags)`` when ``script``'s ``#!`` line runs this Python interpreter's
    binary (``#!/path/python [-u ...]`` or ``#!/usr/bin/env python3 [...]``; a virtualenv's
    link to it included, and kept as the interpreter to launch), else None."""
    import shutil

    first = (script or "").split("\n", 1)[0]
    if not first.startswith("#!"):
        return None
    words = first[2:].split()
    if not words:
        return None
    if os.path.basename(words[0]) == "env" and len(words) > 1:
        words = words[1:]
        if words[0].startswith("-"):  # env -S / -i ...: not followed here
            return None
        found = shutil.which(words[0])
        if not found:
            return None
        words[0] = found
    if not os.path.basename(words[0]).startswith("python"):
        return None
    try:
        same = os.path.realpath(words[0]) == os.path.realpath(sys.executable)
    except OSError:
        return None
    flags = words[1:]
    if not same or any(not f.startswith("-") or f in ("-c", "-m") for f in flags):
        return None
    # launched as the script names it: a virtualenv's interpreter is a link to the same binary
    # but brings its own site-packages (pyvenv.cfg next to the link)
    return words[0], flags


_SHELLS = ("sh", "bash", "dash", "zsh")
_SHELL_META = set("$`|&;<>*?(){}[]!~\\\"'")


def shell_python_command(script: str):
    """``(interpreter, flags, [file.py, args...])`` when ``script`` is a shell script whose
    one command runs a Python file with this interpreter (``python3 train.py --lr 1e-4``,
    optionally ``exec``, after ``set -e``-style lines): the common form of the reference's task
    scripts, which a preloaded successor can run without the shell.  Anything else -- more
    commands, variables, redirections, globs, quoting -- is None."""
    import shlex

    lines = (script or "").splitlines()
    if not lines or not lines[0].startswith("#!"):
        return None
    words = lines[0][2:].split()
    if not words:
        return None
    shell = os.path.basename(words[-1] if os.path.basename(words[0]) == "env" else words[0])
    if shell not in _SHELLS:
        return None
    commands = [l.strip() for l in lines[1:]
                if l.strip() and not l.strip().startswith("#")
                and not l.strip().startswith("set ")]
    if len(commands) != 1 or any(c in _SHELL_META for c in commands[0]):
        return None
    argv = shlex.split(commands[0])
    if argv and argv[0] == "exec":
        argv = argv[1:]
    if len(argv) < 2 or not argv[1].endswith(".py"):
        return None
    found = shebang_python("#!%s\n" % argv[0]) if os.path.isabs(argv[0]) else \
        shebang_python("#!/usr/bin/env %s\n" % argv[0])
    if found is None:
        return None
    return found[0], found[1], argv[1:]

class NodeTask(NodeQueue, NodeStorage, Task):
    """Task on this node; ``provider`` selects CPU-only or GPU placement."""

    def __init__(self, cloud: Cloud, identifier: Identifier, task: TaskSpec):
        self.cloud = cloud
        self.provider = cloud.provider
        self.identifier = identifier
        self.id = identifier.long()
        self.spec = task
        self.root = os.path.join(cloud.state_root(), self.provider, self.id)
        self.reports_dir = os.path.join(self.root, "reports")
        self.sup_dir = os.path.join(self.root, "supervisor")
        self.task_file = os.path.join(self.root, "task.json")
        self.timings: List[StepTiming] = []
        self._saved = _read_json(self.task_file)
        remote = task.remote_storage
        if remote is None and self._saved and self._saved.get("remote_storage"):
            rs = self._saved["remote_storage"]
            remote = RemoteStorage(rs["container"], rs.get("path", ""), rs.get("config", {}))
        self.remote = remote
        # an off-node container (storage/remote.py): the node works on a local copy that is
        # restored from it at create and mirrored back while the task runs
        self.remote_conn = remote_storage.parse(remote.container, remote.path,
                                                remote.config) if remote is not None else None
        if remote is not None and self.remote_conn is None:
            conn = storage.Connection.parse(remote.container)
            base = conn.local_path()
            self.data_dir = os.path.join(base, remote.path.lstrip("/")) if remote.path else base
        else:
            self.data_dir = os.path.join(self.root, "data")
        self.machine: Optional[MachineType] = None

    # -- helpers -------------------------------------------------------------------------------
    @property
    def placement(self) -> Placement:
        return Placement(self.cloud.state_root())

    def _state(self) -> Dict:
        return _read_json(os.path.join(self.sup_dir, "state.json")) or {}

    def control(self, command: str, timeout: float = 2.0) -> Optional[Dict]:
        """One request on the supervisor's control socket (``supervisor/control.sock``:
        ``ping``, ``state``, ``preempt``, ``preempt <rank>``, ``requeue``, ``stop``)."""
        return control_socket(self.sup_dir, command, timeout)

    def supervisor_running(self) -> bool:
        """A supervisor, or the queue waiter of a queued task, is alive (the task is not
        over).  A supervisor that just handed its task back to the queue counts until the
        waiter has taken over state.json."""
        state = self._state()
        pid = int(state.get("pid", 0) or 0)
        if state.get("phase") == "requeued":
            return _now() - float(state.get("heartbeat", 0) or 0) < 30.0
        return bool(pid) and state.get("phase") != "stopped" and pid_alive(pid)

    @classmethod
    def from_root(cls, root: str) -> "NodeTask":
        """The task stored at ``<state_root>/<provider>/<id>`` (queue waiter, agents)."""
        from ..models.cloud import Credentials, NodeCredentials
        from ..models.values import Environment, Size

        saved = _read_json(os.path.join(root, "task.json")) or {}
        state_root = os.path.dirname(os.path.dirname(os.path.abspath(root)))
        cloud = Cloud(provider=saved.get("provider", PROVIDER_LOCAL),
                      region=saved.get("region", "") or "",
                      credentials=Credentials(node=NodeCredentials(state_root=state_root)))
        spec = TaskSpec(size=Size(machine=saved.get("machine") or "m"),
                        parallelism=saved.get("parallelism", 1),
                        environment=Environment(timeout=saved.get("timeout") or 0))
        return cls(cloud, parse_identifier(saved.get("id") or os.path.basename(root)), spec)

    def _machine(self) -> MachineType:
        if self.machine is None:
            name = self.spec.size.machine or (self._saved or {}).get("machine") or "m"
            self.machine = parse_node_machine(name)
            if self.provider == PROVIDER_LOCAL and self.machine.gpus:
                raise ValueError("cloud \"local\" runs on CPUs; use cloud = \"mi355x\" for "
                                 "machine %r" % name)
        return self.machine

    def _definition(self) -> Dict:
        if self._saved:
            return self._saved
        t = self.spec
        env = t.environment
        return {
            "id": self.id, "provider": self.provider, "region": self.cloud.region,
            "machine": t.size.machine, "disk_size": t.size.storage, "image": env.image,
            "parallelism": max(1, int(t.parallelism or 1)), "spot": t.spot,
            "permission_set": t.permission_set, "tags": dict(self.cloud.tags),
            "timeout": env.timeout,
            "deadline": (_now() + env.timeout) if env.timeout and env.timeout > 0 else 0,
            "directory": env.directory, "directory_out": env.directory_out,
            "exclude": list(env.exclude_list or []),
            "environment": env.variables.enrich(),
            "remote_storage": ({"container": self.remote.container, "path": self.remote.path,
                                "config": self.remote.config} if self.remote else None),
            "created_at": _now(),
        }

    def _event(self, code: str, *description: str) -> None:
        os.makedirs(self.sup_dir, exist_ok=True)
        with open(os.path.join(self.sup_dir, "events.jsonl"), "a") as handle:
            handle.write(json.dumps({"time": _now(), "code": code,
                                     "description": list(description)}) + "\n")

    # -- steps ---------------------------------------------------------------------------------
    def _validate(self) -> None:
        machine = self._machine()
        if self.spec.permission_set:
            log.warning("permission_set %r is recorded but ranks run as the current user on "
                        "the node-local runtime", self.spec.permission_set)
        if self.spec.environment.image not in ("", "ubuntu", "nvidia", "rocm", "host"):
            log.warning("image %r: node-local tasks run in the host environment",
                        self.spec.environment.image)
        if machine.gpus and self.provider != PROVIDER_MI355X:
            raise ValueError("GPU machine types need cloud = \"mi355x\"")


    def _knob(self, name: str, default: str) -> str:
        """Runtime knob: the task's own environment block, else the provider's."""
        value = (self._definition().get("environment") or {}).get(name)
        return str(value) if value not in (None, "") else os.environ.get(name, default)

    def resource_mode(self) -> str:
        """``reserve``: the machine type's cores and memory are reserved on the node next to
        the GPUs (disjoint core sets, memory admission; a task that does not fit is queued) --
        the default for ``mi355x``.  ``limit``: they are only limits (affinity capped to
        ``cpus`` cores, the memory limit enforced), like the k8s Job's limits without requests
        (``resource_job.go:107-118``) -- the default for ``local``.  ``TPI_RESOURCE_MODE``."""
        default = "reserve" if self.provider == PROVIDER_MI355X else "limit"
        mode = self._knob("TPI_RESOURCE_MODE", default)
        return mode if mode in ("reserve", "limit") else default

    def spot(self) -> bool:
        """``spot >= 0`` (``values.go:17-22``: 0 auto, > 0 max price): reclaimable."""
        try:
            return float(self._definition().get("spot", -1)) >= 0
        except (TypeError, ValueError):
            return False


    def _spec_json(self) -> Dict:
        d = self._definition()
        parallelism = d["parallelism"]
        gpus = d.get("gpus") or []
        per = len(gpus) // parallelism if gpus else 0
        env = {}
        for key, value in os.environ.items():
            if key in PASSTHROUGH_EXACT or key.startswith(PASSTHROUGH_PREFIXES):
                env[key] = value
        env.pop("HIP_VISIBLE_DEVICES", None)
        env.pop("CUDA_VISIBLE_DEVICES", None)
        env.pop("ROCR_VISIBLE_DEVICES", None)
        env.update(d.get("environment") or {})

        def knob(name: str, default: str) -> str:
            """Runtime knob: the task's own environment block, else the provider's."""
            value = (d.get("environment") or {}).get(name)
            return str(value) if value not in (None, "") else os.environ.get(name, default)

        env.update({
            "TPI_TASK_CLOUD_PROVIDER": self.provider,
            "TPI_TASK_CLOUD_REGION": str(d.get("region", "")),
            "RCLONE_REMOTE": str(self.remote_conn or storage.Connection("local", self.root)),
        })
        visible = ",".join(str(g) for g in gpus)
        numa = [g.get("numa_node", -1) for g in d.get("gpu_info") or []]
        alloc = d.get("allocation") or {}
        ranks = []
        for r in range(parallelism):
            mine = list(range(r * per, (r + 1) * per)) if per else []
            ranks.append({"gpus": visible, "rank_gpus": ",".join(str(i) for i in mine),
                          "cpus": self._rank_cpus(r, alloc)})
        if gpus:
            env["TPI_VISIBLE_GPUS"] = visible
        script_path = os.path.join(self.sup_dir, "script")
        stager = self._stager(d, per, visible, numa)
        return {
            "stager": stager,
            "task_id": self.id, "task_dir": self.root, "workdir": self.data_dir,
            "script": script_path, "env": env, "deadline": d.get("deadline", 0),
            "parallelism": parallelism, "ranks": ranks,
            "master_addr": "127.0.0.1",
            # a base: the supervisor takes the first free port from it (no probing here)
            "master_port": DEFAULT_MASTER_PORT_BASE + (hash(self.id) % 1000) * 7,
            "master_port_probe": True,
            "gang": True, "fail_fast": parallelism > 1, "respawn_on_sigterm": True,
            "max_restarts": int(knob("TPI_MAX_RESTARTS", "-1")),
            "grace_seconds": float(knob("TPI_GRACE_SECONDS", "30")),
            "respawn_delay": float(knob("TPI_RESPAWN_DELAY", "0")),
            # warm standby successors for ranks that call preemption.standby(): the successor's
            # imports overlap the spill; with progressive pinning and the lingering predecessor
            # 100 GB recover in 3.6 s signal-to-restored instead of 5.1 s
            # (profiles/preempt_e2e_100g_round2.md).  TPI_WARM_STANDBY=0 disables.
            "standby": knob("TPI_WARM_STANDBY", "1") != "0",
            # TPI_WARM_STANDBY=hot: the successor is started with the rank, not at the
            # preemption, so it can restore behind a streamed spill
            "standby_hot": knob("TPI_WARM_STANDBY", "1") == "hot",
            "reports_dir": self.reports_dir,
            "state_path": os.path.join(self.sup_dir, "state.json"),
            "events_path": os.path.join(self.sup_dir, "events.jsonl"),
            "leases": [self.placement.lease_path(g) for g in gpus] +
                      ([self.placement.alloc_path(self.id)] if alloc else []),
            "limits": self._limits(alloc),
            "requeue_argv": self._waiter_argv(),
            "sync": self._remote_sync(knob),
            # a preloaded successor per Python rank (runtime/preload.py; TPI_PRELOAD=0: none)
            "preload_argv": self._preload_argv(knob),
            # TPI_PRELOAD=1/auto (default): the parked successor creates its GPU context once
            # the running rank shows it uses the GPU from one process ("plain": never)
            "preload_gpu_auto": knob("TPI_PRELOAD", "1") in ("1", "true", "yes", "auto"),
            "preload_gpu_device": knob("TPI_PRELOAD_GPU_DEVICE", "/dev/kfd"),
        }

    def _preload_argv(self, knob) -> List[str]:
        """The launcher of a preloaded successor (``runtime/preload.py``; the supervisor appends
        the script path), or ``[]``.  On by default (``TPI_PRELOAD=0`` disables) for a script
        that this very interpreter would run (``#!`` naming it, directly or through ``env``;
        interpreter flags are kept), since the successor runs it in-process; off with a hot
        standby (``TPI_WARM_STANDBY=hot``), whose parked successor has the GPU initialised."""
        mode = knob("TPI_PRELOAD", "1")
        if mode not in ("1", "true", "yes", "auto", "plain", "gpu", "gpu-lite"):
            return []
        if knob("TPI_WARM_STANDBY", "1") == "hot":
            return []
        script = self.spec.environment.script
        interp = shebang_python(script)
        target = None  # None: the task script itself (the supervisor appends its path)
        if interp is None:
            found = shell_python_command(script)
            if found is None:
                return []
            interp, target = found[:2], found[2]
        path, flags = interp
        # TPI_PRELOAD=gpu: the parked process also initialises the GPU and prewarms an engine
        code = ("import sys; sys.path.insert(0, %r); "
                "from terraform_provider_iterative_amd.runtime.preload import main; "
                "main(%r, gpu=%r)" % (ROOT, target, {"gpu": True, "gpu-lite": "lite"}.get(mode, False)))
        return [path] + flags + ["-c", code]

    def _remote_sync(self, knob) -> Optional[Dict]:
        """The supervisor's mirror of an off-node container: every ``TPI_SYNC_INTERVAL`` s
        (default 10, as the reference's data loop, tpl:118-124) and once when the ranks are
        done, before the task counts as finished."""
        if self.remote_conn is None:
            return None
        try:
            interval = float(knob("TPI_SYNC_INTERVAL", "10"))
        except ValueError:
            interval = 10.0
        code = ("import sys; sys.path.insert(0, %r); "
                "from terraform_provider_iterative_amd.storage.remote import main; "
                "sys.exit(main(['sync', %r]))" % (ROOT, self.root))
        return {"argv": [sys.executable, "-c", code], "interval": interval if interval > 0 else 0,
                "timeout": float(knob("TPI_REMOTE_SYNC_TIMEOUT", "600"))}

    def _rank_cpus(self, rank: int, alloc: Dict) -> List[int]:
        """Affinity of rank ``rank``: its reserved cores (``reserve`` mode), else -- a limit
        only -- ``machine.cpus`` cores of this node, a different window per rank
        (``TPI_NUMA_PIN=0``: no affinity)."""
        if self._knob("TPI_NUMA_PIN", "1") == "0":
            return []
        rank_cpus = alloc.get("rank_cpus") or []
        if rank < len(rank_cpus) and rank_cpus[rank]:
            return list(rank_cpus[rank])
        cores = node_cpus()
        want = self._machine().cpus
        if not cores or want <= 0 or want >= len(cores):
            return []
        start = (rank * want + (sum(map(ord, self.id)) % len(cores))) % len(cores)
        return sorted(cores[(start + i) % len(cores)] for i in range(want))

    def _limits(self, alloc: Dict) -> Dict:
        """Machine-type limits the supervisor enforces (``resource_job.go:112-118``: k8s turns
        them into pod limits): host memory per rank and the task's ``disk_size``
        (``TPI_ENFORCE_LIMITS=0`` disables)."""
        if self._knob("TPI_ENFORCE_LIMITS", "1") == "0":
            return {}
        machine = self._machine()
        memory = int(alloc.get("memory_mb_per_rank") or 0) or machine.memory_mb
        out = {"rank_memory_mb": memory,
               # the kernel's hard cap (supervisor setup_cgroups): "auto", "off" or a cgroup
               # directory; checkpoint regions (shm, charged to the rank) get one GPU's HBM of
               # headroom per GPU -- a spill mirrors device state, it is not the working set
               "cgroup": self._knob("TPI_MEMORY_CGROUP", "auto")}
        headroom = self._knob("TPI_CGROUP_HEADROOM_MB", "")
        try:
            out["cgroup_headroom_mb"] = int(headroom) if headroom else \
                machine.gpus * HBM_MB_PER_GPU
        except ValueError:
            out["cgroup_headroom_mb"] = machine.gpus * HBM_MB_PER_GPU
        interval = self._knob("TPI_MEMORY_CHECK_INTERVAL", "")
        if interval:
            try:
                out["memory_interval"] = float(interval)
            except ValueError:
                pass
        try:
            disk = float(self._definition().get("disk_size", -1) or -1)
        except (TypeError, ValueError):
            disk = -1
        if disk > 0:
            out["disk_gb"] = disk
        limit_mb = self._knob("TPI_DISK_LIMIT_MB", "")  # finer than disk_size's GB
        if limit_mb:
            out["disk_gb"] = float(limit_mb) / 1000.0
        try:
            out["disk_interval"] = float(self._knob("TPI_DISK_CHECK_INTERVAL", "10"))
        except ValueError:
            pass
        return out

    def _stager(self, d: Dict, per: int, visible: str, numa: List[int]) -> Optional[Dict]:
        """The supervisor's ``stager`` entry when the workdir goes to HBM before the ranks
        start (:mod:`..runtime.stage`), else None."""
        from ..runtime import stage

        environ = dict(os.environ)
        environ.update({k: v for k, v in (d.get("environment") or {}).items() if v is not None})
        if not stage.mode(environ, self.provider, 1 << 62):
            return None  # disabled, or a backend that never stages: skip the walk
        files, nbytes = stage.layout(self.data_dir)
        kind = stage.mode(environ, self.provider, nbytes)
        parallelism = d["parallelism"]
        if kind == "hbm" and not per:
            return None
        if not kind or nbytes == 0:
            return None
        devices = [r * per for r in range(parallelism)] if kind == "hbm" else \
            list(range(parallelism))
        node = [numa[i] if i < len(numa) else -1 for i in devices] if kind == "hbm" else \
            [-1] * parallelism
        entry = stage.plan(self.data_dir, self.sup_dir, devices, node, environ,
                           host=kind == "host", files=files, nbytes=nbytes)
        entry["gpus"] = visible
        return entry

    def _write_script(self) -> None:
        script = self.spec.environment.script or (self._saved or {}).get("script", "")
        path = os.path.join(self.sup_dir, "script")
        if script:
            with open(path + ".tmp", "w") as handle:
                handle.write(script)
            os.chmod(path + ".tmp", 0o755)
            os.replace(path + ".tmp", path)
        elif not os.path.exists(path):
            raise ValueError("task has no script")

    # -- Task interface -------------------------------------------------------------------------
    def create(self) -> None:
        log.info("Creating resources...")
        queued: List[str] = []

        def place():
            try:
                self._place()
            except Queued as why:
                queued.append(str(why))

        def start():
            if queued:
                self._spawn_waiter()
            else:
                self.start()

        steps = [Step("Validating machine...", self._validate),
                 Step("Creating storage...", self._create_storage),
                 Step("Placing task...", place),
                 Step("Writing machine script...", self._write_script)]
        if self.spec.environment.directory:
            steps.append(Step("Uploading Directory...", self.push))
        if self.remote_conn is not None:  # tpl:89: the workdir comes from the container
            steps.append(Step("Restoring Directory from the container...", self._restore_remote))
        steps.append(Step("Starting task...", start))
        run_steps(steps, self.timings)
        log.info("Creation completed" + (" (queued: %s)" % queued[0] if queued else ""))


    def read(self) -> None:
        if not os.path.isdir(self.root):
            raise NotFoundError("task %s not found" % self.id)
        self._saved = _read_json(self.task_file) or self._saved

    def delete(self) -> None:
        log.info("Deleting resources...")
        steps: List[Step] = []
        out = self.spec.environment.directory_out or (self._saved or {}).get("directory_out")
        if out and os.path.isdir(self.root):
            steps.append(Step("Downloading Directory...", self.pull))
        steps += [Step("Stopping task...", self._stop_quiet),
                  Step("Releasing placement...", lambda: self.placement.release(self.id)),
                  Step("Deleting storage...", self._delete_storage)]
        run_steps(steps, self.timings)
        log.info("Deletion completed")

    def _stop_quiet(self) -> None:
        """Stop, and make sure nothing of the task still runs before its GPUs are handed to
        another task and its directory is removed: ranks that outlive ``stop`` (a grace period
        longer than the wait, a slow spill) are killed, process group by process group."""
        if not os.path.isdir(self.root):
            return
        self.stop()
        if self._alive_pids():
            self._kill_remaining()

    def _alive_pids(self) -> List[int]:
        state = self._state()
        # a settled supervisor ("stopped") holds nothing: it only reaps released processes
        # still tearing down (their kernel unmaps of a pinned region), behind the task's end
        sup = int(state.get("pid", 0) or 0) if state.get("phase") != "stopped" else 0
        pids = [sup, int(state.get("stager_pid", 0) or 0)]
        pids += [int(r.get("pid", 0) or 0) for r in state.get("ranks") or []]
        return [p for p in pids if p > 0 and pid_alive(p)]

    def _kill_remaining(self, wait: float = 10.0) -> None:
        state = self._state()
        sup = int(state.get("pid", 0) or 0)
        ranks = [int(r.get("pid", 0) or 0) for r in state.get("ranks") or []]
        ranks.append(int(state.get("stager_pid", 0) or 0))
        for pid in [p for p in ranks if p > 0] + ([sup] if sup > 0 else []):
            for target in (-pid, pid):  # each rank leads its own process group
                try:
                    os.kill(target, signal.SIGKILL)
                except (ProcessLookupError, PermissionError):
                    pass
        deadline = _now() + wait
        while _now() < deadline and self._alive_pids():
            time.sleep(0.02)
        left = self._alive_pids()
        if left:
            raise RuntimeError("task %s: processes %s survive SIGKILL; not releasing its GPUs"
                               % (self.id, left))
        self._event("killed", "processes left after stop were killed")


    def start(self, restart_base: int = 0, force: bool = False) -> None:
        if not force and self.supervisor_running():
            return
        spec = self._spec_json()
        spec["restart_base"] = restart_base
        self._settle_gpus(spec)
        spec_path = os.path.join(self.sup_dir, "spec.json")
        _write_json(spec_path, spec)
        # TPI_SUPERVISOR_BIN: an alternative build (e.g. the ASan/UBSan one of the tests)
        binary = os.environ.get("TPI_SUPERVISOR_BIN") or _build.SUPERVISOR
        if binary == _build.SUPERVISOR:
            _build.build_supervisor()  # content-stamped: compiles only if the sources changed
        logfile = open(os.path.join(self.sup_dir, "supervisor.log"), "ab")
        try:
            proc = subprocess.Popen([binary, "--daemon", spec_path], stdin=subprocess.DEVNULL,
                                    stdout=subprocess.PIPE, stderr=logfile, close_fds=True,
                                    cwd=self.root)
            out, _ = proc.communicate(timeout=30)
        finally:
            logfile.close()
        if proc.returncode != 0:
            raise RuntimeError("supervisor failed to start (see %s)" % os.path.join(
                self.sup_dir, "supervisor.log"))
        pid = int(out.decode().strip() or 0)
        self._event("started", "supervisor pid %d" % pid)


    def stop(self, wait: float = 60.0) -> None:
        state = self._state()
        pid = int(state.get("pid", 0) or 0)
        if state.get("phase") in ("queued", "requeued"):
            # the queue waiter (or the one a requeueing supervisor is about to start) sees
            # the marker and leaves the queue; a waiter that is gone is cleaned up here
            with open(self._stop_marker(), "w"):
                pass
            deadline = _now() + wait
            while _now() < deadline and self.supervisor_running():
                pid = int(self._state().get("pid", 0) or 0)
                if pid and self._state().get("phase") == "queued":
                    try:
                        os.kill(pid, signal.SIGTERM)
                    except ProcessLookupError:
                        pass
                time.sleep(0.02)
            self.placement.dequeue(self.id)
            if self._state().get("phase") in ("queued", "requeued"):
                self._write_queue_state(0, "stopped")
            return
        if not pid or not pid_alive(pid) or state.get("phase") == "stopped":
            return
        if not (self.control("stop") or {}).get("ok"):
            try:
                os.kill(pid, signal.SIGTERM)
            except ProcessLookupError:
                return
        deadline = _now() + wait
        # the task is over once the supervisor has settled (final sync and state written);
        # it may live on a while, reaping released processes that are still exiting
        while (_now() < deadline and pid_alive(pid)
               and self._state().get("phase") != "stopped"):
            time.sleep(0.02)

    def _stop_marker(self) -> str:
        return os.path.join(self.sup_dir, "stop-requested")

    def preempt(self, rank: Optional[int] = None) -> None:
        """Fault injection: preempt every rank, or only ``rank`` (its gang follows when the
        ranks are coupled); they checkpoint, then get respawned."""
        state = self._state()
        pid = int(state.get("pid", 0) or 0)
        if not pid or not pid_alive(pid):
            raise NotFoundError("task %s is not running" % self.id)
        if rank is None:
            if not (self.control("preempt") or {}).get("ok"):
                os.kill(pid, signal.SIGUSR1)
            return
        reply = self.control("preempt %d" % rank)
        if reply is None:
            raise NotFoundError("task %s has no control socket for per-rank preemption" % self.id)
        if not reply.get("ok"):
            raise NotFoundError("task %s: %s" % (self.id, reply.get("error")))


    def status(self) -> Dict[str, int]:
        initial = new_status()
        if self.supervisor_running():
            initial[STATUS_RUNNING] = int(self._state().get("running", 0))
        return storage.status(self.root, initial)

    def events(self) -> List[Event]:
        out = []
        path = os.path.join(self.sup_dir, "events.jsonl")
        try:
            with open(path) as handle:
                for line in handle:
                    line = line.strip()
                    if line:
                        try:
                            out.append(Event.from_json(json.loads(line)))
                        except (ValueError, KeyError):
                            continue
        except OSError:
            pass
        return out

    def _machine_order(self) -> List[str]:
        order = []
        for event in self.events():
            if event.code == "rank-start":
                for item in event.description:
                    if item.startswith("machine "):
                        order.append(item.split(" ", 1)[1])
        return order

    def logs(self) -> List[str]:
        try:
            names = sorted(n for n in os.listdir(self.reports_dir) if n.startswith("task-"))
        except OSError:
            return []
        rank = {uuid: i for i, uuid in enumerate(self._machine_order())}
        names.sort(key=lambda n: (rank.get(n[5:], len(rank)), n))
        out = []
        for name in names:
            try:
                with open(os.path.join(self.reports_dir, name), errors="replace") as handle:
                    out.append(handle.read())
            except OSError:
                continue
        return out

    def get_identifier(self) -> Identifier:
        return self.identifier

    def get_addresses(self) -> List[str]:
        running = self.status().get(STATUS_RUNNING, 0)
        return [node_address()] * running

    def get_key_pair(self):
        raise NotImplementedErr()

    # -- extras ----------------------------------------------------------------------------------
    def gpus(self) -> List[int]:
        return list((self._saved or {}).get("gpus") or [])

    def wait(self, timeout: float = 60.0, poll: float = 0.05) -> Dict[str, int]:
        """Block until the supervisor exits (all ranks finished) or ``timeout``."""
        deadline = _now() + timeout
        while _now() < deadline:
            if not self.supervisor_running():
                break
            time.sleep(poll)
        return self.status()


def list_tasks(cloud: Cloud) -> List[Identifier]:
    base = os.path.join(cloud.state_root(), cloud.provider)
    try:
        names = sorted(os.listdir(base))
    except OSError:
        return []
    out = []
    for name in names:
        try:
            out.append(parse_identifier(name))
        except ValueError:
            continue
    return out
