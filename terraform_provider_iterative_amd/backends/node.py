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
import socket
import subprocess
import time
from typing import Dict, List, Optional

from .. import _build
from ..models.cloud import PROVIDER_LOCAL, PROVIDER_MI355X, Cloud, parse_region_selectors
from ..models.machine_types import MachineType, parse_node_machine
from ..models.values import (STATUS_RUNNING, Event, NotFoundError, NotImplementedErr,
                             RemoteStorage, Task as TaskSpec, new_status)
from ..parallel.placement import Placement, PlacementError, numa_cpus, pid_alive
from ..storage import transfer as storage
from ..utils.identifier import Identifier, parse_identifier
from ..utils.steps import Step, StepTiming, run_steps
from .base import Task

log = logging.getLogger("tpi")

# Host environment a rank inherits besides the task's own variables (the systemd unit of
# the reference starts from a clean environment + EnvironmentFile, tpl:45-59).
PASSTHROUGH_EXACT = ("PATH", "HOME", "USER", "LOGNAME", "LANG", "TZ", "TMPDIR",
                     "LD_LIBRARY_PATH", "PYTHONPATH", "OMP_NUM_THREADS", "MAX_JOBS")
PASSTHROUGH_PREFIXES = ("LC_", "HSA_", "HIP_", "ROCR_", "ROCM_", "NCCL_", "RCCL_", "GPU_",
                        "AMD_", "MIOPEN_", "TORCH_", "PYTORCH_")

DEFAULT_MASTER_PORT_BASE = 29500


def _now() -> float:
    return time.time()


def _write_json(path: str, data) -> None:
    tmp = path + ".tmp"
    with open(tmp, "w") as handle:
        json.dump(data, handle, indent=1, sort_keys=True)
    os.replace(tmp, path)


def _read_json(path: str):
    try:
        with open(path) as handle:
            return json.load(handle)
    except (OSError, ValueError):
        return None


def node_address() -> str:
    try:
        with socket.socket(socket.AF_INET, socket.SOCK_DGRAM) as s:
            s.connect(("10.255.255.255", 1))
            return s.getsockname()[0]
    except OSError:
        return "127.0.0.1"


def _free_port(start: int) -> int:
    for port in range(start, start + 2000):
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
            try:
                s.bind(("127.0.0.1", port))
                return port
            except OSError:
                continue
    return start


class NodeTask(Task):
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
        if remote is not None:
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
        ``ping``, ``state``, ``preempt``, ``stop``); the reply as a dict, or None when no
        supervisor is listening.  The path is reached through ``/proc/self/fd`` because
        AF_UNIX paths are limited to 108 bytes (the supervisor binds the same way)."""
        try:
            dfd = os.open(self.sup_dir, os.O_RDONLY | os.O_DIRECTORY)
        except OSError:
            return None
        try:
            with socket.socket(socket.AF_UNIX, socket.SOCK_STREAM) as sock:
                sock.settimeout(timeout)
                sock.connect("/proc/self/fd/%d/control.sock" % dfd)
                sock.sendall(command.encode() + b"\n")
                chunks = []
                while True:
                    data = sock.recv(65536)
                    if not data:
                        break
                    chunks.append(data)
        except OSError:
            return None
        finally:
            os.close(dfd)
        try:
            return json.loads(b"".join(chunks).decode() or "null")
        except ValueError:
            return None

    def supervisor_running(self) -> bool:
        state = self._state()
        pid = int(state.get("pid", 0) or 0)
        return bool(pid) and state.get("phase") != "stopped" and pid_alive(pid)

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

    def _create_storage(self) -> None:
        for d in (self.root, self.reports_dir, self.sup_dir):
            os.makedirs(d, exist_ok=True)
        os.makedirs(self.data_dir, exist_ok=True)
        if self._saved is None:
            self._saved = self._definition()
            _write_json(self.task_file, self._saved)
            self._event("created", "task %s" % self.id)

    def _place(self) -> None:
        definition = self._definition()
        gpus_per = self._machine().gpus
        total = gpus_per * definition["parallelism"]
        if self.provider != PROVIDER_MI355X or total == 0:
            definition["gpus"] = []
        else:
            selectors = parse_region_selectors(self.cloud.region)
            placement = self.placement
            if "gpus" in selectors:  # explicit pinning, e.g. region = "gpus=2-3"
                wanted = _index_list(selectors["gpus"])
                placement.gpus = [g for g in placement.gpus if g.index in wanted]
            if "numa" in selectors:
                placement.gpus = [g for g in placement.gpus
                                  if str(g.numa_node) == selectors["numa"]]
            try:
                gpus = placement.allocate(self.id, total, task_dir=self.root)
            except PlacementError as error:
                raise PlacementError("%s: %s" % (self.id, error)) from None
            definition["gpus"] = [g.index for g in gpus]
            definition["gpu_info"] = [g.to_json() for g in gpus]
            self._event("placed", "gpus " + ",".join(str(g.index) for g in gpus))
        _write_json(self.task_file, definition)

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
            "RCLONE_REMOTE": str(storage.Connection("local", self.root)),
        })
        visible = ",".join(str(g) for g in gpus)
        numa = [g.get("numa_node", -1) for g in d.get("gpu_info") or []]
        ranks = []
        for r in range(parallelism):
            mine = list(range(r * per, (r + 1) * per)) if per else []
            # affinity: the cores of the socket the rank's first GPU hangs off
            node = numa[mine[0]] if mine and mine[0] < len(numa) else -1
            cpus = numa_cpus(node) if os.environ.get("TPI_NUMA_PIN", "1") != "0" else []
            ranks.append({"gpus": visible, "rank_gpus": ",".join(str(i) for i in mine),
                          "cpus": cpus})
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
            "master_port": _free_port(DEFAULT_MASTER_PORT_BASE + (hash(self.id) % 1000) * 7),
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
            "leases": [self.placement.lease_path(g) for g in gpus],
        }

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
        steps = [Step("Validating machine...", self._validate),
                 Step("Creating storage...", self._create_storage),
                 Step("Placing task...", self._place),
                 Step("Writing machine script...", self._write_script)]
        if self.spec.environment.directory:
            steps.append(Step("Uploading Directory...", self.push))
        steps.append(Step("Starting task...", self.start))
        run_steps(steps, self.timings)
        log.info("Creation completed")

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
        pids = [int(state.get("pid", 0) or 0), int(state.get("stager_pid", 0) or 0)]
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

    def _delete_storage(self) -> None:
        # With a pre-allocated container the data lives outside self.root and is kept
        # (the reference only empties buckets it created, task/aws/task.go:245-299).
        if os.path.isdir(self.root):
            storage.native().remove_tree(self.root)

    def start(self) -> None:
        if self.supervisor_running():
            return
        spec = self._spec_json()
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
        if not pid or not pid_alive(pid) or state.get("phase") == "stopped":
            return
        if not (self.control("stop") or {}).get("ok"):
            try:
                os.kill(pid, signal.SIGTERM)
            except ProcessLookupError:
                return
        deadline = _now() + wait
        while _now() < deadline and pid_alive(pid):
            time.sleep(0.02)

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

    def push(self) -> None:
        directory = self.spec.environment.directory
        if not directory:
            return
        storage.transfer(directory, self.data_dir, self.spec.environment.exclude_list)

    def pull(self) -> None:
        saved = self._saved or {}
        directory = self.spec.environment.directory or saved.get("directory") or "."
        out = self.spec.environment.directory_out or saved.get("directory_out") or ""
        excludes = self.spec.environment.exclude_list or saved.get("exclude") or []
        rules = storage.limit_transfer(out, storage.transfer_rules(excludes))
        storage.transfer(self.data_dir, directory, rules=rules)

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


def _index_list(spec: str) -> List[int]:
    out: List[int] = []
    for part in spec.replace("|", ":").replace(";", ":").split(":"):
        if not part:
            continue
        lo, _, hi = part.partition("-")
        out.extend(range(int(lo), int(hi or lo) + 1))
    return out


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
