"""Tasks on a *remote* node: ``cloud = "mi355x"`` (or ``"local"``) with ``region = "host=..."``.

The reference's whole workflow is remote: ``terraform apply`` on a laptop or CI runner
provisions a machine, uploads the workdir, runs the script there and pulls the results back
(``task/aws/task.go:135-354``; ``machine/storage.go:123-159``).  The node-local runtime of this
framework runs tasks on the node it is installed on; this backend restores the remote
workflow for nodes that already exist (the k8s backend's precedent: no VMs, work lands on
existing nodes selected through ``region``, ``task/k8s/resources/resource_job.go:41-46``).

``region`` keys (comma-separated ``k=v``, like the k8s node selector):

=================  =======================================================================
``host``           ``[user@]hostname`` of the node (required for this backend)
``port``           SSH port
``root``           task state root on the node (default: the node's ``TPI_STATE_ROOT`` or
                   ``~/.local/state/tpi``)
``gpus``, ``numa`` placement constraints, applied on the node (see ``backends/node.py``)
=================  =======================================================================

Client environment: ``TPI_SSH_COMMAND`` (default ``ssh -o BatchMode=yes``), the node's
framework checkout ``TPI_REMOTE_FRAMEWORK`` (default: this checkout's path) and interpreter
``TPI_REMOTE_PYTHON`` (default ``python3``).  Each operation is one transport command
running ``backends/agent.py`` on the node.  The workdir travels as a tar stream through the
same channel, built from the same filter rules as a local push (default excludes, anchored
bare patterns, ``storage.go:123-159``), and comes back filtered like ``Pull`` with
``LimitTransfer(directory_out)`` (``storage.go:267-280``).
"""
from __future__ import annotations

import json
import logging
import os
import re
import shlex
import subprocess
import threading
from typing import Any, Dict, List, Optional

from ..models.cloud import Cloud, parse_region_selectors
from ..models.values import Event, NotFoundError, NotImplementedErr, Task as TaskSpec
from ..storage import transfer as storage
from ..utils.identifier import Identifier, parse_identifier
from ..utils.steps import Step, StepTiming, run_steps
from . import agent
from .base import Task

log = logging.getLogger("tpi")

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# region keys consumed by the transport; the rest go to the node's own placement
TRANSPORT_KEYS = ("host", "port", "root")


class RemoteNodeError(RuntimeError):
    pass


def is_remote(cloud: Cloud) -> bool:
    return "host" in parse_region_selectors(cloud.region)


def _node_region(region: str) -> str:
    keep = []
    for item in (region or "").split(","):
        key = item.partition("=")[0].strip()
        if item.strip() and key not in TRANSPORT_KEYS:
            keep.append(item.strip())
    return ",".join(keep)


_HOST = re.compile(r"^(?:[A-Za-z0-9._][A-Za-z0-9._-]*@)?(?:[A-Za-z0-9_][A-Za-z0-9._-]*|\[[0-9A-Fa-f:.]+\])$")


class Transport:
    """One command per operation through ``TPI_SSH_COMMAND <host> <remote command>``."""

    def __init__(self, cloud: Cloud):
        sel = parse_region_selectors(cloud.region)
        self.host = sel["host"]
        # the host goes into ssh's argv: "-oProxyCommand=..." would be parsed as an option
        if not _HOST.match(self.host or ""):
            raise ValueError("region host %r is not [user@]hostname" % self.host)
        self.port = sel.get("port")
        if self.port is not None and not str(self.port).isdigit():
            raise ValueError("region port %r is not a number" % self.port)
        self.state_root = sel.get("root", "")
        self.provider = cloud.provider
        self.region = _node_region(cloud.region)
        self.framework = os.environ.get("TPI_REMOTE_FRAMEWORK", ROOT)
        self.python = os.environ.get("TPI_REMOTE_PYTHON", "python3")
        self.ssh = shlex.split(os.environ.get("TPI_SSH_COMMAND", "ssh -o BatchMode=yes"))

    def _argv(self, op: str, request: Dict[str, Any]) -> List[str]:
        req = dict(request, provider=self.provider, region=self.region,
                   state_root=self.state_root)
        remote = "cd %s && exec %s -m terraform_provider_iterative_amd.backends.agent %s %s" % (
            shlex.quote(self.framework), shlex.quote(self.python), op,
            agent.encode_request(req))
        argv = list(self.ssh)
        if self.port:
            argv += ["-p", str(self.port)]
        return argv + [self.host, remote]

    def call(self, op: str, request: Dict[str, Any], stdin=None, timeout: float = 600.0) -> Any:
        proc = subprocess.run(self._argv(op, request), stdin=stdin, stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, timeout=timeout)
        answer = None
        for line in proc.stdout.decode(errors="replace").splitlines():
            if line.startswith(agent.MARKER):
                answer = json.loads(line[len(agent.MARKER):])
        if answer is None:
            raise RemoteNodeError("%s on %s: no answer (exit %d): %s" % (
                op, self.host, proc.returncode, proc.stderr.decode(errors="replace")[-2000:]))
        if "error" in answer:
            if answer.get("kind") == "NotFoundError":
                raise NotFoundError(answer["error"])
            raise RemoteNodeError("%s on %s: %s: %s" % (op, self.host, answer.get("kind"),
                                                        answer["error"]))
        return answer.get("result")

    def popen(self, op: str, request: Dict[str, Any], **kwargs) -> subprocess.Popen:
        return subprocess.Popen(self._argv(op, request), **kwargs)


class RemoteNodeTask(Task):
    """A task run by the node runtime of another host (see module docstring)."""

    def __init__(self, cloud: Cloud, identifier: Identifier, task: TaskSpec):
        self.cloud = cloud
        self.identifier = identifier
        self.id = identifier.long()
        self.spec = task
        self.transport = Transport(cloud)
        self.timings: List[StepTiming] = []
        self._view: Optional[Dict[str, Any]] = None

    def _request(self, **extra) -> Dict[str, Any]:
        spec = agent.spec_to_json(self.spec)
        # the workdir and the output directory are paths on *this* host: upload and download
        # are done from here (push/pull), the node never touches them
        spec["environment"]["directory"] = spec["environment"]["directory_out"] = ""
        return dict(extra, id=self.id, spec=spec)

    # -- Task interface -------------------------------------------------------------------------
    def create(self) -> None:
        log.info("Creating resources on %s...", self.transport.host)
        steps = [Step("Creating task on %s..." % self.transport.host,
                      lambda: self.transport.call("create", self._request()))]
        if self.spec.environment.directory:
            steps.append(Step("Uploading Directory...", self.push))
        steps.append(Step("Starting task...", self.start))
        run_steps(steps, self.timings)
        log.info("Creation completed")

    def read(self) -> None:
        view = self.transport.call("describe", self._request())
        if not view.get("exists"):
            raise NotFoundError("task %s not found on %s" % (self.id, self.transport.host))
        self._view = view

    def _described(self) -> Dict[str, Any]:
        if self._view is None:
            self.read()
        return self._view

    def delete(self) -> None:
        log.info("Deleting resources on %s...", self.transport.host)
        steps: List[Step] = []
        if self.spec.environment.directory_out:
            steps.append(Step("Downloading Directory...", self._pull_if_exists))
        steps.append(Step("Deleting task on %s..." % self.transport.host,
                          lambda: self.transport.call("delete", self._request())))
        run_steps(steps, self.timings)
        log.info("Deletion completed")

    def _pull_if_exists(self) -> None:
        try:
            self.read()
        except NotFoundError:
            return
        self.pull()

    def start(self) -> None:
        self.transport.call("start", self._request())

    def stop(self) -> None:
        self.transport.call("stop", self._request())

    def preempt(self, rank: Optional[int] = None) -> None:
        self.transport.call("preempt", self._request(rank=rank))

    def push(self) -> None:
        """Stream the filtered workdir (same rules as a local push) into the node's storage."""
        directory = self.spec.environment.directory
        if not directory:
            return
        flt = storage.make_filter(storage.transfer_rules(self.spec.environment.exclude_list))
        proc = self.transport.popen("push", self._request(), stdin=subprocess.PIPE,
                                    stdout=subprocess.PIPE, stderr=subprocess.PIPE)
        # drain the answer channels while the tar stream is written (no pipe-buffer deadlock)
        out, err = bytearray(), bytearray()
        readers = [threading.Thread(target=lambda f=f, b=b: b.extend(f.read()), daemon=True)
                   for f, b in ((proc.stdout, out), (proc.stderr, err))]
        for r in readers:
            r.start()
        stats = {"files": 0, "bytes": 0}
        try:
            stats = agent.write_tar(storage.Connection.parse(directory).local_path(), flt,
                                    proc.stdin)
        except BrokenPipeError:
            pass  # the node ended the transfer early: its answer says why
        finally:
            try:
                proc.stdin.close()
            except BrokenPipeError:
                pass
        proc.wait(timeout=3600)
        for r in readers:
            r.join()
        answer = None
        for line in out.decode(errors="replace").splitlines():
            if line.startswith(agent.MARKER):
                answer = json.loads(line[len(agent.MARKER):])
        if not answer or "error" in answer:
            raise RemoteNodeError("push to %s failed: %s" % (
                self.transport.host, (answer or {}).get("error") or err.decode()[-2000:]))
        log.info("Uploaded %d files (%s) to %s", stats["files"],
                 storage.human_size(stats["bytes"]), self.transport.host)

    def pull(self) -> None:
        """The node's task storage, limited to ``directory_out``, into the local workdir."""
        import tarfile  # remote-node pulls only

        env = self.spec.environment
        local = storage.Connection.parse(env.directory or ".").local_path()
        proc = self.transport.popen("pull", self._request(directory_out=env.directory_out,
                                                          exclude=list(env.exclude_list)),
                                    stdout=subprocess.PIPE, stderr=subprocess.PIPE)
        count = 0
        try:
            with tarfile.open(fileobj=proc.stdout, mode="r|") as tar:
                for member in agent._safe_members(tar):
                    if member.isdir():
                        continue
                    dest = os.path.join(local, member.name)
                    os.makedirs(os.path.dirname(dest), exist_ok=True)
                    src = tar.extractfile(member)
                    with open(dest + ".tpi-part", "wb") as out:
                        while True:
                            block = src.read(8 << 20)
                            if not block:
                                break
                            out.write(block)
                    os.chmod(dest + ".tpi-part", member.mode & 0o777)
                    os.replace(dest + ".tpi-part", dest)
                    count += 1
        finally:
            err = proc.stderr.read()
            proc.wait(timeout=600)
        if proc.returncode != 0:
            raise RemoteNodeError("pull from %s failed (exit %d): %s" % (
                self.transport.host, proc.returncode, err.decode(errors="replace")[-2000:]))
        log.info("Downloaded %d files from %s", count, self.transport.host)

    def status(self) -> Dict[str, int]:
        return dict(self._described()["status"])

    def events(self) -> List[Event]:
        return [Event.from_json(e) for e in self._described()["events"]]

    def logs(self) -> List[str]:
        return list(self._described()["logs"])

    def get_identifier(self) -> Identifier:
        return self.identifier

    def get_addresses(self) -> List[str]:
        return list(self._described()["addresses"])

    def get_key_pair(self):
        raise NotImplementedErr()

    def gpus(self) -> List[int]:
        return list(self._described().get("gpus") or [])


def list_tasks(cloud: Cloud) -> List[Identifier]:
    out = []
    for name in Transport(cloud).call("list", {})["ids"]:
        try:
            out.append(parse_identifier(name))
        except ValueError:
            continue
    return out
