"""Remote end of the ``host=`` node backend (``backends/ssh.py``).

The reference drives remote machines through cloud APIs and a bucket
(``task/aws/task.go:135-354``, ``machine/storage.go:123-159``).  Here a remote MI355X node runs
this framework too; the client reaches it with one command transport (``ssh host``) per
operation and this module performs the operation on that node's own runtime::

    python -m terraform_provider_iterative_amd.backends.agent <op> <base64 JSON request>

``op`` is ``create`` (validate, storage, placement, script; no upload, no start), ``start``,
``stop``, ``preempt``, ``describe`` (existence, status, events, logs, addresses, GPUs in one
round trip), ``delete``, ``list``, ``push`` (a tar stream on stdin is unpacked into the task's
storage), ``pull`` (the task's storage, filtered like ``Pull``, as a tar stream on stdout).
Every op except ``pull`` answers with one ``TPI-AGENT <json>`` line on stdout, also on
failure (``{"error": ..., "kind": ...}`` and exit status 1), so login banners or stray output
on the remote shell cannot be mistaken for the answer.
"""
from __future__ import annotations

import base64
import datetime as _dt
import json
import os
import sys
from typing import Any, Dict

MARKER = "TPI-AGENT "


def encode_request(data: Dict[str, Any]) -> str:
    return base64.urlsafe_b64encode(json.dumps(data, sort_keys=True).encode()).decode()


def decode_request(text: str) -> Dict[str, Any]:
    return json.loads(base64.urlsafe_b64decode(text.encode()).decode())


def spec_to_json(spec) -> Dict[str, Any]:
    """The parts of a task definition the remote node needs (variables already enriched on the
    client: empty values inherit from the *client's* environment, ``values.go:102-118``)."""
    env = spec.environment
    remote = spec.remote_storage
    return {
        "size": {"machine": spec.size.machine, "storage": spec.size.storage},
        "environment": {"image": env.image, "script": env.script,
                        "variables": dict(env.variables.enrich()), "timeout": env.timeout,
                        "directory": env.directory, "directory_out": env.directory_out,
                        "exclude_list": list(env.exclude_list)},
        "permission_set": spec.permission_set, "spot": spec.spot,
        "parallelism": spec.parallelism,
        "remote_storage": None if remote is None else {
            "container": remote.container, "path": remote.path, "config": dict(remote.config)},
    }


def spec_from_json(data: Dict[str, Any]):
    from ..models.values import Environment, RemoteStorage, Size, Task, Variables

    env = data.get("environment") or {}
    rs = data.get("remote_storage")
    return Task(
        size=Size(**(data.get("size") or {})),
        environment=Environment(image=env.get("image", "ubuntu"), script=env.get("script", ""),
                                variables=Variables(env.get("variables") or {}),
                                timeout=float(env.get("timeout") or 0),
                                directory=env.get("directory", ""),
                                directory_out=env.get("directory_out", ""),
                                exclude_list=list(env.get("exclude_list") or [])),
        permission_set=data.get("permission_set", ""), spot=float(data.get("spot", -1)),
        parallelism=int(data.get("parallelism", 1)),
        remote_storage=None if not rs else RemoteStorage(rs["container"], rs.get("path", ""),
                                                         rs.get("config") or {}))


def _cloud(req: Dict[str, Any]):
    from ..models.cloud import Cloud, Credentials, NodeCredentials

    root = req.get("state_root") or ""
    return Cloud(provider=req["provider"], region=req.get("region") or "",
                 credentials=Credentials(node=NodeCredentials(state_root=root)))


def _task(req: Dict[str, Any]):
    from ..utils.identifier import parse_identifier
    from .node import NodeTask

    return NodeTask(_cloud(req), parse_identifier(req["id"]), spec_from_json(req.get("spec") or {}))


def _describe(task) -> Dict[str, Any]:
    from ..models.values import NotFoundError

    try:
        task.read()
    except NotFoundError:
        return {"exists": False}
    return {"exists": True, "status": task.status(),
            "events": [e.to_json() for e in task.events()], "logs": task.logs(),
            "addresses": task.get_addresses(), "gpus": task.gpus()}


def _safe_members(tar: "tarfile.TarFile"):
    """Regular files and directories with relative, non-escaping names only."""
    for member in tar:
        name = os.path.normpath(member.name)
        if name.startswith(("/", "..")) or os.path.isabs(name) or not (member.isfile() or
                                                                     member.isdir()):
            raise ValueError("refusing tar member %r" % member.name)
        yield member


def _push(task) -> Dict[str, Any]:
    os.makedirs(task.data_dir, exist_ok=True)
    count = size = 0
    import tarfile

    with tarfile.open(fileobj=sys.stdin.buffer, mode="r|") as tar:
        for member in _safe_members(tar):
            if member.isdir():
                os.makedirs(os.path.join(task.data_dir, member.name), exist_ok=True)
                continue
            dest = os.path.join(task.data_dir, member.name)
            os.makedirs(os.path.dirname(dest), exist_ok=True)
            src = tar.extractfile(member)
            tmp = dest + ".tpi-part"
            with open(tmp, "wb") as out:
                while True:
                    block = src.read(8 << 20)
                    if not block:
                        break
                    out.write(block)
            os.chmod(tmp, member.mode & 0o777)
            os.utime(tmp, (member.mtime, member.mtime))
            os.replace(tmp, dest)
            count += 1
            size += member.size
    return {"files": count, "bytes": size}


def _pull(task, req: Dict[str, Any]) -> None:
    from ..storage import transfer as storage

    rules = storage.limit_transfer(req.get("directory_out") or "",
                                   storage.transfer_rules(req.get("exclude") or []))
    write_tar(task.data_dir, storage.make_filter(rules), sys.stdout.buffer)


def write_tar(root: str, flt, stream) -> Dict[str, int]:
    """Files under ``root`` accepted by ``flt`` (relative names) as a tar stream."""
    from ..ops import native

    count = size = 0
    import tarfile

    with tarfile.open(fileobj=stream, mode="w|") as tar:
        if os.path.isdir(root):
            for rel, nbytes, _mtime, _mode, is_dir in native().walk(root, flt):
                if is_dir:
                    continue
                tar.add(os.path.join(root, rel), arcname=rel, recursive=False)
                count += 1
                size += nbytes
    stream.flush()
    return {"files": count, "bytes": size}


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    op, req = argv[0], decode_request(argv[1]) if len(argv) > 1 else {}
    try:
        if op == "pull":
            _pull(_task(req), req)
            return 0
        if op == "list":
            from .node import list_tasks

            result: Any = {"ids": [i.long() for i in list_tasks(_cloud(req))]}
        else:
            task = _task(req)
            if op == "create":
                task._validate()
                task._create_storage()
                task._place()
                task._write_script()
                result = {"gpus": task.gpus() or (task._saved or {}).get("gpus") or []}
            elif op == "start":
                task.start()
                result = {}
            elif op == "stop":
                task.stop()
                result = {}
            elif op == "preempt":
                task.preempt(req.get("rank"))
                result = {}
            elif op == "push":
                result = _push(task)
            elif op == "describe":
                result = _describe(task)
            elif op == "delete":
                task.delete()
                result = {}
            else:
                raise ValueError("unknown agent op %r" % op)
    except Exception as error:  # reported to the client, which re-raises it
        print(MARKER + json.dumps({"error": str(error), "kind": type(error).__name__}),
              flush=True)
        return 1
    print(MARKER + json.dumps({"ok": True, "result": result,
                               "time": _dt.datetime.now(_dt.timezone.utc).timestamp()}),
          flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
