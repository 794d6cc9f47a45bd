"""Off-node ``storage.container``: a directory on another machine, reached over SSH.

The reference lets a task keep its data and results in a pre-allocated bucket or volume that
outlives the machine (``storage.container`` + ``container_opts``,
``iterative/resource_task.go:380-397``; the rclone connection of ``task/common/machine/
storage.go:236-263``; ``task/aws/resources/data_source_bucket.go:15-62``;
``task/k8s/resources/data_source_persistent_volume.go``).  On a node runtime the durable place
is another node, and the channel to it is the one the remote-node backend already uses: the
SSH command transport (``TPI_SSH_COMMAND``, default ``ssh -o BatchMode=yes``).  The storage
node needs nothing but ``sh``, ``tar``, ``cat`` and ``mv`` -- like an rclone sftp remote.

Forms of ``storage.container`` (``container_opts``: ``host``, ``port``, ``user``, ``root``)::

    ssh://[user@]host[:port]/abs/dir        URL form
    [user@]host:/abs/dir                     scp form
    :ssh,host='h',port='22':/abs/dir         rclone form (what ``Connection`` renders)

Layout, as in the reference's bucket (``RCLONE_REMOTE/data``, ``RCLONE_REMOTE/reports``,
machine-script.sh.tpl:51,89,108-124)::

    <dir>/data/       the task's working directory (restored into the node at create, synced
                      back every TPI_SYNC_INTERVAL s while it runs and once at the end)
    <dir>/reports/    task-<machine>, status-<machine> logs and statuses

``leo delete`` pulls ``storage.output`` from ``<dir>/data`` and leaves the container in place
(the reference only empties buckets it created, ``task/aws/task.go:245-299``).
"""
from __future__ import annotations

import json
import logging
import os
import posixpath
import re
import shlex
import subprocess
import tempfile
import threading
from typing import Dict, Iterable, List, Optional, Tuple

from . import objectnames
from .transfer import Connection, make_filter, transfer_rules
from ..ops import native

log = logging.getLogger("tpi")

BACKENDS = ("ssh", "sftp")
_URL = re.compile(r"^ssh://(?:(?P<user>[A-Za-z0-9._-]+)@)?(?P<host>[A-Za-z0-9_][A-Za-z0-9._-]*|\[[0-9A-Fa-f:.]+\])"
                  r"(?::(?P<port>\d+))?(?P<path>/.*)?$")
_SCP = re.compile(r"^(?:(?P<user>[A-Za-z0-9._-]+)@)?(?P<host>[A-Za-z0-9_][A-Za-z0-9._-]*):(?P<path>/.*)$")
_HOST = re.compile(r"^(?:[A-Za-z0-9._][A-Za-z0-9._-]*@)?(?:[A-Za-z0-9_][A-Za-z0-9._-]*|\[[0-9A-Fa-f:.]+\])$")


def parse(container: str, path: str = "", opts: Optional[Dict[str, str]] = None
          ) -> Optional[Connection]:
    """The SSH :class:`Connection` named by a ``storage.container`` value (None: not an
    off-node container).  ``opts`` (``container_opts``) may give ``host``/``port``/``user``
    and a ``root`` that a relative directory is taken under.  Object-store containers
    (``s3://``, ``gs://``, ``az://`` and rclone's forms) parse to their own connections
    (:mod:`storage.objectstore`)."""
    obj = objectnames.parse(container, path, opts)
    if obj is not None:
        return obj
    opts = dict(opts or {})
    conn = None
    m = _URL.match(container) if container.startswith("ssh://") else _SCP.match(container)
    if m:
        conn = Connection("ssh", m.group("host"), m.group("path") or "/",
                          {"host": m.group("host")})
        if m.group("user"):
            conn.config["user"] = m.group("user")
        if m.groupdict().get("port"):
            conn.config["port"] = m.group("port")
    elif container.startswith(":"):
        parsed = Connection.parse(container)
        if parsed.backend in BACKENDS:
            rest, host = parsed.container, parsed.config.get("host", "")
            if ":" in rest:  # "host:/dir"
                head, _, rest = rest.partition(":")
                host = host or head
            elif host and rest.startswith(host + "/"):  # str(Connection): "host/dir"
                rest = rest[len(host):]
            conn = Connection("ssh", host, rest, dict(parsed.config))
    elif opts.get("host") and container:
        conn = Connection("ssh", opts["host"], container, {})
    if conn is None:
        return None
    for key in ("host", "port", "user"):
        if opts.get(key):
            conn.config[key] = str(opts[key])
    conn.config.setdefault("host", conn.container)
    directory = conn.path or "/"
    if not directory.startswith("/"):
        directory = posixpath.join(opts.get("root") or "/", directory)
    if path:
        directory = posixpath.join(directory, path.lstrip("/"))
    conn.path = posixpath.normpath(directory)
    conn.container = conn.config["host"]
    return conn


def is_remote(value: str) -> bool:
    """Does ``value`` (a container or a file path) name a location on another node?"""
    if not value:
        return False
    if objectnames.is_object_store(value):
        return True
    if value.startswith("ssh://"):
        return bool(_URL.match(value))
    return bool(_SCP.match(value)) or value.startswith(tuple(":%s," % b for b in BACKENDS))


class SSHRemote:
    """File operations on the storage node, one transport command each."""

    def __init__(self, conn: Connection):
        if conn.backend not in BACKENDS:
            raise ValueError("not an ssh connection: %s" % conn)
        host = conn.config.get("host") or conn.container
        if conn.config.get("user") and "@" not in host:
            host = "%s@%s" % (conn.config["user"], host)
        if not _HOST.match(host):  # it goes into ssh's argv: no options smuggled in
            raise ValueError("storage host %r is not [user@]hostname" % host)
        port = conn.config.get("port")
        if port is not None and not str(port).isdigit():
            raise ValueError("storage port %r is not a number" % port)
        self.host, self.port, self.root = host, port, conn.path or "/"
        self.ssh = shlex.split(os.environ.get("TPI_SSH_COMMAND", "ssh -o BatchMode=yes"))

    def path(self, *parts: str) -> str:
        return posixpath.normpath(posixpath.join(self.root, *[p.lstrip("/") for p in parts]))

    def _argv(self, command: str) -> List[str]:
        argv = list(self.ssh)
        if self.port:
            argv += ["-p", str(self.port)]
        return argv + [self.host, command]

    def run(self, command: str, stdin: Optional[bytes] = None, timeout: float = 3600.0) -> bytes:
        proc = subprocess.run(self._argv(command), input=stdin, stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, timeout=timeout)
        if proc.returncode != 0:
            raise OSError("storage node %s: %s: exit %d: %s" % (
                self.host, command[:200], proc.returncode,
                proc.stderr.decode(errors="replace")[-1000:]))
        return proc.stdout

    def exists(self, rel: str = "") -> bool:
        try:
            self.run("test -e %s" % shlex.quote(self.path(rel)))
            return True
        except OSError:
            return False

    # -- trees (tar streams, filtered on this side) ----------------------------------------------
    def put_tree(self, local_dir: str, rel: str, rules: Optional[List[str]] = None,
                 only: Optional[Iterable[str]] = None) -> Dict[str, int]:
        """Copy ``local_dir`` (filter ``rules``; ``only``: just these relative paths) into
        ``<root>/<rel>`` -- rclone copy semantics: nothing there is deleted."""
        import tarfile  # SSH containers only: not on every apply's import path

        flt = make_filter(transfer_rules([]) if rules is None else rules)
        entries = [e for e in native().walk(local_dir, flt) if not e[4]]
        if only is not None:
            wanted = set(only)
            entries = [e for e in entries if e[0] in wanted]
        dest = self.path(rel)
        command = "mkdir -p %s && tar -x -f - -C %s" % (shlex.quote(dest), shlex.quote(dest))
        proc = subprocess.Popen(self._argv(command), stdin=subprocess.PIPE,
                                stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
        nbytes = 0
        err = b""

        def drain():
            nonlocal err
            err = proc.stderr.read()

        reader = threading.Thread(target=drain, daemon=True)
        reader.start()
        try:
            with tarfile.open(fileobj=proc.stdin, mode="w|") as tar:
                for relpath, size, _mtime, _mode, _ in entries:
                    tar.add(os.path.join(local_dir, relpath), arcname=relpath, recursive=False)
                    nbytes += size
        finally:
            proc.stdin.close()
            rc = proc.wait()
            reader.join()
        if rc != 0:
            raise OSError("storage node %s: upload into %s failed (exit %d): %s" % (
                self.host, dest, rc, err.decode(errors="replace")[-1000:]))
        return {"files": len(entries), "bytes": nbytes}

    def get_tree(self, rel: str, local_dir: str, rules: Optional[List[str]] = None
                 ) -> Dict[str, int]:
        """Copy ``<root>/<rel>`` into ``local_dir`` through filter ``rules`` (a missing remote
        directory copies nothing)."""
        import tarfile

        src = self.path(rel)
        command = "if [ -d %s ]; then tar -c -f - -C %s .; fi" % (shlex.quote(src),
                                                                 shlex.quote(src))
        flt = make_filter(transfer_rules([]) if rules is None else rules)
        proc = subprocess.Popen(self._argv(command), stdout=subprocess.PIPE,
                                stderr=subprocess.PIPE)
        files = nbytes = 0
        os.makedirs(local_dir, exist_ok=True)
        try:
            with tarfile.open(fileobj=proc.stdout, mode="r|") as tar:
                for member in tar:
                    name = posixpath.normpath(member.name)
                    if name in (".", "") or not member.isfile():
                        continue
                    if name.startswith("../") or name.startswith("/") or not flt.include_file(name):
                        continue
                    target = os.path.join(local_dir, name)
                    os.makedirs(os.path.dirname(target), exist_ok=True)
                    src_f = tar.extractfile(member)
                    tmp = target + ".tpi-partial"
                    with open(tmp, "wb") as out:
                        while True:
                            block = src_f.read(1 << 22)
                            if not block:
                                break
                            out.write(block)
                    os.chmod(tmp, member.mode & 0o777 or 0o644)
                    os.replace(tmp, target)
                    files += 1
                    nbytes += member.size
        except tarfile.ReadError as error:  # an empty stream: no such directory there
            if files:
                raise OSError("storage node %s: bad tar stream: %s" % (self.host, error))
        finally:
            rc = proc.wait()
        if rc != 0:
            raise OSError("storage node %s: download of %s failed (exit %d): %s" % (
                self.host, src, rc, proc.stderr.read().decode(errors="replace")[-1000:]))
        return {"files": files, "bytes": nbytes}

    def remove(self, rels: Iterable[str]) -> None:
        paths = [shlex.quote(self.path(r)) for r in rels]
        for i in range(0, len(paths), 256):
            self.run("rm -f -- %s" % " ".join(paths[i:i + 256]))

    # -- single files ---------------------------------------------------------------------------
    def put_file(self, local: str, rel: str) -> int:
        dest = self.path(rel)
        tmp = dest + ".tpi-partial"
        command = "mkdir -p %s && cat > %s && mv -f %s %s" % (
            shlex.quote(posixpath.dirname(dest)), shlex.quote(tmp), shlex.quote(tmp),
            shlex.quote(dest))
        with open(local, "rb") as f:
            proc = subprocess.run(self._argv(command), stdin=f, stdout=subprocess.DEVNULL,
                                  stderr=subprocess.PIPE, timeout=3600)
        if proc.returncode != 0:
            raise OSError("storage node %s: writing %s failed: %s" % (
                self.host, dest, proc.stderr.decode(errors="replace")[-1000:]))
        return os.path.getsize(local)

    def put_bytes(self, data: memoryview, rel: str) -> int:
        """Write a buffer as one file (a checkpoint slot straight from its host region)."""
        view = memoryview(data).cast("B")
        dest = self.path(rel)
        tmp = dest + ".tpi-partial"
        command = "mkdir -p %s && cat > %s && mv -f %s %s" % (
            shlex.quote(posixpath.dirname(dest)), shlex.quote(tmp), shlex.quote(tmp),
            shlex.quote(dest))
        proc = subprocess.Popen(self._argv(command), stdin=subprocess.PIPE,
                                stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
        err = b""

        def drain():
            nonlocal err
            err = proc.stderr.read()

        reader = threading.Thread(target=drain, daemon=True)
        reader.start()
        try:
            for off in range(0, view.nbytes, 64 << 20):
                proc.stdin.write(view[off:off + (64 << 20)])
        except BrokenPipeError:
            pass
        finally:
            proc.stdin.close()
            rc = proc.wait()
            reader.join()
        if rc != 0:
            raise OSError("storage node %s: writing %s failed: %s" % (
                self.host, dest, err.decode(errors="replace")[-1000:]))
        return view.nbytes

    def get_file(self, rel: str, local: str) -> int:
        src = self.path(rel)
        tmp = local + ".tpi-partial"
        with open(tmp, "wb") as f:
            proc = subprocess.run(self._argv("cat %s" % shlex.quote(src)), stdout=f,
                                  stderr=subprocess.PIPE, timeout=3600)
        if proc.returncode != 0:
            os.remove(tmp)
            raise FileNotFoundError("storage node %s: %s: %s" % (
                self.host, src, proc.stderr.decode(errors="replace")[-500:]))
        os.replace(tmp, local)
        return os.path.getsize(local)


def open_remote(conn: Connection):
    """The file operations of an off-node container: :class:`SSHRemote`, or an object store's
    (:func:`storage.objectstore.open_remote`) -- the same interface."""
    if conn.backend in BACKENDS:
        return SSHRemote(conn)
    from . import objectstore  # the HTTP clients: only for a task that names an object store

    return objectstore.open_remote(conn)


def describe(conn: Connection) -> str:
    """A container for logs and events (an object store's credentials left out)."""
    return str(conn) if conn.backend in BACKENDS else objectnames.describe(conn)


def split_file(location: str) -> Tuple[SSHRemote, str]:
    """(remote, file path) of a remote file location (any of the container forms)."""
    conn = parse(location)
    if conn is None:
        raise ValueError("%r is not a remote location" % location)
    directory, name = posixpath.split(conn.path)
    conn.path = directory or ("/" if conn.backend in BACKENDS else "")
    return open_remote(conn), name


def fetch(location: str, directory: Optional[str] = None) -> str:
    """Download a remote file into a local temporary file; returns its path (the caller
    removes it)."""
    remote, name = split_file(location)
    fd, tmp = tempfile.mkstemp(prefix="tpi-fetch-", suffix="-" + name, dir=directory)
    os.close(fd)
    try:
        remote.get_file(name, tmp)
    except BaseException:
        os.remove(tmp)
        raise
    return tmp


def file_exists(location: str) -> bool:
    remote, name = split_file(location)
    return remote.exists(name)


def store(local: str, location: str) -> int:
    remote, name = split_file(location)
    return remote.put_file(local, name)


def object_source(location: str):
    """``(remote, key)`` of an object-store file location, read in place by ranged requests
    (:meth:`ObjectRemote.read_into`); None for other locations (fetched whole)."""
    if not objectnames.is_object_store(location):
        return None
    return split_file(location)


def store_bytes(data: memoryview, location: str) -> int:
    """Write a buffer to a remote file location (no local temporary file)."""
    remote, name = split_file(location)
    return remote.put_bytes(data, name)


# -- the running task's mirror (the reference's 10 s data loop and its final copy) --------------

MANIFEST = "remote-sync.json"


def _snapshot(directory: str, rules: Optional[List[str]] = None) -> Dict[str, List[int]]:
    if not os.path.isdir(directory):
        return {}
    flt = make_filter(transfer_rules([]) if rules is None else rules)
    return {e[0]: [e[1], e[2]] for e in native().walk(directory, flt) if not e[4]}


def sync_task(task_root: str) -> int:
    """Mirror a task's working directory and reports into its off-node container: files new
    or changed since the last sync are uploaded, files this mirror uploaded earlier and that
    are gone locally are removed there (``rclone sync`` of ``machine-script.sh.tpl:118-124``,
    limited to what it wrote -- other data in the container is never touched).  Returns 0, or
    1 on a transport error (reported on stderr; the next sync retries)."""
    with open(os.path.join(task_root, "task.json")) as f:
        saved = json.load(f)
    rs = saved.get("remote_storage") or {}
    conn = parse(rs.get("container", ""), rs.get("path", ""), rs.get("config") or {})
    if conn is None:
        return 0
    remote = open_remote(conn)
    manifest_path = os.path.join(task_root, "supervisor", MANIFEST)
    try:
        with open(manifest_path) as f:
            last = json.load(f)
    except (OSError, ValueError):
        last = {}
    state = {}
    try:
        for sub, local in (("data", os.path.join(task_root, "data")),
                           ("reports", os.path.join(task_root, "reports"))):
            rules = transfer_rules(saved.get("exclude") or []) if sub == "data" else ["+ **"]
            now = _snapshot(local, rules)
            before = {k: v for k, v in (last.get(sub) or {}).items()}
            changed = [p for p, meta in now.items() if before.get(p) != meta]
            gone = [p for p in before if p not in now]
            if changed:
                remote.put_tree(local, sub, rules, only=changed)
            if gone and sub == "data":
                remote.remove([posixpath.join(sub, p) for p in gone])
            state[sub] = now
    except (OSError, subprocess.SubprocessError, ValueError) as error:
        print("tpi-remote-sync: %s" % error, file=__import__("sys").stderr, flush=True)
        return 1
    tmp = manifest_path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(state, f)
    os.replace(tmp, manifest_path)
    return 0


def main(argv: Optional[List[str]] = None) -> int:
    import sys

    argv = sys.argv[1:] if argv is None else argv
    if len(argv) != 2 or argv[0] != "sync":
        print("usage: remote sync <task root>", file=sys.stderr)
        return 2
    return sync_task(argv[1])


if __name__ == "__main__":
    raise SystemExit(main())
