"""Storage sync library (reference: ``task/common/machine/storage.go``).

The reference drives rclone against cloud buckets; here a task's "remote" is a directory of
the node (the task's storage root, or a pre-allocated ``storage.container`` directory), and
the copy engine is the native parallel walker in ``csrc/native/transfer.cpp`` with rclone's
filter semantics (``csrc/native/filter.cpp``).
"""
from __future__ import annotations

import json
import logging
import os
import posixpath
import shutil
from typing import Dict, Iterable, List, Optional

from ..utils.record import field, record
from ..models.values import STATUS_FAILED, STATUS_SUCCEEDED, NotFoundError, new_status
from ..ops import native

log = logging.getLogger("tpi")

# storage.go:37-41
DEFAULT_TRANSFER_EXCLUDES = ["- /main.tf", "- /terraform.tfstate*", "- /.terraform**"]


def _go_join_root(rule: str) -> str:
    """``filepath.Join("/", rule)`` (clean, rooted, no trailing slash)."""
    cleaned = posixpath.normpath("/" + rule)
    if cleaned.startswith("//"):
        cleaned = "/" + cleaned.lstrip("/")
    return cleaned


def is_rclone_filter(rule: str) -> bool:
    return rule.startswith("+ ") or rule.startswith("- ")


def transfer_rules(exclude: Optional[Iterable[str]] = None) -> List[str]:
    """Default excludes + user rules; bare patterns become anchored excludes
    (``storage.go:127-141``)."""
    rules = list(DEFAULT_TRANSFER_EXCLUDES)
    for rule in exclude or []:
        rules.append(rule if is_rclone_filter(rule) else "- " + _go_join_root(rule))
    return rules


def limit_transfer(subdir: str, rules: List[str]) -> List[str]:
    """Restrict a transfer to one sub-directory (``storage.go:267-280``)."""
    directory = posixpath.normpath(subdir) if subdir else ""
    if directory in ("", "."):
        return rules
    return list(rules) + ["+ " + _go_join_root(directory),
                          "+ " + posixpath.join(_go_join_root(directory), "**"),
                          "- /**"]


def make_filter(rules: Iterable[str]):
    return native().Filter(list(rules))


def human_size(size: float) -> str:
    """docker/go-units HumanSize (decimal units, 4 significant digits)."""
    units = ["B", "kB", "MB", "GB", "TB", "PB", "EB", "ZB", "YB"]
    i = 0
    while size >= 1000 and i < len(units) - 1:
        size /= 1000.0
        i += 1
    return ("%.4g%s" % (size, units[i]))


def _local_path(remote: str) -> str:
    conn = Connection.parse(remote)
    return conn.local_path()


def _copy_threads() -> int:
    """``TPI_PUSH_THREADS``, else one per CPU this process may run on, 8-16."""
    env = os.environ.get("TPI_PUSH_THREADS")
    if env:
        return max(1, int(env))
    try:
        cpus = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        cpus = os.cpu_count() or 8
    return max(8, min(16, cpus))


def link_tree(source: str, destination: str, exclude: Optional[Iterable[str]] = None) -> Dict:
    """Hard-link ``source``'s files (rclone filter rules as :func:`transfer`) into
    ``destination`` instead of copying them: an apply of a 10 GB workdir then costs metadata
    operations only.  Opt-in (``TPI_PUSH_LINK=1``) because a link is not a snapshot: a file
    the user edits in place after the apply, or the task rewrites in place, is the same file
    on both sides (a file replaced by rename -- what most editors and the task's output
    sync do -- is not).  Files on another filesystem, or where links are refused, are
    copied.  Returns ``{"linked", "copied", "bytes"}``."""
    src, dst = _local_path(source), _local_path(destination)
    flt = make_filter(transfer_rules(exclude))
    linked = copied = nbytes = 0
    os.makedirs(dst, exist_ok=True)
    for rel, size, _mtime, _mode, is_dir in native().walk(src, flt):
        target = os.path.join(dst, rel)
        if is_dir:
            os.makedirs(target, exist_ok=True)
            continue
        os.makedirs(os.path.dirname(target), exist_ok=True)
        if os.path.lexists(target):
            os.remove(target)
        try:
            os.link(os.path.join(src, rel), target)
            linked += 1
        except OSError:  # EXDEV, EPERM, ...: copy this one
            shutil.copy2(os.path.join(src, rel), target)
            copied += 1
        nbytes += size
    log.info("Linked %d files (%s), copied %d", linked, human_size(nbytes), copied)
    return {"linked": linked, "copied": copied, "bytes": nbytes}


def transfer(source: str, destination: str, exclude: Optional[Iterable[str]] = None,
             rules: Optional[List[str]] = None, threads: int = 0) -> Dict:
    """Copy ``source`` -> ``destination`` with filter rules (``storage.go:123-159``).

    ``rules`` (already in rclone form) overrides the default-exclude construction, which is
    how :func:`limit_transfer` results are applied.
    """
    src, dst = _local_path(source), _local_path(destination)
    rules = transfer_rules(exclude) if rules is None else rules
    flt = make_filter(rules)
    entries = native().walk(src, flt)
    files = [e for e in entries if not e[4]]
    log.info("Transferring %s (%d files)...", human_size(sum(e[1] for e in files)), len(files))
    # 64 MiB copy_file_range pieces, handed out round-robin over files (writers of one file
    # serialise on its inode lock).  A copy into tmpfs / the page cache is bound per thread by
    # page allocation + memcpy (~2-3 GB/s), so it scales with the threads the task may use.
    # 10 x 1 GB on the MI355X box's /tmp, 16 threads, median of 5: 63.7 GB/s with 64 MiB
    # pieces (61.7-65.6), 58.7 with 256 MiB (50.8-59.2) (profiles/round6/r6v/summary.txt)
    stats = native().copy_dir(src, dst, flt, threads or _copy_threads(), 64 << 20)
    log.debug("transfer %s -> %s: %s", src, dst, stats)
    return stats


def delete(destination: str) -> int:
    """Remove a remote directory tree (``storage.go:161-186``)."""
    path = _local_path(destination)
    if not os.path.exists(path):
        raise NotFoundError("storage not found: %s" % path)
    return native().remove_tree(path)


def check_storage(remote: str) -> None:
    """``storage.go:214-225``: the remote must be listable (a missing dir is fine)."""
    path = _local_path(remote)
    if os.path.exists(path) and not os.access(path, os.R_OK | os.X_OK):
        raise PermissionError("failed to access remote storage: %s" % path)


def reports(remote: str, prefix: str) -> List[str]:
    """Contents of ``<remote>/reports/<prefix>-*`` sorted by name (``storage.go:58-93``)."""
    directory = os.path.join(_local_path(remote), "reports")
    try:
        names = sorted(os.listdir(directory))
    except FileNotFoundError:
        return []
    out = []
    for name in names:
        if not name.startswith(prefix + "-") or name.endswith(".tmp"):
            continue
        try:
            with open(os.path.join(directory, name), "r", errors="replace") as handle:
                out.append(handle.read())
        except FileNotFoundError:
            continue
    return out


def logs(remote: str) -> List[str]:
    return reports(remote, "task")


def status(remote: str, initial: Optional[Dict[str, int]] = None) -> Dict[str, int]:
    """Fold ``status-*`` reports into the status map (``storage.go:99-121``)."""
    result = dict(initial) if initial is not None else new_status()
    for report in reports(remote, "status"):
        data = json.loads(report)
        code = str(data.get("code", "") or "")
        if code:
            key = STATUS_SUCCEEDED if code == "0" else STATUS_FAILED
            result[key] = result.get(key, 0) + 1
        elif data.get("result") == "timeout":
            result[STATUS_FAILED] = result.get(STATUS_FAILED, 0) + 1
    return result


@record
class Connection:
    """rclone-style connection string (``storage.go:229-263``).

    ``:backend,k='v':container/path``; the node runtime understands ``local`` (and bare
    paths); other backends are kept for configuration compatibility.
    """

    backend: str = "local"
    container: str = ""
    path: str = ""
    config: Dict[str, str] = field(default_factory=dict)

    def __str__(self) -> str:
        opts = sorted("%s='%s'" % (k, v) for k, v in self.config.items())
        conn_opts = ("," + ",".join(opts)) if opts else ""
        pth = ""
        if self.path:
            pth = posixpath.normpath(self.path)
            if not pth.startswith("/"):
                pth = "/" + pth
        return ":%s%s:%s%s" % (self.backend, conn_opts, self.container, pth)

    @classmethod
    def parse(cls, remote: str) -> "Connection":
        if not remote.startswith(":"):
            return cls(backend="local", container=remote)
        # split ``backend,k='v',...`` from the path at the first ':' outside quotes, and the
        # options at ',' outside quotes (a quoted value may hold either, e.g. an endpoint URL)
        parts, cur, quote, rest = [], "", "", None
        for i, ch in enumerate(remote[1:], 1):
            if quote:
                if ch == quote:
                    quote = ""
                cur += ch
            elif ch in "'\"":
                quote = ch
                cur += ch
            elif ch == ",":
                parts.append(cur)
                cur = ""
            elif ch == ":":
                rest = remote[i + 1:]
                break
            else:
                cur += ch
        if rest is None:
            raise ValueError("malformed connection string %r" % remote)
        parts.append(cur)
        config = {}
        for item in parts[1:]:
            key, _, value = item.partition("=")
            config[key] = value.strip("'\"")
        return cls(backend=parts[0], container=rest, config=config)

    @classmethod
    def existing_bucket(cls, provider: str, container: str, path: str = "",
                        config: Optional[Dict[str, str]] = None,
                        credentials: Optional[Dict[str, str]] = None) -> "Connection":
        """Connection of a pre-allocated ``storage.container`` per cloud (the reference's
        ``ExistingS3Bucket`` / ``ExistingBucket`` / ``ExistingBlobContainer`` data sources,
        ``task/{aws,gcp,az}/resources/data_source_*.go``)."""
        config = dict(config or {})
        credentials = credentials or {}
        if provider == "aws":
            return cls("s3", container, path, {
                "provider": "AWS", "region": config.get("region", ""),
                "access_key_id": credentials.get("AccessKeyID", ""),
                "secret_access_key": credentials.get("SecretAccessKey", ""),
                "session_token": credentials.get("SessionToken", "")})
        if provider == "gcp":
            return cls("googlecloudstorage", container, path, {
                "service_account_credentials": credentials.get("ApplicationCredentials", "")})
        if provider == "az":
            return cls("azureblob", container, path, config)
        if provider in ("local", "mi355x"):
            return cls("local", container, path, config)
        raise ValueError("no storage backend for provider %r" % provider)

    def local_path(self) -> str:
        if self.backend != "local":
            raise NotImplementedError(
                "backend %r is not reachable from the node-local runtime" % self.backend)
        return os.path.join(self.container, self.path.lstrip("/")) if self.path else self.container
