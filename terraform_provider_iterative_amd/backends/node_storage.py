"""Task storage of a node task (a :class:`~.node.NodeTask` mixin): the task directory, the
workdir push into it (or into an off-node container), its restore from the container, and
the output pull.

Reference: ``machine.Transfer`` (rclone ``sync.CopyDir`` with filter rules,
``task/common/machine/storage.go:123-159``) in ``Push``/``Pull`` of every backend
(``task/aws/task.go:316-322``), ``LimitTransfer`` for the output (``storage.go:267-280``).
"""
from __future__ import annotations

import logging
import os
import time

from ..storage import remote as remote_storage
from ..storage import transfer as storage
from .nodeio import _write_json

log = logging.getLogger("tpi")


class NodeStorage:
    """The storage half of :class:`~.node.NodeTask`."""

    def _create_storage(self) -> None:
        for d in (self.root, self.reports_dir, self.sup_dir):
            os.makedirs(d, exist_ok=True)
        try:
            os.remove(self._stop_marker())
        except FileNotFoundError:
            pass
        os.makedirs(self.data_dir, exist_ok=True)
        if self._saved is None:
            self._saved = self._definition()
            _write_json(self.task_file, self._saved)
            self._event("created", "task %s" % self.id)

    def push(self) -> None:
        directory = self.spec.environment.directory
        if not directory:
            return
        if self.remote_conn is not None:  # into the container; the node restores from it
            stats = remote_storage.open_remote(self.remote_conn).put_tree(
                directory, "data", storage.transfer_rules(self.spec.environment.exclude_list))
            log.info("Uploaded %d files to %s", stats["files"],
                     remote_storage.describe(self.remote_conn))
            return
        t0 = time.perf_counter()
        if os.environ.get("TPI_PUSH_LINK", "") in ("1", "true", "yes"):
            # hard links instead of copies (opt-in: no snapshot, see storage.link_tree)
            st = storage.link_tree(directory, self.data_dir, self.spec.environment.exclude_list)
            self._event("pushed", "%d files" % (st["linked"] + st["copied"]),
                        "%d bytes" % st["bytes"], "%.3f s" % (time.perf_counter() - t0),
                        "hard links %d" % st["linked"])
            return
        # the default: a snapshot of the workdir -- each file reflinked (FICLONE: shared
        # extents, copy-on-write) where the filesystem can, else copied by 16 threads
        st = storage.transfer(directory, self.data_dir, self.spec.environment.exclude_list)
        self._event("pushed", "%d files" % st.get("files", 0), "%d bytes" % st.get("bytes", 0),
                    "%.3f s" % (time.perf_counter() - t0),
                    "reflinked %d" % st.get("cloned", 0))

    def _restore_remote(self) -> None:
        stats = remote_storage.open_remote(self.remote_conn).get_tree("data", self.data_dir,
                                                                    ["+ **"])
        self._event("container-restored", remote_storage.describe(self.remote_conn),
                    "%d files" % stats["files"], "%d bytes" % stats["bytes"])

    def pull(self) -> None:
        saved = self._saved or {}
        directory = self.spec.environment.directory or saved.get("directory") or "."
        out = self.spec.environment.directory_out or saved.get("directory_out") or ""
        excludes = self.spec.environment.exclude_list or saved.get("exclude") or []
        rules = storage.limit_transfer(out, storage.transfer_rules(excludes))
        if self.remote_conn is not None:  # the container holds the task's final data
            remote_storage.open_remote(self.remote_conn).get_tree("data", directory, rules)
            return
        storage.transfer(self.data_dir, directory, rules=rules)

    def _delete_storage(self) -> None:
        # With a pre-allocated container the data lives outside self.root and is kept
        # (the reference only empties buckets it created, task/aws/task.go:245-299).
        if os.path.isdir(self.root):
            storage.native().remove_tree(self.root)
