"""Wait for changes under a directory (inotify), so ``leo read --follow`` on the node runtime
prints log lines as the supervisor writes them instead of on the reference's 3-second poll
(``cmd/leo/read/read.go:124``).  Falls back to sleeping when inotify is unavailable."""
from __future__ import annotations

import ctypes
import ctypes.util
import os
import select
import time
from typing import Iterable, Optional

IN_MODIFY, IN_CLOSE_WRITE, IN_CREATE, IN_MOVED_TO = 0x2, 0x8, 0x100, 0x80
IN_NONBLOCK, IN_CLOEXEC = 0o4000, 0o2000000


class DirectoryWatch:
    def __init__(self, paths: Iterable[str]):
        self.fd: Optional[int] = None
        try:
            libc = ctypes.CDLL(ctypes.util.find_library("c") or "libc.so.6", use_errno=True)
            fd = libc.inotify_init1(IN_NONBLOCK | IN_CLOEXEC)
            if fd < 0:
                return
            mask = IN_MODIFY | IN_CLOSE_WRITE | IN_CREATE | IN_MOVED_TO
            watched = 0
            for path in paths:
                if os.path.isdir(path) and libc.inotify_add_watch(fd, path.encode(), mask) >= 0:
                    watched += 1
            if watched:
                self.fd = fd
            else:
                os.close(fd)
        except (OSError, AttributeError):
            self.fd = None

    def wait(self, timeout: float) -> bool:
        """Block until something changed (True) or ``timeout`` elapsed (False)."""
        if self.fd is None:
            time.sleep(timeout)
            return False
        ready, _, _ = select.select([self.fd], [], [], timeout)
        if ready:
            try:
                while os.read(self.fd, 65536):
                    pass
            except BlockingIOError:
                pass
            return True
        return False

    def close(self) -> None:
        if self.fd is not None:
            os.close(self.fd)
            self.fd = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
