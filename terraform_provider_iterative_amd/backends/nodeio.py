"""Small file and control-socket helpers shared by the node backend's modules
(``node.py``, ``node_queue.py``, ``node_storage.py``)."""
from __future__ import annotations

import json
import os
import time
from typing import Dict, Optional


def control_socket(sup_dir: str, command: str, timeout: float = 2.0) -> Optional[Dict]:
    """One request on a supervisor's control socket (``<sup_dir>/control.sock``); the reply as
    a dict, or None when no supervisor is listening.  The path is reached through
    ``/proc/self/fd`` because AF_UNIX paths are limited to 108 bytes (the supervisor binds
    the same way)."""
    import socket  # not on `tpi apply`'s path (tests/test_import_budget.py)

    try:
        dfd = os.open(sup_dir, os.O_RDONLY | os.O_DIRECTORY)
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
