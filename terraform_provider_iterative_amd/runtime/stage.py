"""The task runtime's HBM workdir: plan the stager, attach to its copies from a rank.

The reference restores a task's workdir on each of its ``parallelism`` machines before the
script starts (``machine-script.sh.tpl:89``; ``resource_auto_scaling_group.go:70``) and
re-syncs it every 10 s (``tpl:118-124``).  On the ``mi355x`` backend the supervisor starts
``tpi-stager`` (``csrc/stager/stager.cpp``) first: the workdir becomes one flat image in HBM
on every rank's GPU (sharded H2D over every GPU's own PCIe link + one in-place RCCL
all-gather over xGMI), verified by the shard-hash kernel, and the stager stays up to write
dirty shards back on the reference's cadence.  Ranks start with ``TPI_HBM_WORKDIR`` naming
the stager's manifest and map their copy zero-copy with :func:`attach` -- no user code is
needed for the staging itself.  The ranks start while the stager is still loading (their
interpreter and framework start-up overlaps the H2D copies, and the first log line does not
wait for the workdir); :func:`attach` blocks until the manifest lands.

Knobs (task ``environment`` or the provider's environment):

=========================  =====================================================================
``TPI_STAGE``              ``auto`` (default: stage mi355x tasks whose workdir holds at least
                           ``TPI_STAGE_MIN_BYTES``), ``hbm`` (always), ``host`` (images in
                           ``/dev/shm``: CPU rehearsal, any backend), ``off``
``TPI_STAGE_MIN_BYTES``    default 64 MiB
``TPI_STAGE_METHOD``       ``sharded`` (default), ``broadcast``, ``independent``
``TPI_SYNC_INTERVAL``      write-back cadence in seconds (default 10, as tpl:118-124; 0 = off)
``TPI_STAGE_WRITEBACK``    ``1`` (default) / ``0``
``TPI_STAGE_THREADS``      page-cache reader threads per GPU loader (default 16: 10 GB on one
                           MI355X stages at 39 GB/s with 8, 50 GB/s with 16 -- the PCIe-bound
                           H2D then sets the pace; profiles/config2_stager_threads_round2.json)
``TPI_STAGE_CHUNK_BYTES``  pinned ring chunk (default 64 MiB; 256 MiB was slower: 32 GB/s)
``TPI_STAGE_WAIT``         ``1``: start the ranks only once the workdir is staged (default ``0``)
``TPI_HBM_WORKDIR_TIMEOUT`` how long :func:`attach` waits for the stager (default 600 s)
=========================  =====================================================================
"""
from __future__ import annotations

import json
import os
from typing import Dict, List, Optional, Sequence, Tuple

ALIGN = 4096
DEFAULT_MIN_BYTES = 64 << 20
METHODS = ("sharded", "broadcast", "independent")


def _env(environ, key: str, default: str) -> str:
    value = environ.get(key)
    return default if value in (None, "") else str(value)


def layout(root: str) -> Tuple[List[Tuple[str, int, int]], int]:
    """Every regular file under ``root`` (already filtered by the push) as ``(relative path,
    image offset, size)`` at 4 KiB-aligned offsets, sorted; and the unpadded image size."""
    from ..ops import native
    from ..storage.transfer import make_filter

    files, off = [], 0
    for rel, size, _mtime, _mode, is_dir in sorted(native().walk(root, make_filter([]))):
        if is_dir:
            continue
        files.append((rel, off, int(size)))
        off += (int(size) + ALIGN - 1) // ALIGN * ALIGN
    return files, off


def mode(environ, provider: str, nbytes: int) -> str:
    """``"hbm"``, ``"host"`` or ``""`` (no staging) for a task of ``provider`` whose workdir
    holds ``nbytes``."""
    want = _env(environ, "TPI_STAGE", "auto").lower()
    if want in ("off", "0", "no", "false"):
        return ""
    if want == "host":
        return "host"
    if provider != "mi355x":
        return ""
    if want == "hbm":
        return "hbm"
    return "hbm" if nbytes >= int(_env(environ, "TPI_STAGE_MIN_BYTES", str(DEFAULT_MIN_BYTES))) \
        else ""


def plan(root: str, sup_dir: str, devices: Sequence[int], numa: Sequence[int],
         environ, host: bool = False, files=None, nbytes: Optional[int] = None) -> Dict:
    """Write ``<sup_dir>/stage.json`` for ``tpi-stager`` and return the supervisor's
    ``stager`` spec entry."""
    from .. import _build

    if files is None or nbytes is None:
        files, nbytes = layout(root)
    n = max(1, len(devices))
    quantum = ALIGN * n
    total = max(quantum, (nbytes + quantum - 1) // quantum * quantum)
    method = _env(environ, "TPI_STAGE_METHOD", "sharded")
    if method not in METHODS:
        raise ValueError("TPI_STAGE_METHOD must be one of %s" % (METHODS,))
    manifest = os.path.join(sup_dir, "stage-manifest.json")
    spec = {
        "root": root, "files": [list(f) for f in files], "total": total,
        "devices": list(devices), "numa": list(numa), "method": method,
        "chunk_bytes": int(_env(environ, "TPI_STAGE_CHUNK_BYTES", str(64 << 20))),
        "nbuf": 4, "threads": int(_env(environ, "TPI_STAGE_THREADS", "16")),
        "shard_bytes": 1 << 20, "manifest": manifest,
        "events": os.path.join(sup_dir, "events.jsonl"),
        "sync_interval": float(_env(environ, "TPI_SYNC_INTERVAL", "10")),
        "writeback": _env(environ, "TPI_STAGE_WRITEBACK", "1") != "0",
        "host": bool(host), "verify": True,
        "shm_prefix": "/dev/shm/tpi-stage-%s" % os.path.basename(os.path.dirname(sup_dir)),
    }
    path = os.path.join(sup_dir, "stage.json")
    with open(path + ".tmp", "w") as handle:
        json.dump(spec, handle)
    os.replace(path + ".tmp", path)
    binary = os.environ.get("TPI_STAGER_BIN") or _build.STAGER
    if binary == _build.STAGER:
        _build.build_stager()
    return {"argv": [binary, path], "manifest": manifest,
            "log": os.path.join(sup_dir, "stager.log"),
            "timeout": float(_env(environ, "TPI_STAGE_TIMEOUT", "600")),
            "before_ranks": _env(environ, "TPI_STAGE_WAIT", "0") not in ("0", "false", "no")}


# ---- rank side --------------------------------------------------------------------------------

class HbmWorkdir:
    """A rank's zero-copy view of the staged workdir (:func:`attach`)."""

    def __init__(self, manifest: Dict, rank: int, buffer, mapping: Optional[int] = None):
        self.manifest = manifest
        self.rank = rank
        self.root = manifest["root"]
        self.total = int(manifest["total"])
        self.files = [(f[0], int(f[1]), int(f[2])) for f in manifest["files"]]
        self._index = {f[0]: (f[1], f[2]) for f in self.files}
        self.buffer = buffer  # 1-D uint8 tensor (device, or host for host-mode images)
        self.stats = manifest.get("stats", {})
        self._mapping = mapping

    def tensor(self, path: str):
        """The bytes of ``path`` (relative to the workdir) as a uint8 view of the image."""
        off, size = self._index[path]
        return self.buffer[off:off + size]

    def paths(self) -> List[str]:
        return [f[0] for f in self.files]

    def digest(self, shard_bytes: int = 1 << 20):
        from ..ops import shard_hash

        return shard_hash(self.buffer, shard_bytes=shard_bytes)

    def close(self) -> None:
        self.buffer = None
        if self._mapping:
            from ..ops import hip

            import ctypes

            hip().tpi_ipc_close(ctypes.c_void_p(self._mapping))
            self._mapping = None


def wait_staged(path: str, timeout: Optional[float] = None) -> float:
    """Block until the stager published ``path`` (seconds waited).  Raises RuntimeError when
    the supervisor marked staging failed (``<path>.failed``) and TimeoutError after
    ``timeout`` (default ``TPI_HBM_WORKDIR_TIMEOUT`` or 600 s)."""
    import time

    if timeout is None:
        timeout = float(os.environ.get("TPI_HBM_WORKDIR_TIMEOUT", "600"))
    t0 = time.monotonic()
    delay = 0.0005
    while not os.path.exists(path):
        if os.path.exists(path + ".failed"):
            with open(path + ".failed") as handle:
                raise RuntimeError("workdir staging failed: %s" % handle.read().strip())
        if time.monotonic() - t0 > timeout:
            raise TimeoutError("workdir not staged after %.0f s (%s)" % (timeout, path))
        time.sleep(delay)
        delay = min(delay * 2, 0.005)
    return time.monotonic() - t0


def attach(manifest: Optional[str] = None, rank: Optional[int] = None,
           timeout: Optional[float] = None) -> HbmWorkdir:
    """Map this rank's copy of the staged workdir (``$TPI_HBM_WORKDIR``), waiting for the
    stager if it is still loading (:func:`wait_staged`)."""
    path = manifest or os.environ.get("TPI_HBM_WORKDIR")
    if not path:
        raise RuntimeError("no staged workdir: TPI_HBM_WORKDIR is not set (TPI_STAGE=off, "
                           "a small workdir, or staging failed -- see events.jsonl)")
    waited = wait_staged(path, timeout)
    with open(path) as handle:
        data = json.load(handle)
    data.setdefault("stats", {})["attach_wait_s"] = round(waited, 4)
    rank = int(os.environ.get("RANK", "0")) if rank is None else rank
    entry = data["ranks"][rank]
    if data.get("host"):
        import numpy as np
        import torch

        arr = np.memmap(entry["path"], dtype=np.uint8, mode="r+", shape=(int(data["total"]),))
        return HbmWorkdir(data, rank, torch.from_numpy(arr))
    from ..ops import hip

    lib = hip()
    device = int(entry["device"])
    ptr = _ipc_open_bounded(lib, bytes.fromhex(entry["ipc"]), device, int(data["total"]))
    from .stage_native import _device_tensor

    buffer = _device_tensor(ptr, int(data["total"]), device)
    return HbmWorkdir(data, rank, buffer, mapping=ptr)


def _ipc_open_bounded(lib, handle: bytes, device: int, nbytes: int,
                      timeout: Optional[float] = None) -> int:
    """``hipIpcOpenMemHandle`` of the stager's image, bounded by ``TPI_IPC_OPEN_TIMEOUT``
    (default 30 s here): an import that never returns (the HIP runtime's IPC import can spin
    forever, ``profiles/round5/ipc_cause.md``) fails the rank with a ``workdir-attach-failed``
    event instead of hanging it.  The opener is a daemon thread, so a stuck one cannot hold up
    the process's exit; if it returns after the deadline it closes its own mapping."""
    import ctypes
    import threading
    import time

    if timeout is None:
        try:
            timeout = float(os.environ.get("TPI_IPC_OPEN_TIMEOUT", "30"))
        except ValueError:
            timeout = 30.0
    result: Dict[str, object] = {}
    lock = threading.Lock()

    def opener() -> None:
        ptr = ctypes.c_void_p()
        rc = lib.tpi_ipc_open(handle, device, ctypes.byref(ptr))
        with lock:
            if "abandoned" not in result:
                result["rc"], result["ptr"] = rc, ptr.value
                return
        if rc == 0:
            lib.tpi_ipc_close(ptr)

    t0 = time.monotonic()
    thread = threading.Thread(target=opener, name="tpi-workdir-attach", daemon=True)
    thread.start()
    thread.join(timeout)
    with lock:
        if "rc" not in result:
            result["abandoned"] = True
    if "abandoned" in result:
        from ..checkpoint.preemption import journal

        message = ("workdir attach: hipIpcOpenMemHandle of the staged %.2f GB image on device "
                   "%d did not return within %.1f s (TPI_IPC_OPEN_TIMEOUT)" % (
                       nbytes / 1e9, device, timeout))
        journal("workdir-attach-failed", message)
        raise TimeoutError(message)
    lib.check(int(result["rc"]), "hipIpcOpenMemHandle")
    from ..checkpoint.preemption import journal

    journal("workdir-attached", "%.2f GB" % (nbytes / 1e9),
            "ipc open %.4f s" % (time.monotonic() - t0))
    return int(result["ptr"])


def __getattr__(name: str):
    """The ctypes side (DLPack views, the native loader) lives in :mod:`.stage_native`, so
    that planning a task's staging -- every ``tpi apply`` of an ``mi355x`` task -- does not
    import ``ctypes``; ``stage.Loader`` and ``stage._device_tensor`` still resolve here."""
    if name in ("Loader", "_device_tensor"):
        from . import stage_native

        return getattr(stage_native, name)
    raise AttributeError(name)
