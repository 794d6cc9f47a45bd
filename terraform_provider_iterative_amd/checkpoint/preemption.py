"""Preemption (SIGTERM) handling for rank processes.

The reference distinguishes preemption from completion on the VM: a machine that is
shutting down writes no status and gets respawned with the workdir restored from the bucket
(``machine-script.sh.tpl:10-15,51,89``).  Here the supervisor forwards SIGTERM to the ranks;
a rank that installed :func:`install` checkpoints its registered tensors to host memory (and
optionally the storage root) and exits with :data:`PREEMPTED_EXIT_CODE`, and its successor
calls :func:`resume` to restore them.
"""
from __future__ import annotations

import json
import logging
import os
import signal
import sys
import threading
import time
from typing import Callable, Dict, List, Optional

from .checkpointer import Checkpointer, CheckpointError

log = logging.getLogger("tpi.preemption")

PREEMPTED_EXIT_CODE = 143  # 128 + SIGTERM, what an un-handled SIGTERM would report

_registered: List[Checkpointer] = []
_persist_paths: Dict[int, str] = {}
_callbacks: List[Callable[[], Optional[Dict]]] = []
_installed = False
_fired = threading.Event()


def register(checkpointer: Checkpointer, persist_path: Optional[str] = None) -> None:
    _registered.append(checkpointer)
    if persist_path:
        _persist_paths[id(checkpointer)] = persist_path


def on_preempt(callback: Callable[[], Optional[Dict]]) -> None:
    """Callback run before the save; may return metadata (e.g. ``{"step": n}``)."""
    _callbacks.append(callback)


def preempted() -> bool:
    return _fired.is_set()


def journal(code: str, *description: str) -> None:
    """Append a phase event to the task's event journal (``TPI_EVENTS_FILE``, set by the
    supervisor), shown in ``iterative_task.events`` next to placement/start/exit events.
    One ``O_APPEND`` write per line, so concurrent ranks do not interleave."""
    path = os.environ.get("TPI_EVENTS_FILE")
    if not path:
        return
    rank = os.environ.get("RANK", "0")
    line = json.dumps({"time": time.time(), "code": code,
                       "description": ["rank " + rank] + list(description)}) + "\n"
    try:
        fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_APPEND, 0o644)
        try:
            os.write(fd, line.encode())
        finally:
            os.close(fd)
    except OSError:
        pass


def _describe(res) -> List[str]:
    return ["%d bytes" % res.bytes, "%d on the wire" % res.wire_bytes,
            "%.3f s" % res.seconds, "%.1f GB/s" % res.gbps]


def checkpoint_all(metadata: Optional[Dict] = None, on_stream=None) -> List[float]:
    """Save every registered checkpointer; returns per-checkpointer GB/s.  ``on_stream``
    (single checkpointer only): stream the save to the successor (see
    :meth:`Checkpointer.save`); called once the successor may start."""
    meta = dict(metadata or {})
    t0 = time.perf_counter()
    for cb in _callbacks:
        extra = cb()
        if extra:
            meta.update(extra)
    t_cb = time.perf_counter() - t0
    rates = []
    for ck in _registered:
        if on_stream is not None and len(_registered) == 1 and _hbm_handoff():
            try:  # the successor on this GPU copies our HBM while we spill to the host
                t1 = time.perf_counter()
                if ck.export_hbm():
                    journal("checkpoint-hbm-export", "successor may copy device to device",
                            "hand-off check %.3f s" % _phase.get("handoff-check", 0.0),
                            "callbacks %.3f s" % t_cb,
                            "export %.3f s" % (time.perf_counter() - t1))
            except Exception as error:  # the host path still works
                journal("checkpoint-hbm-export-failed", str(error))
        res = ck.save(meta, on_stream=on_stream if len(_registered) == 1 else None)
        rates.append(res.gbps)
        journal("checkpoint-saved", *_describe(res))
        path = _persist_paths.get(id(ck))
        if path:
            t0 = time.perf_counter()
            ck.persist(path)
            journal("checkpoint-persisted", path, "%.3f s" % (time.perf_counter() - t0))
    return rates


# -- periodic checkpoint cadence (reference: the 10 s data-sync loop, machine-script.sh.tpl:
#    118-124, which re-syncs the workdir to the bucket whenever its newest mtime changed) ------

_tick_last: Optional[float] = None
_tick_pending: Dict[int, object] = {}  # id(checkpointer) -> PendingSave of the last tick


def sync_interval() -> float:
    """Seconds between periodic checkpoints (``TPI_SYNC_INTERVAL``, default 10 as in the
    reference; 0 or less disables :func:`tick`)."""
    try:
        return float(os.environ.get("TPI_SYNC_INTERVAL", "10"))
    except ValueError:
        return 10.0


def _collect_finished() -> bool:
    """Journal the async spills of earlier ticks that have completed; True if none is still
    running."""
    running = False
    for key, pending in list(_tick_pending.items()):
        if not pending.done():
            running = True
            continue
        del _tick_pending[key]
        try:
            res = pending.result()
            journal("checkpoint-synced", "async", *_describe(res),
                    "stall %.1f ms" % (pending.stall_s * 1e3))
        except CheckpointError as error:
            journal("checkpoint-sync-failed", str(error))
    return not running


def _agree(due: bool) -> bool:
    """Ranks of one job checkpoint the same step: with ``torch.distributed`` initialised the
    decision is the minimum over ranks (one 4-byte all-reduce per call; every rank must call
    :func:`tick` at the same steps)."""
    dist = sys.modules.get("torch.distributed")
    if dist is None or not dist.is_available() or not dist.is_initialized() or \
            dist.get_world_size() < 2:
        return due
    import torch

    device = "cpu"
    if dist.get_backend() == "nccl":
        device = torch.device("cuda", torch.cuda.current_device())
    flag = torch.tensor([1 if due else 0], dtype=torch.int32, device=device)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    return bool(flag.item())


def tick(metadata: Optional[Dict] = None, force: bool = False) -> bool:
    """Periodic checkpoint hook: call it at a step boundary (where the registered tensors are
    consistent).  Every :func:`sync_interval` seconds it checkpoints every registered
    :class:`Checkpointer` into its host region, so a rank that dies without a SIGTERM (OOM,
    crash, SIGKILL after the grace period) still leaves a recent checkpoint behind.

    ``TPI_SYNC_MODE``:
      ``async`` (default)  HBM snapshot + background spill (:meth:`Checkpointer.save_async`):
                           the training stream stalls only for the snapshot, the PCIe leg
                           overlaps the next steps.  A tick that finds the previous spill still
                           running is skipped, never queued.
      ``sync``             incremental (:meth:`Checkpointer.sync`): only tiles whose device
                           digest changed since the last tick cross PCIe -- cheapest for mostly
                           frozen state (fine-tuning adapters, embeddings); blocks the caller.

    The first call arms the timer.  Returns True when this call checkpointed.  Each completed
    checkpoint is journalled (``checkpoint-synced``) with its bytes, wire bytes and time.  In a
    multi-rank job all ranks decide together (:func:`_agree`), so they checkpoint the same step
    and :meth:`TrainingState.resume_consistent` finds it on every rank.
    """
    global _tick_last
    if _fired.is_set() or not _registered:
        return False
    now = time.monotonic()
    idle = _collect_finished()
    if _tick_last is None and not force:
        _tick_last = now
        return False
    interval = sync_interval()
    if interval <= 0 and not force:
        return False
    due = idle and (force or now - _tick_last >= interval)
    if not _agree(due):
        return False
    meta = {"reason": "periodic"}
    for cb in _callbacks:
        extra = cb()
        if extra:
            meta.update(extra)
    meta.update(metadata or {})
    mode = os.environ.get("TPI_SYNC_MODE", "async")
    for ck in _registered:
        if mode == "sync":
            t0 = time.perf_counter()
            res = ck.sync(meta)
            journal("checkpoint-synced", "incremental", "%d dirty tiles" % res.dirty_tiles,
                    *_describe(res), "%.1f ms" % ((time.perf_counter() - t0) * 1e3))
        else:
            _tick_pending[id(ck)] = ck.save_async(meta)
    _tick_last = now
    _collect_finished()  # host tensors save synchronously: journal them now
    return True


def _handoff_safe() -> bool:
    """May the successor start while this process is still exiting?  Its teardown (unpinning
    the host region) takes ~1.4 s per 100 GB but holds this process's HBM until the end, so
    hand off early only when a second copy of the current HBM footprint fits next to it."""
    if os.environ.get("TPI_EARLY_HANDOFF", "1") in ("0", "false", "no"):
        return False
    torch = sys.modules.get("torch")
    if torch is None or not torch.cuda.is_initialized():
        return True
    try:
        for dev in range(torch.cuda.device_count()):
            free, total = torch.cuda.mem_get_info(dev)
            if total - free > free:
                return False
    except Exception:
        return False
    return True


_phase: Dict[str, float] = {}  # handler phase durations (s), for the journal


def _hbm_handoff() -> bool:
    """Export the tensors for a device-to-device hand-off (TPI_HBM_HANDOFF, default on)."""
    return os.environ.get("TPI_HBM_HANDOFF", "1") not in ("0", "false", "no")


def _stream_handoff() -> bool:
    """Release the successor when the spill *starts* (TPI_STREAM_HANDOFF, default on): it
    restores each chunk as it lands.  Needs one registered checkpointer, a supervisor to tell,
    and room for the successor's copy of the state next to ours (:func:`_handoff_safe`)."""
    if os.environ.get("TPI_STREAM_HANDOFF", "1") in ("0", "false", "no"):
        return False
    return len(_registered) == 1 and bool(os.environ.get("TPI_NOTIFY_FD")) and _handoff_safe()


def notify_released() -> bool:
    """Tell the supervisor the spill is complete (``TPI_NOTIFY_FD``), so it can respawn this
    rank now instead of after the exit; returns whether a notification was sent."""
    if not os.environ.get("TPI_NOTIFY_FD") or not _handoff_safe():
        return False
    return _notify(b"released\n")


def _notify(message: bytes) -> bool:
    fd = os.environ.get("TPI_NOTIFY_FD")
    if not fd:
        return False
    try:
        os.write(int(fd), message)
        return True
    except (OSError, ValueError):
        return False


def standby(prefetch_path: Optional[str] = None) -> bool:
    """Warm-standby point of a rank script: call it once the imports are done.

    In a normal incarnation it announces to the supervisor that this script can run as a warm
    standby and returns False at once.  When the rank is preempted, the supervisor then starts
    its successor immediately with ``TPI_STANDBY=1``: that process gets here (torch imported,
    GPU initialised) while the old rank is still spilling, starts mapping ``prefetch_path`` (the
    spill region, :func:`..host.prefetch`) and blocks until the supervisor activates it --
    right after the old rank has released -- then returns True and resumes from the spill.
    A standby that is not needed is killed (or sees EOF and exits quietly).
    """
    if os.environ.get("TPI_STANDBY") != "1":
        _notify(b"standby\n")
        return False
    cancel = threading.Event()
    torch = sys.modules.get("torch")
    if torch is not None and torch.cuda.is_initialized():
        # the successor's Checkpointer takes this engine instead of creating one (~0.1 s)
        from .checkpointer import prewarm_engine

        prewarm_engine(torch.cuda.current_device())
    if prefetch_path:
        from .host import prefetch, watch_prefetch

        if not prefetch(prefetch_path):
            # hot standby (started with the rank): the spill file appears later; map and pin
            # it then, long before a preemption
            watch_prefetch(prefetch_path, cancel)
    fd = int(os.environ.get("TPI_STANDBY_FD", "4"))
    while True:
        try:
            msg = os.read(fd, 16)
            break
        except InterruptedError:
            continue
    cancel.set()
    if not msg.startswith(b"go"):
        os._exit(0)  # discarded before activation
    os.close(fd)
    os.environ.pop("TPI_STANDBY", None)
    journal("standby-activated")
    _notify(b"standby\n")  # the activated process can itself be succeeded by a standby
    return True


def _linger() -> None:
    """After an early hand-off, stay alive (host region still pinned) until the supervisor
    says the successor restored (SIGUSR2) or ``TPI_LINGER_SECONDS`` (default 20) pass: the
    kernel's unpinning of a 100 GB region on exit (~1.4 s) would otherwise run during the
    successor's restore and halve its DMA rate (profiles/preempt_e2e_100g_round1.md)."""
    try:
        timeout = float(os.environ.get("TPI_LINGER_SECONDS", "20"))
    except ValueError:
        timeout = 20.0
    if timeout <= 0 or not hasattr(signal, "sigtimedwait"):
        return
    sys.stdout.flush()
    signal.pthread_sigmask(signal.SIG_BLOCK, [signal.SIGUSR2])
    got = signal.sigtimedwait([signal.SIGUSR2], timeout)
    journal("predecessor-exit", "successor restored" if got else "linger timeout")


def notify_restored() -> bool:
    """Tell the supervisor this incarnation restored its state (its predecessor may go)."""
    return _notify(b"restored\n")


def _handler(signum, frame):  # pragma: no cover - exercised in subprocess tests
    if _fired.is_set():
        return
    _fired.set()
    # The successor's "restored" reaches us as SIGUSR2 (see _linger).  With a streamed
    # hand-off it can arrive while this save is still finishing (final header, persist); its
    # default action would kill us mid-write, so it stays pending until _linger takes it.
    if hasattr(signal, "pthread_sigmask"):
        signal.pthread_sigmask(signal.SIG_BLOCK, [signal.SIGUSR2])
    journal("preempt-signal", "signal %d" % signum)
    t0 = time.perf_counter()
    released = []

    def stream_started():
        # the successor starts now and restores behind the spill (other PCIe direction);
        # journalled first, so the phase journal orders it before the supervisor's release
        if _stream_handoff():
            journal("checkpoint-streaming", "successor may start")
        if notify_released():
            released.append(True)

    try:
        t_safe = time.perf_counter()
        stream = stream_started if _stream_handoff() else None
        _phase["handoff-check"] = time.perf_counter() - t_safe
        rates = checkpoint_all({"reason": "preempted", "signal": signum}, on_stream=stream)
        print("tpi: preemption checkpoint saved in %.3fs (%s GB/s)" % (
            time.perf_counter() - t0, ", ".join("%.1f" % r for r in rates)), flush=True)
        code = PREEMPTED_EXIT_CODE
        if released or notify_released():
            if not released:
                journal("checkpoint-released", "successor may start")
            _linger()
        for ck in _registered:  # an HBM hand-off nobody took is stale once we exit
            manifest = ck._hbm_manifest_path()
            if manifest and os.path.exists(manifest):
                try:
                    os.remove(manifest)
                except OSError:
                    pass
    except Exception as error:
        print("tpi: preemption checkpoint FAILED: %s" % error, file=sys.stderr, flush=True)
        code = 1
    sys.stdout.flush()
    os._exit(code)


def install(signals=(signal.SIGTERM,)) -> None:
    global _installed
    for sig in signals:
        signal.signal(sig, _handler)
    _installed = True
    # The hand-off check's first device-memory query costs ~0.1 s on MI355X (measured in the
    # handler: signal -> HBM export 0.11 s); pay it now, not after the signal.
    _handoff_safe()


def resume(checkpointer: Checkpointer, persist_path: Optional[str] = None) -> Optional[Dict]:
    """Restore from the host region (or ``persist_path``) if a complete checkpoint exists.

    Returns the checkpoint metadata, or ``None`` for a fresh start -- only when there is no
    complete checkpoint anywhere.  A checkpoint that exists but fails verification (corrupt
    tiles) has already been partly unpacked into the tensors, so it never turns into a fresh
    start: the persisted copy is tried next, and if that fails too :class:`CheckpointError`
    is raised.
    """
    failure: Optional[CheckpointError] = None
    header = checkpointer.latest()  # complete, or still streaming in from the predecessor
    if header is not None and checkpointer.hbm_ready():
        try:  # the predecessor on this GPU is alive and exported its tensors: copy from HBM
            res = checkpointer.restore_hbm()
            journal("checkpoint-restored", "HBM hand-off", *_describe(res),
                    "ipc open %.3f s" % getattr(checkpointer, "hbm_open_s", 0.0),
                    "ipc close %.3f s" % getattr(checkpointer, "hbm_close_s", 0.0))
            notify_restored()
            return header.get("metadata", {})
        except Exception as error:  # fall back to the host region
            journal("checkpoint-hbm-failed", str(error))
    if header is not None:
        try:
            res = checkpointer.restore()
            journal("checkpoint-restored", "host region", *_describe(res))
            notify_restored()
            return header.get("metadata", {})
        except CheckpointError as error:
            failure = error
            journal("checkpoint-corrupt", "host region", str(error))
    if persist_path and os.path.exists(persist_path):
        try:
            res = checkpointer.load(persist_path)
        except CheckpointError as error:
            journal("checkpoint-corrupt", persist_path, str(error))
            raise CheckpointError("no usable checkpoint: host region: %s; %s: %s"
                                  % (failure or "none", persist_path, error)) from error
        journal("checkpoint-restored", persist_path, *_describe(res))
        notify_restored()
        return checkpointer.header().get("metadata", {})
    if failure is not None:
        raise CheckpointError("checkpoint failed verification and no persisted copy exists: %s"
                              % failure) from failure
    return None
