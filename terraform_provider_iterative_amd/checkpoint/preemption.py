"""Preemption (SIGTERM) handling for rank processes.

The reference distinguishes preemption from completion on the VM: a machine that is
shutting down writes no status and gets respawned with the workdir restored from the bucket
(``machine-script.sh.tpl:10-15,51,89``).  Here the supervisor forwards SIGTERM to the ranks;
a rank that installed :func:`install` checkpoints its registered tensors to host memory (and
optionally the storage root) and exits with :data:`PREEMPTED_EXIT_CODE`, and its successor
calls :func:`resume` to restore them.

**Where the save happens.**  The reference leaves consistency to the user script, which
resumes from files it wrote at its own points (``README.md:88-101``).  A tensor checkpoint
taken at whatever bytecode a signal interrupts can be torn: weights already updated by
``opt.step()`` next to the old step counter, or half of AdamW's ``_foreach`` moment updates.
So the signal handler only *records* the request; the save runs at the next **step boundary**
-- :func:`step` (or :func:`tick`), called by the training loop where the registered tensors
are consistent -- and every rank of a job saves the same boundary (:mod:`.agreement`: one
shared cache line per rank, no per-step collective).

* The signal is seen even while the main thread is blocked in C (a collective, a device
  sync): CPython's C-level handler writes it to a wakeup pipe that a watcher thread reads
  (``signal.set_wakeup_fd``), so the request, its journal line and its deadline do not wait
  for the interpreter.
* A script that never calls :func:`step`/:func:`tick` keeps the old behaviour (save in the
  handler, journalled ``consistency signal``).
* A rank that reaches no boundary within ``TPI_PREEMPT_FALLBACK_SECONDS`` (default half of
  the supervisor's grace period ``TPI_GRACE_SECONDS``) is saved by the watcher thread anyway,
  journalled ``preempt-torn-risk`` and marked ``consistency torn-risk`` in the metadata, which
  :meth:`TrainingState.resume_consistent` refuses by default.
"""
from __future__ import annotations

import json
import logging
import os
import select
import signal
import sys
import threading
import time
from typing import Any, Callable, Dict, List, Optional, Tuple

from .checkpointer import Checkpointer, CheckpointError

log = logging.getLogger("tpi.preemption")

from .device_gates import (HANDOFF_HEADROOM, PARKED_OVERHEAD, PREEMPTED_EXIT_CODE,  # noqa: F401
                           STICKY_HIP_ERRORS, SUCCESSOR_OVERHEAD, _device_settled_for_handoff,
                           _hbm_fatal, _sticky_device_error, successor_need,
                           wait_for_device_memory)

_registered: List[Checkpointer] = []
_persist_paths: Dict[int, str] = {}
_callbacks: List[Callable[[], Optional[Dict]]] = []
_installed = False
_signals: tuple = (signal.SIGTERM,)

_requested = threading.Event()   # a preemption signal arrived
_fired = threading.Event()       # the preemption save started (at most one per process)
_usr2 = threading.Event()        # the successor restored: a lingering predecessor may exit
_save_lock = threading.Lock()
_note_lock = threading.Lock()
_signal_info: Dict[str, float] = {}
_boundary_seen = False           # the loop calls step()/tick(): saves wait for a boundary
_last_step: Optional[int] = None  # user step of the last boundary
_agreement = None
_wakeup_r: Optional[int] = None
_standby_script = False          # the script calls standby(spill): its successor waits for HBM


def register(checkpointer: Checkpointer, persist_path: Optional[str] = None) -> None:
    _registered.append(checkpointer)
    if persist_path:
        _persist_paths[id(checkpointer)] = persist_path


def on_preempt(callback: Callable[[], Optional[Dict]]) -> None:
    """Callback run before every save (preemption or periodic); may return metadata."""
    _callbacks.append(callback)


def preempted() -> bool:
    """A preemption was requested (the rank will save at its next step boundary)."""
    return _requested.is_set()


def saving() -> bool:
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


def _collect_metadata(base: Dict) -> Dict:
    meta = dict(base)
    for cb in _callbacks:
        extra = cb()
        if extra:
            meta.update(extra)
    return meta


def checkpoint_all(metadata: Optional[Dict] = None, on_stream=None,
                   exported: Optional[List[Checkpointer]] = None,
                   release_behind: bool = False) -> List[float]:
    """Save every registered checkpointer; returns per-checkpointer GB/s.  ``on_stream``
    (single checkpointer only): stream the save to the successor (see
    :meth:`Checkpointer.save`); called once the successor may start.  Checkpointers whose
    tensors were exported for an HBM hand-off are appended to ``exported``: their memory must
    stay allocated, and this process alive, until the successor is done with it."""
    t0 = time.perf_counter()
    meta = _collect_metadata({})
    meta.update(metadata or {})
    t_cb = time.perf_counter() - t0
    rates = []
    _phase["released-behind-bytes"] = 0
    for ck in _registered:
        if (on_stream is not None and len(_registered) == 1 and _hbm_handoff()
                and not release_behind):  # memory freed behind the spill is no hand-off
            try:  # the successor on this GPU copies our HBM while we spill to the host
                t1 = time.perf_counter()
                if ck.export_hbm(meta):
                    if exported is not None:
                        exported.append(ck)
                    journal("checkpoint-hbm-export", "successor may copy device to device",
                            "hand-off check %.3f s" % _phase.get("handoff-check", 0.0),
                            "callbacks %.3f s" % t_cb,
                            "export %.3f s" % (time.perf_counter() - t1))
            except Exception as error:  # the host path still works
                journal("checkpoint-hbm-export-failed", str(error))
        res = ck.save(meta, on_stream=on_stream if len(_registered) == 1 else None,
                      release_behind=release_behind)
        rates.append(res.gbps)
        journal("checkpoint-saved", *_describe(res))
        if getattr(res, "released_bytes", 0):
            _phase["released-behind-bytes"] += int(res.released_bytes)
            journal("device-memory-released", "%.1f GB behind the spill" % (
                res.released_bytes / 1e9))
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
_slots_warned = False


def sync_interval() -> float:
    """Seconds between periodic checkpoints (``TPI_SYNC_INTERVAL``, default 10 as in the
    reference; 0 or less disables the cadence)."""
    try:
        return float(os.environ.get("TPI_SYNC_INTERVAL", "10"))
    except ValueError:
        return 10.0


def sync_codec() -> Optional[str]:
    """Codec of the periodic background spills (``TPI_SYNC_CODEC``): ``none`` by default --
    a spill next to the training loop costs the loop ~6x less GPU time without the TPZ1
    encode kernels, and nothing waits for it (``profiles/async_codec_round3.md``); ``tpz1``
    shortens the spill instead; ``auto`` uses each checkpointer's own codec.  Preemption
    saves keep the checkpointer's codec: their spill is on the recovery path."""
    value = os.environ.get("TPI_SYNC_CODEC", "none").strip().lower()
    if value in ("none", "tpz1"):
        return value
    return None


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


def _periodic_save(step_no: Optional[int], metadata: Optional[Dict]) -> None:
    global _slots_warned
    meta = _collect_metadata({"reason": "periodic", "consistency": "boundary"})
    if step_no is not None:
        meta["step"] = step_no
    meta.update(metadata or {})
    mode = os.environ.get("TPI_SYNC_MODE", "async")
    codec = sync_codec()
    for ck in _registered:
        if len(ck.slots) == 1 and not _slots_warned:
            _slots_warned = True  # the spill overwrites the one copy: a crash mid-spill loses it
            journal("checkpoint-sync-warning", "slots=1: each periodic spill invalidates the "
                    "only copy while it runs; Checkpointer(slots=2) keeps the previous one")
        if mode == "sync":
            t0 = time.perf_counter()
            res = ck.sync(meta)
            journal("checkpoint-synced", "incremental", "%d dirty tiles" % res.dirty_tiles,
                    *_describe(res), "%.1f ms" % ((time.perf_counter() - t0) * 1e3))
        else:
            _tick_pending[id(ck)] = ck.save_async(meta, codec=codec)
    _collect_finished()  # host tensors save synchronously: journal them now


def step(step: Optional[int] = None, metadata: Optional[Dict] = None,
         force: bool = False) -> bool:
    """Step-boundary hook: call it where the registered tensors are consistent (after the
    optimizer step *and* the step counter update), at the same points on every rank.

    * A pending preemption is saved here -- on every rank at the same boundary -- and the
      process exits (this call does not return then).
    * Every :func:`sync_interval` seconds (rank 0's clock decides for the job) it takes a
      periodic checkpoint of every registered :class:`Checkpointer`, so a rank that dies
      without a SIGTERM (OOM, crash, SIGKILL after the grace period) still leaves a recent
      checkpoint behind.  ``force=True`` checkpoints now (every rank must pass it at the same
      boundary).

    ``step`` (the loop's own counter) is recorded in every save's metadata.  Returns True when
    this call took a periodic checkpoint.

    ``TPI_SYNC_MODE``:
      ``async`` (default)  HBM snapshot + background spill (:meth:`Checkpointer.save_async`):
                           the training stream stalls only for the snapshot, the PCIe leg
                           overlaps the next steps.  A tick that finds the previous spill still
                           running is skipped, never queued.
      ``sync``             incremental (:meth:`Checkpointer.sync`): only tiles whose device
                           digest changed since the last tick cross PCIe -- cheapest for mostly
                           frozen state (fine-tuning adapters, embeddings); blocks the caller.
    """
    global _boundary_seen, _last_step, _agreement, _tick_last
    _boundary_seen = True
    if step is not None:
        _last_step = step
    elif metadata and isinstance(metadata.get("step"), int):
        _last_step = metadata["step"]
    if _fired.is_set():  # a fallback save is running in the watcher: stop touching tensors
        threading.Event().wait()
    if _agreement is None:
        from . import agreement

        _agreement = agreement.create()
    now = time.monotonic()
    idle = _collect_finished()
    interval = sync_interval()
    due = False
    if _registered and _tick_last is None and not force:
        _tick_last = now  # the first call arms the timer
    elif _registered and (force or (interval > 0 and idle and now - _tick_last >= interval)):
        due = True
    shared = _agreement.kind == "shm"
    preempt_here, periodic_here = _agreement.arrive(_requested.is_set(),
                                                    due and not force)
    if preempt_here:
        _boundary_save()  # does not return
    if shared and _agreement.proposed:
        _tick_last = now  # rank 0 chose the next periodic boundary: the interval restarts
    if force or periodic_here:
        _periodic_save(_last_step, metadata)
        _tick_last = now
        return True
    return False


def tick(metadata: Optional[Dict] = None, force: bool = False) -> bool:
    """:func:`step` with the step number (if any) taken from ``metadata["step"]``."""
    return step(None, metadata, force)


def _handoff_safe() -> bool:
    """May the successor start while this process is still exiting?  Its teardown (unpinning
    the host region) takes ~1.4 s per 100 GB but holds this process's HBM until the end, so
    hand off early only when a second copy of the current HBM footprint fits next to it --
    by the successor's own measure (:func:`successor_need`, the room
    :func:`wait_for_device_memory` waits for) and the driver's count as well as the runtime's.
    A looser test here (footprint <= free) let a 150 GB state export its HBM that its
    successor then could not make room for: both waited for the other until the 20 s linger
    ran out (profiles/round6/r6f)."""
    if os.environ.get("TPI_EARLY_HANDOFF", "1") in ("0", "false", "no"):
        return False
    torch = sys.modules.get("torch")
    if torch is None or not torch.cuda.is_initialized():
        return True
    from ..parallel.placement import device_vram_usage

    try:
        states = _registered_state_bytes()
        # a hot standby parked with its context and engine: that memory is in the count already
        overhead = PARKED_OVERHEAD if _standby_parked() else SUCCESSOR_OVERHEAD
        for dev in range(torch.cuda.device_count()):
            free, total = torch.cuda.mem_get_info(dev)
            # the successor's copy is the registered state (a hot standby's own context is
            # already in use next to it); without a registered plan, all memory in use
            state = states.get(dev, 0) if states else total - free
            if not state:
                continue
            usage = device_vram_usage(dev)
            if usage is not None:
                free = min(free, usage[1] - usage[0])
            if free < successor_need(state, overhead=overhead):
                return False
    except Exception:
        return False
    return True


def _standby_marker(spill: str) -> str:
    return spill + ".standby"


def _mark_parked(spill: str) -> None:
    """A hot standby with its GPU context and engine made: say so next to the spill (its pid),
    so the predecessor counts its memory as already allocated (:func:`_handoff_safe`)."""
    path = _standby_marker(spill)
    tmp = "%s.%d.tmp" % (path, os.getpid())
    try:
        with open(tmp, "w") as handle:
            handle.write(str(os.getpid()))
        os.replace(tmp, path)
    except OSError:
        pass


def _unmark_parked(spill: str) -> None:
    path = _standby_marker(spill)
    try:
        with open(path) as handle:
            mine = handle.read().strip() == str(os.getpid())
        if mine:
            os.remove(path)
    except (OSError, ValueError):
        pass


def _standby_parked() -> bool:
    """Is a hot standby of a registered checkpointer's spill parked now (its marker names a
    live process other than this one)?"""
    from .base import _writer_alive

    for ck in _registered:
        spill = getattr(ck, "path", None)
        if not spill:
            continue
        try:
            with open(_standby_marker(spill)) as handle:
                pid = int(handle.read().strip() or 0)
        except (OSError, ValueError):
            continue
        if pid > 0 and pid != os.getpid() and _writer_alive(pid):
            return True
    return False


def _registered_state_bytes() -> Dict[int, int]:
    """Bytes of the registered checkpointers' states per device index ({} when none is
    bound yet)."""
    out: Dict[int, int] = {}
    for ck in _registered:
        plan = getattr(ck, "plan", None)
        total = getattr(plan, "total", None) if plan is not None else None
        if total:
            dev = int(getattr(ck, "device_index", 0) or 0)
            out[dev] = out.get(dev, 0) + int(total)
    return out


_phase: Dict[str, float] = {}  # handler phase durations (s), for the journal


def _hbm_handoff() -> bool:
    """Export the tensors for a device-to-device hand-off (TPI_HBM_HANDOFF, default on)."""
    return os.environ.get("TPI_HBM_HANDOFF", "1") not in ("0", "false", "no")


def _stream_handoff(safe: Optional[bool] = None) -> bool:
    """Release the successor when the spill *starts* (TPI_STREAM_HANDOFF, default on): it
    restores each chunk as it lands.  Needs one registered checkpointer, a supervisor to tell,
    and room for the successor's copy of the state next to ours (:func:`_handoff_safe`, or
    the caller's ``safe`` when it already asked)."""
    if os.environ.get("TPI_STREAM_HANDOFF", "1") in ("0", "false", "no"):
        return False
    if len(_registered) != 1 or not os.environ.get("TPI_NOTIFY_FD"):
        return False
    return _handoff_safe() if safe is None else safe


# The preemption save decides once whether a successor may run next to this process (one
# device-memory query); notify_released() then follows that decision instead of asking again
# (the answer can flip while the footprint sits near half of HBM).
_handoff_decision: Optional[bool] = None


def notify_released() -> bool:
    """Tell the supervisor the spill is complete (``TPI_NOTIFY_FD``), so it can respawn this
    rank now instead of after the exit; returns whether a notification was sent."""
    safe = _handoff_decision if _handoff_decision is not None else _handoff_safe()
    if not os.environ.get("TPI_NOTIFY_FD") or not safe:
        return False
    return _notify(b"released\n")


def requeue_requested() -> bool:
    """The supervisor is reclaiming this task for an on-demand one (``TPI_REQUEUE_FILE``
    exists): no successor will run on this GPU, so the save hands nothing off, frees the HBM
    and the process leaves right after it."""
    path = os.environ.get("TPI_REQUEUE_FILE")
    return bool(path) and os.path.exists(path)


def _notify(message: bytes) -> bool:
    fd = os.environ.get("TPI_NOTIFY_FD")
    if not fd:
        return False
    try:
        os.write(int(fd), message)
        return True
    except (OSError, ValueError):
        return False


def standby(prefetch_path: Optional[str] = None, materialize: bool = False) -> bool:
    """Warm-standby point of a rank script: call it once the imports are done.

    In a normal incarnation it announces to the supervisor that this script can run as a warm
    standby and returns False at once.  When the rank is preempted, the supervisor then starts
    its successor immediately with ``TPI_STANDBY=1``: that process gets here (torch imported,
    GPU initialised) while the old rank is still spilling, starts mapping ``prefetch_path`` (the
    spill region, :func:`..host.prefetch`) and blocks until the supervisor activates it --
    right after the old rank has released -- then returns True and resumes from the spill.
    A standby that is not needed is killed (or sees EOF and exits quietly).

    ``materialize``: the script restores with :func:`materialize` (the state is allocated
    group by group as the predecessor frees it), so nothing waits here for room for the whole
    state (:func:`wait_for_device_memory`).
    """
    global _standby_script
    _standby_script = bool(prefetch_path)
    wait_memory = bool(prefetch_path) and not materialize
    if os.environ.get("TPI_STANDBY") != "1":
        _notify(b"standby\n")
        if wait_memory:  # a cold successor of a big-state predecessor
            wait_for_device_memory(prefetch_path)
        return False
    cancel = threading.Event()
    torch = sys.modules.get("torch")
    if torch is not None and torch.cuda.is_initialized():
        # the successor's Checkpointer takes this engine instead of creating one (~0.1 s)
        from .checkpointer import prewarm_engine

        prewarm_engine(torch.cuda.current_device())
        if prefetch_path:
            _mark_parked(prefetch_path)
    if prefetch_path:
        from .host import prefetch, wait_pinned, watch_prefetch

        if not prefetch(prefetch_path):
            # hot standby (started with the rank): the spill file appears later; map and pin
            # it then, long before a preemption
            watch_prefetch(prefetch_path, cancel)

        def pinned():  # journal when the whole spill is pinned: from then on a restore
            # never waits for a window (bench/bench_preempt.py waits for this)
            t0 = time.monotonic()
            while not cancel.is_set():
                took = wait_pinned(prefetch_path, cancel=cancel)
                if took is not None:
                    journal("standby-pinned", "%.1f GB" % (os.path.getsize(prefetch_path) / 1e9),
                            "%.3f s after standby()" % (time.monotonic() - t0))
                    return
                cancel.wait(0.05)

        threading.Thread(target=pinned, name="tpi-standby-pinned", daemon=True).start()
    fd = int(os.environ.get("TPI_STANDBY_FD", "4"))
    while True:
        try:
            msg = os.read(fd, 64)
            break
        except InterruptedError:
            continue
    cancel.set()
    if prefetch_path:  # parked no more: activated (the offer was decided) or discarded
        _unmark_parked(prefetch_path)
    if not msg.startswith(b"go"):
        os._exit(0)  # discarded before activation
    os.close(fd)
    for word in msg.split():  # "go port=N": this incarnation's rendezvous port
        if word.startswith(b"port="):
            os.environ["MASTER_PORT"] = word[5:].decode()
    os.environ.pop("TPI_STANDBY", None)
    journal("standby-activated")
    if wait_memory:
        # parked with a context and engine: only the state (and descriptors) are still to come
        parked = torch is not None and torch.cuda.is_initialized()
        wait_for_device_memory(prefetch_path,
                               overhead=PARKED_OVERHEAD if parked else SUCCESSOR_OVERHEAD)
    _notify(b"standby\n")  # the activated process can itself be succeeded by a standby
    return True


def _linger() -> None:
    """After an early hand-off, stay alive (host region still pinned) until the supervisor
    says the successor restored (SIGUSR2, seen through :data:`_usr2`) or
    ``TPI_LINGER_SECONDS`` (default 20) pass: the kernel's unpinning of a 100 GB region on exit
    (~1.4 s) would otherwise run during the successor's restore and halve its DMA rate
    (profiles/preempt_e2e_100g_round1.md)."""
    try:
        timeout = float(os.environ.get("TPI_LINGER_SECONDS", "20"))
    except ValueError:
        timeout = 20.0
    if timeout <= 0:
        return
    sys.stdout.flush()
    got = _usr2.wait(timeout)
    journal("predecessor-exit", "successor restored" if got else "linger timeout")


def _await_successor(ck: Checkpointer) -> str:
    """After exporting ``ck``'s tensors for an HBM hand-off: return only once no successor
    can still be reading them (:meth:`Checkpointer.claim_hbm` protocol) -- a successor that
    claimed them closed its mappings (claim and manifest gone) or died, or nobody claimed them
    and this process withdrew the offer by claiming them itself, which it does on SIGUSR2
    (the supervisor: the successor restored elsewhere / closed / died) or after
    ``TPI_LINGER_SECONDS``.  A live claimer is waited for up to ``TPI_HANDOFF_CLOSE_TIMEOUT``
    (default 600 s).  Returns how it ended (journalled)."""
    try:
        soft = float(os.environ.get("TPI_LINGER_SECONDS", "20"))
    except ValueError:
        soft = 20.0
    try:
        hard = float(os.environ.get("TPI_HANDOFF_CLOSE_TIMEOUT", "600"))
    except ValueError:
        hard = 600.0
    from .checkpointer import _writer_alive

    sys.stdout.flush()
    t0 = time.monotonic()
    me = os.getpid()
    manifest = ck._hbm_manifest_path()
    while True:
        owner = ck.hbm_claim_owner()
        waited = time.monotonic() - t0
        if owner == me:
            how = "withdrawn"
        elif owner is None:
            if manifest and not os.path.exists(manifest):
                how = "successor closed"  # claimed, copied, unmapped, claim dropped
            elif (_usr2.is_set() or waited >= max(soft, 0.0)) and ck.claim_hbm():
                how = "withdrawn"
            else:
                how = None
        elif owner == 0:  # a claim without a pid: taken for a live claimer, never a dead one
            how = ("timeout with an unreadable claim" if waited >= hard else None)
        elif not _writer_alive(owner):
            how = "successor died"
        elif waited >= hard:
            how = "timeout with the hand-off still mapped by pid %d" % owner
        else:
            how = None
        if how is not None:
            journal("predecessor-exit", how, "waited %.3f s" % waited)
            return how
        _usr2.wait(0.005)
        if _usr2.is_set() and owner not in (None, me):
            time.sleep(0.005)  # a live claimer: SIGUSR2 alone is no reason to go


def notify_restored(hbm: bool = False) -> bool:
    """Tell the supervisor this incarnation restored its state.  From the host region its
    predecessor may go now; from the predecessor's HBM (``hbm``) only after :func:`notify_closed`."""
    return _notify(b"restored hbm\n" if hbm else b"restored\n")


def notify_closed() -> bool:
    """The predecessor's exported HBM is no longer mapped here: it may exit."""
    return _notify(b"closed\n")


def fallback_seconds() -> float:
    """How long a requested preemption waits for a step boundary before the watcher saves
    anyway (``TPI_PREEMPT_FALLBACK_SECONDS``; default half of ``TPI_GRACE_SECONDS``, the
    supervisor's SIGTERM -> SIGKILL window, itself 30 s by default)."""
    try:
        return float(os.environ["TPI_PREEMPT_FALLBACK_SECONDS"])
    except (KeyError, ValueError):
        pass
    try:
        grace = float(os.environ.get("TPI_GRACE_SECONDS", "30"))
    except ValueError:
        grace = 30.0
    return max(0.5 * grace, 0.1)


def _boundary_mode() -> bool:
    """Does a preemption wait for the next step boundary?  ``TPI_PREEMPT_AT``: ``auto``
    (default: yes once the loop has called :func:`step`/:func:`tick`), ``boundary`` (always),
    ``signal`` (never: save in the handler, the pre-boundary behaviour)."""
    at = os.environ.get("TPI_PREEMPT_AT", "auto")
    if at == "signal":
        return False
    return at == "boundary" or _boundary_seen


def _note_signal(signum: int) -> bool:
    """Record a preemption request once (handler or watcher, whichever runs first)."""
    with _note_lock:
        if _requested.is_set():
            return False
        _signal_info["signum"] = signum
        _signal_info["time"] = time.time()
        _signal_info["mono"] = time.monotonic()
        _requested.set()
    journal("preempt-signal", "signal %d" % signum,
            "save at the next step boundary" if _boundary_mode() else "save now (no step hook)")
    return True


def _save_and_exit(consistency: str, ordinal: Optional[int] = None) -> None:
    """Run the preemption save once and exit; returns only if another thread is saving.

    * preemption (a successor follows on this GPU): stream the spill to it, export the HBM
      for a device-to-device copy when both copies fit, and stay until the successor no
      longer needs this process (:func:`_await_successor` / :func:`_linger`);
    * reclaim (:func:`requeue_requested`: an on-demand task takes the GPU): plain save, free
      the HBM, ``released`` -- the supervisor hands the GPU over at once -- and leave;
    * a failed spill after an HBM export still waits for the successor: its device copy is
      then the only good one.
    """
    global _handoff_decision
    if not _save_lock.acquire(blocking=False):
        return
    _fired.set()
    signum = int(_signal_info.get("signum", signal.SIGTERM))
    t0 = time.perf_counter()
    released: List[bool] = []
    exported: List[Checkpointer] = []
    requeue = requeue_requested()
    t_safe = time.perf_counter()
    _handoff_decision = safe = _handoff_safe()  # evaluated once: one device-memory query
    stream_ok = not requeue and _stream_handoff(safe)
    # too big for two copies, but the successor waits for room (standby(spill)): stream to
    # it anyway and free each tensor's HBM behind the spill -- its allocation and restore
    # then run under our spill instead of after it
    big_stream = (not requeue and not safe and consistency == "boundary" and _standby_script
                  and _release_hbm_enabled() and _stream_handoff(True)
                  and os.environ.get("TPI_BIG_STREAM", "1") not in ("0", "false", "no"))
    _phase["handoff-check"] = time.perf_counter() - t_safe

    def stream_started():
        # the successor starts now and restores behind the spill (other PCIe direction);
        # journalled first, so the phase journal orders it before the supervisor's release
        journal("checkpoint-streaming", "successor may start" if not big_stream else
                "successor may start; it waits for the HBM freed behind the spill")
        if (_notify(b"released\n") if big_stream else notify_released()):
            released.append(True)

    meta = {"reason": "requeued" if requeue else "preempted", "signal": signum,
            "consistency": consistency}
    if _last_step is not None:
        meta["step"] = _last_step
    if ordinal is not None:
        meta["boundary"] = ordinal
    code = 1
    # may _teardown free the HBM explicitly?  At a boundary, yes.  From a signal-time save on
    # the main thread only when no process group exists: the script is mid-step there, and a
    # collective whose peer is already gone would block hipFree until SIGKILL.
    at_boundary = consistency == "boundary" or (
        consistency == "signal" and threading.current_thread() is threading.main_thread()
        and not _process_group_active())
    # a reclaim, or a state too big for a successor's copy next to ours: every tensor's HBM
    # goes back as soon as it is in host memory, so the driver clears it under the spill
    release_behind = (consistency == "boundary" and _release_hbm_enabled() and not stream_ok
                      and (requeue or not safe))
    try:
        rates = checkpoint_all(meta, on_stream=stream_started if (stream_ok or big_stream)
                               else None, exported=exported, release_behind=release_behind)
        print("tpi: preemption checkpoint saved in %.3fs (%s GB/s)" % (
            time.perf_counter() - t0, ", ".join("%.1f" % r for r in rates)), flush=True)
        code = PREEMPTED_EXIT_CODE
        freed = 0
        if (not released and not exported and consistency == "boundary"
                and _release_hbm_enabled() and (requeue or not safe)):
            # a reclaim, or a state too big for two copies in HBM: the next process on this
            # GPU could only allocate after our exit (and the kernel's unpinning of our region,
            # ~1.4 s per 100 GB).  Free our HBM now instead -- we are at a step boundary on
            # the main thread, nothing will touch the tensors again, nobody imported them --
            # and hand off while the host region stays pinned.
            t1 = time.perf_counter()
            freed = _release_device_memory()
            journal("device-memory-released", "%.1f GB" % (freed / 1e9),
                    "%.3f s" % (time.perf_counter() - t1))
        # release_behind: the save itself already gave the tensors' HBM back (freed above
        # measures ~0 then), so the GPU may go just the same
        freed += int(_phase.get("released-behind-bytes", 0))
        if (not released and (safe or freed)
                and os.environ.get("TPI_NOTIFY_FD")):
            # journalled first, so the phase journal orders it before the supervisor's
            # rank-released (which the notification triggers)
            journal("checkpoint-released", "reclaim: the GPU may go" if requeue
                    else "successor may start")
            if _notify(b"released\n"):
                released.append(True)
            else:
                journal("checkpoint-release-failed", "the supervisor's notify pipe is gone")
        if released and not requeue:
            if exported:
                _await_successor(exported[0])
            else:
                _linger()
    except Exception as error:
        print("tpi: preemption checkpoint FAILED: %s" % error, file=sys.stderr, flush=True)
        journal("checkpoint-failed", str(error))
        if exported:  # a successor may be copying our HBM: now the only good copy
            _await_successor(exported[0])
    _withdraw_handoffs()
    sys.stdout.flush()
    _teardown(code, at_boundary)


def _process_group_active() -> bool:
    """A torch.distributed process group is initialised in this process (never imports
    torch.distributed itself)."""
    dist = sys.modules.get("torch.distributed")
    try:
        return bool(dist is not None and dist.is_available() and dist.is_initialized())
    except Exception:
        return True  # unknown: the conservative answer


def _withdraw_handoffs() -> None:
    """An HBM hand-off nobody took is stale once we exit: claim it (no successor can start
    importing now), then remove the manifest and the claim."""
    for ck in _registered:
        manifest = ck._hbm_manifest_path()
        if not manifest:
            continue
        owner = ck.hbm_claim_owner()
        if owner not in (None, os.getpid()):
            continue  # a successor's (alive: timeout) -- it removes it after closing
        if os.path.exists(manifest) and not ck.claim_hbm():
            continue
        for path in (manifest, ck._hbm_claim_path()):
            try:
                os.remove(path)
            except OSError:
                pass


def _teardown(code: int, release_device: bool = True) -> None:
    """Give back this process's HBM explicitly (timed in the journal: ``predecessor-teardown``)
    and ``os._exit``; the kernel's own teardown of the address space and GPU context that
    follows shows in the supervisor's ``exit-trace`` events.  ``release_device`` only when no
    other thread may still run device work on the tensors (a boundary save on the main thread).

    ``TPI_EXPLICIT_TEARDOWN``: ``hbm`` (default) frees the device memory and leaves the pinned
    host region to the kernel; ``full`` also unregisters and unmaps the region first; ``0``
    goes straight to ``os._exit``.  Measured on MI355X with a 100 GB region
    (profiles/round4/teardown.md): unmapping it explicitly after a hot hand-off takes ~11 s
    (the munmap keeps invalidating the live GPU context's user-pointer mappings), the kernel's
    exit-time teardown ~1.3 s; freeing 100 GB of HBM first costs 0.07 s and hands it to the
    next process on the GPU at once."""
    mode = os.environ.get("TPI_EXPLICIT_TEARDOWN", "hbm").strip().lower()
    if mode in ("0", "false", "no", "off"):
        os._exit(code)
    phases = []
    try:
        t0 = time.perf_counter()
        if release_device:
            freed = _release_device_memory()
            if freed:
                phases.append("hbm %.1f GB %.3f s" % (freed / 1e9, time.perf_counter() - t0))
        for ck in _registered if mode in ("full", "1", "true", "yes") else ():
            region = getattr(ck, "region", None)
            if region is None or not getattr(region, "registered", False):
                continue
            split: Dict[str, float] = {}
            region.close(split)  # unregister (unpin) + unmap; a /dev/shm file keeps its pages
            phases.append("host region %.1f GB: unregister %.3f s, unmap %.3f s" % (
                region.size / 1e9, split.get("unregister", 0.0), split.get("unmap", 0.0)))
        if phases:
            journal("predecessor-teardown", *phases)
    except Exception as error:  # never keep a preempted process alive over its teardown
        journal("predecessor-teardown-failed", str(error))
    try:
        sys.stdout.flush()
    except Exception:  # nobody reads our output any more (e.g. a killed supervisor)
        pass
    os._exit(code)


def _release_hbm_enabled() -> bool:
    return os.environ.get("TPI_RELEASE_HBM", "1") not in ("0", "false", "no")


def _release_device_memory() -> int:
    """Free (almost) all of this process's HBM after its preemption save: the registered
    checkpointers' engines and tensors, then every other CUDA tensor still alive (gradients,
    activations kept for the next step, communication buckets), then the caching allocator's
    cache.  Only from the boundary save on the main thread: the process is about to exit and
    nothing queued or running uses the tensors (the device is synchronized first).  Returns
    the reserved bytes given back."""
    torch = sys.modules.get("torch")
    if torch is None or not torch.cuda.is_initialized():
        return 0
    import gc

    devices = range(torch.cuda.device_count())
    torch.cuda.synchronize()
    before = sum(torch.cuda.memory_reserved(d) for d in devices)
    for ck in _registered:
        try:
            ck.release_device()
        except Exception as error:  # keep going: the rest still frees memory
            journal("device-memory-release-failed", str(error))
    import warnings

    with warnings.catch_warnings():  # isinstance() on lazy module objects can warn
        warnings.simplefilter("ignore")
        for obj in gc.get_objects():
            try:
                if isinstance(obj, torch.Tensor) and obj.is_cuda:
                    obj.untyped_storage().resize_(0)
            except Exception:
                continue
    torch.cuda.empty_cache()
    return max(0, before - sum(torch.cuda.memory_reserved(d) for d in devices))


def _boundary_save() -> None:
    ordinal = getattr(_agreement, "ordinal", None)
    waited = time.monotonic() - _signal_info.get("mono", time.monotonic())
    desc = ["boundary %s" % ordinal, "waited %.3f s" % waited]
    if _last_step is not None:
        desc.insert(1, "step %d" % _last_step)
    journal("preempt-boundary", *desc)
    _save_and_exit("boundary", ordinal)
    threading.Event().wait()  # the watcher's fallback save owns the process now


def _on_signal(signum, frame):  # pragma: no cover - exercised in subprocess tests
    _note_signal(signum)
    if not _boundary_mode() and not _fired.is_set():
        _save_and_exit("signal")  # no step hook in this script: save where it stands


def _on_usr2(signum, frame):  # pragma: no cover - exercised in subprocess tests
    _usr2.set()


def _watch(rfd: int) -> None:
    """Watcher thread: sees signals through the wakeup pipe even while the main thread is
    blocked in C, and saves anyway when no step boundary comes in time."""
    preempt_signals = {int(s) for s in _signals}
    while True:
        timeout = None
        if _requested.is_set() and not _fired.is_set():
            timeout = max(0.0, _signal_info["mono"] + fallback_seconds() - time.monotonic())
        try:
            ready, _, _ = select.select([rfd], [], [], timeout)
        except InterruptedError:
            continue
        if not ready:
            if _fired.is_set():
                continue
            journal("preempt-torn-risk", "no step boundary within %.1f s" % fallback_seconds(),
                    "last step %s" % _last_step)
            _save_and_exit("torn-risk" if _boundary_mode() else "signal")
            continue
        try:
            data = os.read(rfd, 64)
        except (BlockingIOError, InterruptedError):
            continue
        if not data:
            return
        for signum in data:
            if signum == signal.SIGUSR2:
                _usr2.set()
            elif signum in preempt_signals:
                _note_signal(signum)


def install(signals=(signal.SIGTERM,)) -> None:
    """Arm preemption handling (call from the main thread).  SIGTERM records a request (saved
    at the next :func:`step`, or at once in a script that never calls it); SIGUSR2 from the
    supervisor lets a lingering predecessor exit."""
    global _installed, _signals, _wakeup_r
    _signals = tuple(signals)
    for sig in signals:
        signal.signal(sig, _on_signal)
    signal.signal(signal.SIGUSR2, _on_usr2)
    if _wakeup_r is None:
        r, w = os.pipe()
        os.set_blocking(w, False)
        try:
            signal.set_wakeup_fd(w, warn_on_full_buffer=False)
        except ValueError:  # not the main thread: the Python handlers still work
            os.close(r)
            os.close(w)
        else:
            _wakeup_r = r
            threading.Thread(target=_watch, args=(r,), name="tpi-preempt-watch",
                             daemon=True).start()
    _installed = True
    # The hand-off check's first device-memory query costs ~0.1 s on MI355X (measured in the
    # handler: signal -> HBM export 0.11 s); pay it now, not after the signal.
    _handoff_safe()


def _persisted(path: str) -> bool:
    """A persisted checkpoint exists at ``path`` (a local file, or one in an off-node
    ``storage.container``)."""
    from ..storage import remote

    if remote.is_remote(path):
        try:
            return remote.file_exists(path)
        except (OSError, ValueError):
            return False
    return os.path.exists(path)


def materialize(spill: str, device: Any = None, **kwargs) -> Optional[Tuple[Checkpointer,
                                                                          Dict[str, Any], Dict]]:
    """Successor side of a big-state hand-off: create and restore the tensors of the spill
    region ``spill`` group by group (:meth:`Checkpointer.materialize`), behind the
    predecessor's streamed save while it runs, each group allocated as soon as the
    predecessor's freed HBM has room for it.  Returns ``(checkpointer, tensors, metadata)``,
    or None when ``spill`` holds no checkpoint (a fresh start: allocate as usual).  The
    script builds its model around the tensors (e.g. on the ``meta`` device, then
    :func:`..training.assign_materialized`) instead of allocating it first; call
    :func:`standby` with ``materialize=True``."""
    if not spill or not os.path.exists(spill) or os.path.getsize(spill) == 0:
        return None
    try:
        ck, tensors, res = Checkpointer.materialize(spill, device, **kwargs)
    except CheckpointError as error:
        if "no checkpoint" in str(error):
            return None
        journal("checkpoint-corrupt", "host region (materialize)", str(error))
        raise
    stats = getattr(ck, "materialize_stats", {})
    journal("checkpoint-restored", "host region, materialized in %d groups" % stats.get("groups", 0),
            *_describe(res), "allocation waits %.3f s" % stats.get("alloc_wait_s", 0.0),
            "streamed" if stats.get("streamed") else "complete copy")
    notify_restored()
    return ck, tensors, dict(getattr(ck, "materialized_metadata", {}) or {})


def resume(checkpointer: Checkpointer, persist_path: Optional[str] = None,
           generation: Optional[int] = None) -> Optional[Dict]:
    """Restore from the host region (or ``persist_path``) if a complete checkpoint exists.

    Returns the checkpoint metadata, or ``None`` for a fresh start -- only when there is no
    complete checkpoint anywhere.  A checkpoint that exists but fails verification (corrupt
    tiles) has already been partly unpacked into the tensors, so it never turns into a fresh
    start: the persisted copy is tried next, and if that fails too :class:`CheckpointError`
    is raised.  ``generation``: restore that copy of the region (see
    :meth:`Checkpointer.candidates`) rather than the newest.
    """
    failure: Optional[CheckpointError] = None
    header = checkpointer.latest()  # complete, or still streaming in from the predecessor
    if generation is not None:
        header = next(({"generation": c["generation"], "metadata": c["metadata"]}
                       for c in checkpointer.candidates() if c["generation"] == generation),
                      None)
        if header is None:
            raise CheckpointError("no checkpoint of generation %d in the region" % generation)
    meta = (header or {}).get("metadata", {})
    if meta.get("consistency") in ("torn-risk", "signal"):
        journal("checkpoint-torn-risk", "restoring a save taken at %s" % meta["consistency"],
                "step %s" % meta.get("step"))
    # The HBM copy is the state of the predecessor's last save (its boundary): the newest
    # state there is -- newer than a host copy whose spill failed, present even when none
    # completed.  A caller that asks for a specific generation (resume_consistent: the copy the
    # gang agreed on) gets the HBM only when it is that generation.
    hbm = checkpointer.hbm_metadata()
    if hbm is not None and generation is not None and hbm["generation"] != generation:
        hbm = None
    if hbm is not None and not _device_settled_for_handoff(checkpointer):
        hbm = None  # over-committed device: its buffers may move under the copy -- host route
    if hbm is not None:
        try:  # the predecessor on this GPU is alive and exported its tensors: copy from HBM
            res = checkpointer.restore_hbm()
            journal("checkpoint-restored", "HBM hand-off", *_describe(res),
                    "ipc open %.3f s" % getattr(checkpointer, "hbm_open_s", 0.0),
                    "kernels %.4f s" % res.device_seconds,
                    "steps " + " ".join("%s %.4f" % kv for kv in
                                        getattr(checkpointer, "hbm_phases", {}).items()),
                    "%.1f GB free at the copy" % (
                        getattr(checkpointer, "hbm_free_before_copy", 0) / 1e9))
            notify_restored(hbm=True)

            def behind():  # after "restored": the unmapping, then the host copy's durability
                checkpointer.wait_hbm_close()
                journal("hbm-handoff-closed",
                        "ipc close %.3f s" % getattr(checkpointer, "hbm_close_s", 0.0))
                notify_closed()  # the predecessor may exit now
                t0 = time.perf_counter()
                done = checkpointer.wait_stream(timeout=float(os.environ.get(
                    "TPI_DURABLE_TIMEOUT", "600")))
                if done is None:  # no spill running (any more): is the restored copy there?
                    if checkpointer.durable(hbm["generation"] or
                                            (header or {}).get("generation") or 0):
                        done = True
                    elif not checkpointer.closing:
                        done = False
                if done is False:  # resumed from HBM, but the predecessor's spill failed
                    journal("checkpoint-not-durable", "the predecessor's host copy failed; "
                            "no host checkpoint until this rank saves")
                    print("tpi: WARNING: resumed from the predecessor's HBM, but its host "
                          "spill failed: no durable checkpoint until the next save",
                          file=sys.stderr, flush=True)
                elif done is None and checkpointer.closing:
                    journal("checkpoint-durability-unknown", "the checkpointer was closed "
                            "before the predecessor's host copy finished")
                else:
                    journal("checkpoint-durable", "host copy complete %.3f s after restore"
                            % (time.perf_counter() - t0))

            checkpointer.watch(behind, "tpi-handoff-durability")
            # the exported state is the predecessor's last boundary: newer than a host copy
            # whose spill failed, and there even when no host copy completed at all
            return hbm["metadata"] or (header or {}).get("metadata", {})
        except Exception as error:  # fall back to the host region -- unless the GPU is gone
            if _sticky_device_error(checkpointer, error):
                _hbm_fatal(checkpointer, error)  # does not return under a supervisor
                raise
            journal("checkpoint-hbm-failed", str(error), "%.1f GB free at the copy" % (
                getattr(checkpointer, "hbm_free_before_copy", 0) / 1e9))
    if header is not None:
        try:
            res = checkpointer.restore(generation=generation)
            journal("checkpoint-restored", "host region", *_describe(res))
            notify_restored()
            return header.get("metadata", {})
        except CheckpointError as error:
            failure = error
            journal("checkpoint-corrupt", "host region", str(error))
    if persist_path and _persisted(persist_path):
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
