"""Device-memory gates and fatal device errors of the preemption hand-off (split out of
:mod:`.preemption`, which re-exports every name here).

* :func:`successor_need` / :func:`wait_for_device_memory`: the room a successor needs before
  it allocates its predecessor's state, and its wait for it by the driver's count as well as
  the runtime's (a predecessor offers its HBM only when that room exists next to it,
  ``preemption._handoff_safe``);
* :func:`_device_settled_for_handoff`: the HBM hand-off copy runs only on a device that is not
  over-committed;
* :func:`_sticky_device_error` / :func:`_hbm_fatal`: a sticky HIP error in the copy is fatal
  for the process -- the hand-off is withdrawn and the respawn restores from the host copy.

Why (the round-5/6 faults): ``profiles/round6/handoff_fault.md``.  Reference: a replacement
for a reclaimed spot VM is a fresh machine from the group's launch template
(``task/aws/resources/resource_auto_scaling_group.go:51-106``) and never inherits its
predecessor's memory; on one node the same GPU changes hands instead, and these gates (with
``parallel/placement.py`` ``settle_gpus`` for a task's start) stand in for that guarantee.
"""
from __future__ import annotations

import os
import sys
import time
from typing import Optional

from .checkpointer import Checkpointer

PREEMPTED_EXIT_CODE = 143  # 128 + SIGTERM (preemption.PREEMPTED_EXIT_CODE)


def _journal(code: str, *description: str) -> None:
    from .preemption import journal

    journal(code, *description)


SUCCESSOR_OVERHEAD = 2 << 30  # a successor's GPU context and checkpoint engine, still to come
PARKED_OVERHEAD = 256 << 20   # ... when it already holds them (a parked hot standby): the
#                               hand-off's descriptors and digests only


def successor_need(state_bytes: int, margin: float = 0.01,
                   overhead: int = SUCCESSOR_OVERHEAD) -> int:
    """Device memory a successor needs free before it allocates a state of ``state_bytes``:
    the state + ``margin`` (the caching allocator's rounding), + ``overhead`` for what it has
    not allocated yet -- its GPU context and engine (2 GiB), or, for a hot standby parked with
    both, ``PARKED_OVERHEAD`` (its memory is already in the device's count).  A 150 GB state
    next to a parked hot standby needs 151.8 GB free (the 2 GiB measure, 153.7 GB, sent it to the
    big-state path in ``profiles/round6/r6g``, ``r6h``: 153.2-153.7 GB were free)."""
    return int(state_bytes * (1 + margin)) + int(overhead)


def wait_for_device_memory(spill: str, margin: float = 0.01,
                           timeout: Optional[float] = None,
                           overhead: int = SUCCESSOR_OVERHEAD) -> Optional[float]:
    """A successor's gate before it allocates the state of ``spill`` (its predecessor's
    checkpoint region): block until the device has room for the state
    (:func:`successor_need`) by the *driver's* count as well as the HIP runtime's, or until
    ``timeout`` (``TPI_STREAM_TIMEOUT``, default 30 s).  Returns the seconds waited (None:
    nothing to wait for -- no state in ``spill``, or no GPU); every wait is journalled
    (``successor-hbm-wait``).

    * The predecessor still streams a state too big for two copies: it frees its tensors
      behind its spill (``Checkpointer.save(release_behind=True)``), and the restore streams
      behind the spill as room appears.
    * The predecessor is gone: its HBM is not back yet -- the driver wipes freed VRAM and
      releases it seconds after the exit, while the runtime already reports it free.
      Allocating on top of it made the driver evict buffers under the hand-off copy (the
      round-5 faults, ``profiles/round5/ipc_cause.md``), so the successor waits for that too.
    Called by ``preemption.standby`` before the script allocates its state."""
    from .checkpointer import region_total, streaming_writer

    torch = sys.modules.get("torch")
    if torch is None or not torch.cuda.is_available():
        return None
    peer = streaming_writer(spill)
    total = peer["total"] if peer is not None else region_total(spill)
    if not total:
        return None
    need = successor_need(total, margin, overhead)
    if timeout is None:
        timeout = float(os.environ.get("TPI_STREAM_TIMEOUT", "30"))
    dev = torch.cuda.current_device()
    from ..parallel.placement import device_vram_usage

    t0 = time.monotonic()
    free = driver_free = 0
    fits = declined = False
    while True:
        free, _ = torch.cuda.mem_get_info(dev)
        usage = device_vram_usage(dev)
        driver_free = free if usage is None else usage[1] - usage[0]
        fits = min(free, driver_free) >= need
        if fits or time.monotonic() - t0 >= timeout:
            break
        if peer is not None and streaming_writer(spill) is None:
            peer = None  # the spill is done: from now on only the driver's count matters
        if peer is None and not declined:
            # a predecessor that exported its HBM keeps it until a successor claims it: with
            # no room for our copy next to it, withdraw the offer so it exits now (restore
            # from the host copy) instead of both waiting out its linger
            from .handoff import decline_hbm_handoff

            declined = True
            if decline_hbm_handoff(spill):
                _journal("successor-hbm-declined", "%.1f GB needed" % (need / 1e9),
                         "free %.1f GB (driver %.1f GB)" % (free / 1e9, driver_free / 1e9))
        time.sleep(0.005)
    waited = time.monotonic() - t0
    _journal("successor-hbm-wait", "%.1f GB needed" % (need / 1e9), "waited %.3f s" % waited,
             "free %.1f GB (driver %.1f GB)" % (free / 1e9, driver_free / 1e9),
             "predecessor streaming" if peer is not None else "predecessor done",
             *([] if fits else ["timed out: allocating anyway"]))
    return waited


HANDOFF_HEADROOM = 1 << 30  # free device memory (driver's count) an HBM hand-off copy needs


def _device_settled_for_handoff(checkpointer: Checkpointer) -> bool:
    """May the HBM hand-off copy run now?  Only on a device that is not over-committed: the
    driver's count leaves ``HANDOFF_HEADROOM`` free and holds no more orphaned memory (exited
    processes, frees still being wiped) than a GPU carries idle.  Over-committed VRAM makes the
    driver evict buffers -- the predecessor's, which this process maps over HIP IPC, among
    them -- and the round-5/6 hand-off faults happened on such devices
    (``profiles/round6/handoff_fault.md``).  Waits up to ``TPI_HANDOFF_DRAIN_TIMEOUT``
    (default 10 s) for the drain; False sends the restore to the host copy.  The state seen is
    kept on the checkpointer (``hbm_device_state``: the fault dump's context) and journalled
    whenever it waited or refused."""
    from ..parallel.placement import ORPHAN_LIMIT, kfd_gpu_id, orphaned_vram
    import ctypes

    from ..ops import hip

    lib = hip(required=False)
    if lib is None:
        return True
    bus = ctypes.create_string_buffer(64)
    if lib.tpi_device_pci_bus_id(getattr(checkpointer, "device_index", 0) or 0, bus, 64) != 0:
        return True
    pci = bus.value.decode().lower()
    gid = kfd_gpu_id(pci)
    try:
        timeout = float(os.environ.get("TPI_HANDOFF_DRAIN_TIMEOUT", "10"))
    except ValueError:
        timeout = 10.0
    t0 = time.monotonic()
    while True:
        st = orphaned_vram(pci, gid)
        if st is None:
            return True
        checkpointer.hbm_device_state = dict(st, pci=pci)
        room = st["total"] - st["used"] >= HANDOFF_HEADROOM
        settled = st["orphaned"] is None or st["orphaned"] <= ORPHAN_LIMIT
        waited = time.monotonic() - t0
        if (room and settled) or waited >= timeout:
            break
        time.sleep(0.005)
    desc = ["VRAM in use %.1f of %.1f GB" % (st["used"] / 1e9, st["total"] / 1e9),
            "held by no process %s" % ("?" if st["orphaned"] is None else
                                       "%.1f GB" % (st["orphaned"] / 1e9)),
            "waited %.3f s" % waited]
    if not (room and settled):
        _journal("checkpoint-hbm-skipped", "device over-committed: restoring from the host copy",
                 *desc)
        return False
    if waited > 0.001:
        _journal("handoff-device-settled", *desc)
    return True


STICKY_HIP_ERRORS = ("illegal memory access", "illegal address", "illegal instruction",
                     "launch failure", "hardware exception", "memory access fault", "ecc error")


def _sticky_device_error(checkpointer: Checkpointer, error: BaseException) -> bool:
    """Did ``error`` leave this process's GPU context unusable?  A kernel fault is sticky in
    HIP: every later call on the device fails, so no restore -- from the host copy either --
    can run in this process any more (round 5, r5g: the "fallback" after a faulting hand-off
    copy died the same way).  Known messages, else one synchronisation probe."""
    text = str(error).lower()
    if any(word in text for word in STICKY_HIP_ERRORS):
        return True
    torch = sys.modules.get("torch")
    if torch is None or not torch.cuda.is_initialized():
        return False
    try:
        torch.cuda.synchronize(getattr(checkpointer, "device_index", None))
        return False
    except Exception as probe:
        return any(word in str(probe).lower() for word in STICKY_HIP_ERRORS) or \
            "hip" in str(probe).lower()


def _hbm_fatal(checkpointer: Checkpointer, error: BaseException) -> None:
    """A sticky device error during the HBM hand-off: fatal for this process.  The hand-off
    is withdrawn (manifest removed: the predecessor may exit, and no successor imports it
    again) and, under a supervisor, the rank exits as preempted -- its respawn is a new
    process with a new GPU context, which restores from the host copy.  Without a supervisor
    the caller re-raises."""
    _journal("checkpoint-hbm-fatal", str(error),
             "sticky device error: this process's GPU context is unusable, so there is no "
             "fallback in it", "dump %s" % getattr(checkpointer, "hbm_fault_dump", None),
             "the respawn restores from the host copy" if os.environ.get("TPI_NOTIFY_FD")
             else "no supervisor: raised to the script")
    try:
        os.remove(checkpointer._hbm_manifest_path())
    except (OSError, TypeError):
        pass
    checkpointer.release_hbm_claim()
    if not os.environ.get("TPI_NOTIFY_FD"):
        return
    print("tpi: FATAL: the HBM hand-off copy failed with a sticky device error (%s); exiting "
          "%d so the supervisor respawns this rank from the host copy" % (
              error, PREEMPTED_EXIT_CODE), file=sys.stderr, flush=True)
    os._exit(PREEMPTED_EXIT_CODE)
