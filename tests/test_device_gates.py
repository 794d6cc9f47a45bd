"""Device-memory and IPC gates of the recovery path, on CPU with fakes of the driver calls
(ADVICE r5):

* the successor's allocation gate (``preemption.wait_for_device_memory``) waits for the
  driver's count as well as the runtime's, also after its predecessor has exited;
* a sticky device error in the HBM hand-off is fatal for the process: the hand-off is
  withdrawn and, under a supervisor, the rank exits as preempted so that its respawn (a new
  GPU context) restores from the host copy;
* the staged-workdir attach is bounded (``TPI_IPC_OPEN_TIMEOUT``) and journalled.
"""
import json
import os
import subprocess
import sys
import textwrap
import threading
import time
import types

import pytest

from terraform_provider_iterative_amd.checkpoint import preemption
from terraform_provider_iterative_amd.runtime import stage

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GB = 10 ** 9


class FakeCuda:
    def __init__(self, free):
        self.free = free

    def is_available(self):
        return True

    def is_initialized(self):
        return True

    def current_device(self):
        return 0

    def mem_get_info(self, dev):
        return self.free, 288 * GB


def _events(path):
    with open(path) as f:
        return [json.loads(line) for line in f]


def test_successor_waits_for_the_drivers_count_after_the_predecessor_exited(
        tmp_path, monkeypatch):
    from terraform_provider_iterative_amd.checkpoint import checkpointer as ckmod
    from terraform_provider_iterative_amd.parallel import placement

    events = tmp_path / "events.jsonl"
    monkeypatch.setenv("TPI_EVENTS_FILE", str(events))
    # the runtime already reports the exited predecessor's 190 GB free; the driver does not
    fake = types.SimpleNamespace(cuda=FakeCuda(270 * GB))
    monkeypatch.setitem(sys.modules, "torch", fake)
    monkeypatch.setattr(ckmod, "streaming_writer", lambda path: None)  # predecessor gone
    monkeypatch.setattr(ckmod, "region_total", lambda path: 100 * GB)
    used = {"v": 200 * GB}
    monkeypatch.setattr(placement, "device_vram_usage", lambda dev: (used["v"], 288 * GB))
    timer = threading.Timer(0.4, lambda: used.update(v=10 * GB))
    timer.start()
    waited = preemption.wait_for_device_memory(str(tmp_path / "spill"), timeout=10)
    timer.join()
    assert 0.3 < waited < 5
    rec = [e for e in _events(events) if e["code"] == "successor-hbm-wait"][-1]
    assert "predecessor done" in rec["description"] and not any(
        "timed out" in d for d in rec["description"])
    # bounded: a count that never comes back costs the timeout, then the allocation goes on
    used["v"] = 250 * GB
    t0 = time.monotonic()
    preemption.wait_for_device_memory(str(tmp_path / "spill"), timeout=0.3)
    assert time.monotonic() - t0 < 2
    rec = [e for e in _events(events) if e["code"] == "successor-hbm-wait"][-1]
    assert any("timed out" in d for d in rec["description"])
    # no state in the region: nothing to wait for
    monkeypatch.setattr(ckmod, "region_total", lambda path: None)
    assert preemption.wait_for_device_memory(str(tmp_path / "spill"), timeout=5) is None


def test_sticky_device_errors_are_recognised():
    ck = types.SimpleNamespace(device_index=0)
    assert preemption._sticky_device_error(
        ck, RuntimeError("tpi_copy_segments failed: hipStreamSynchronize: an illegal memory "
                         "access was encountered"))
    assert not preemption._sticky_device_error(
        ck, RuntimeError("HIP IPC import of the predecessor's HBM did not return within 10 s"))


FATAL_SCRIPT = textwrap.dedent('''
    import os, sys
    sys.path.insert(0, %(root)r)
    from terraform_provider_iterative_amd.checkpoint import preemption

    class Ck:
        device_index = 0
        hbm_fault_dump = "/tmp/x.fault.json"
        released = False
        def latest(self): return {"generation": 1, "metadata": {"step": 3}}
        def hbm_metadata(self): return {"generation": 1, "metadata": {"step": 4}}
        def restore_hbm(self):
            raise RuntimeError("tpi_copy_segments failed: hipStreamSynchronize: an illegal "
                               "memory access was encountered")
        def _hbm_manifest_path(self): return %(manifest)r
        def release_hbm_claim(self): print("claim released", flush=True)
        def restore(self, generation=None): raise AssertionError("no fallback in this process")

    preemption.resume(Ck())
    print("resume returned", flush=True)
''')


@pytest.mark.parametrize("supervised", [True, False])
def test_a_sticky_error_in_the_hand_off_is_fatal_not_a_fallback(tmp_path, supervised):
    manifest = tmp_path / "spill.hbm"
    manifest.write_text("{}")
    events = tmp_path / "events.jsonl"
    env = dict(os.environ, TPI_EVENTS_FILE=str(events))
    env.pop("TPI_NOTIFY_FD", None)
    if supervised:
        env["TPI_NOTIFY_FD"] = "1"  # any open fd: only its presence matters here
    proc = subprocess.run([sys.executable, "-c", FATAL_SCRIPT % {"root": ROOT,
                                                                 "manifest": str(manifest)}],
                          env=env, capture_output=True, text=True, timeout=60)
    recs = _events(events)
    fatal = [e for e in recs if e["code"] == "checkpoint-hbm-fatal"]
    assert fatal and "illegal memory access" in fatal[0]["description"][1]
    assert not any(e["code"] == "checkpoint-hbm-failed" for e in recs)
    assert not manifest.exists()  # withdrawn: the predecessor may go, nobody imports again
    assert "claim released" in proc.stdout
    assert "resume returned" not in proc.stdout
    if supervised:
        assert proc.returncode == preemption.PREEMPTED_EXIT_CODE, proc.stderr
        assert "respawns this rank from the host copy" in proc.stderr
    else:
        assert proc.returncode != 0 and "illegal memory access" in proc.stderr


class StuckLib:
    """``tpi_ipc_open`` that blocks until released (hipIpcOpenMemHandle spinning)."""

    def __init__(self):
        self.release = threading.Event()
        self.closed = []

    def tpi_ipc_open(self, handle, device, out):
        self.release.wait(30)
        out._obj.value = 0x1000
        return 0

    def tpi_ipc_close(self, ptr):
        self.closed.append(ptr.value)
        return 0

    def check(self, rc, what):
        assert rc == 0, what


def test_workdir_attach_is_bounded_and_journalled(tmp_path, monkeypatch):
    events = tmp_path / "events.jsonl"
    monkeypatch.setenv("TPI_EVENTS_FILE", str(events))
    lib = StuckLib()
    t0 = time.monotonic()
    with pytest.raises(TimeoutError, match="TPI_IPC_OPEN_TIMEOUT"):
        stage._ipc_open_bounded(lib, b"\0" * 64, 0, 3 * GB, timeout=0.3)
    assert time.monotonic() - t0 < 2
    assert [e["code"] for e in _events(events)] == ["workdir-attach-failed"]
    lib.release.set()  # the stuck import returns late: its mapping is closed, not leaked
    deadline = time.monotonic() + 5
    while not lib.closed and time.monotonic() < deadline:
        time.sleep(0.01)
    assert lib.closed == [0x1000]
    # an import that returns in time maps and is journalled
    lib2 = StuckLib()
    lib2.release.set()
    assert stage._ipc_open_bounded(lib2, b"\0" * 64, 0, 3 * GB, timeout=5) == 0x1000
    assert _events(events)[-1]["code"] == "workdir-attached" and not lib2.closed


class FakeCudaDevices(FakeCuda):
    TOTAL = 288 * 2 ** 30  # an MI355X: 288 GiB = 309.2 GB

    def device_count(self):
        return 1

    def mem_get_info(self, dev):
        return self.free, self.TOTAL


def test_early_hand_off_needs_the_successors_room_by_both_counts(monkeypatch):
    """The predecessor offers its HBM only when the successor's own measure (state + 1 % +
    2 GiB) fits next to it -- "footprint <= free" offered states the successor then could not
    make room for, and both waited out the linger (r6f)."""
    from terraform_provider_iterative_amd.parallel import placement

    cuda = FakeCudaDevices(0)
    monkeypatch.setitem(sys.modules, "torch", types.SimpleNamespace(cuda=cuda))
    monkeypatch.delenv("TPI_EARLY_HANDOFF", raising=False)
    driver = {"used": None}
    monkeypatch.setattr(placement, "device_vram_usage",
                        lambda dev: None if driver["used"] is None
                        else (driver["used"], cuda.TOTAL))
    cuda.free = cuda.TOTAL - 154 * GB  # footprint 154 <= free 155.2, but the need is 157.7
    assert not preemption._handoff_safe()
    cuda.free = cuda.TOTAL - 152 * GB  # a 150 GB state + context: still two copies
    assert preemption._handoff_safe()
    cuda.free = cuda.TOTAL - 102 * GB  # 100 GB state
    assert preemption._handoff_safe()
    driver["used"] = 210 * GB  # ... unless the driver still holds an exited process's memory
    assert not preemption._handoff_safe()
    assert preemption.successor_need(100 * GB) == 101 * GB + 2 * 2 ** 30
    # with a registered state the measure is that state, not everything in use: a hot
    # standby's context (here 2 GB) sits next to a 150 GB state, and a second copy still fits
    driver["used"] = None
    ck = types.SimpleNamespace(plan=types.SimpleNamespace(total=150 * GB), device_index=0)
    monkeypatch.setattr(preemption, "_registered", [ck])
    cuda.free = cuda.TOTAL - 154 * GB
    assert preemption._handoff_safe()
    ck.plan.total = 153 * GB
    assert not preemption._handoff_safe()


PREDECESSOR = textwrap.dedent('''
    import os, sys, time
    sys.path.insert(0, %(root)r)
    from terraform_provider_iterative_amd.checkpoint import preemption
    from terraform_provider_iterative_amd.checkpoint.handoff import _SpillOffer

    open(%(spill)r + ".hbm", "w").write("{}")  # the exported offer
    print("offered", flush=True)
    t0 = time.monotonic()
    how = preemption._await_successor(_SpillOffer(%(spill)r))
    print("exit: %%s after %%.2f s" %% (how, time.monotonic() - t0), flush=True)
''')


def test_successor_withdraws_an_offer_it_cannot_make_room_for(tmp_path, monkeypatch):
    from terraform_provider_iterative_amd.checkpoint import checkpointer as ckmod
    from terraform_provider_iterative_amd.parallel import placement

    spill = str(tmp_path / "spill")
    events = tmp_path / "events.jsonl"
    env = dict(os.environ, TPI_EVENTS_FILE=str(events), TPI_LINGER_SECONDS="60")
    pred = subprocess.Popen([sys.executable, "-c", PREDECESSOR % {"root": ROOT, "spill": spill}],
                            env=env, stdout=subprocess.PIPE, text=True)
    try:
        assert pred.stdout.readline().strip() == "offered"
        monkeypatch.setenv("TPI_EVENTS_FILE", str(events))
        # the predecessor holds its 150 GB state, and memory an earlier process left is still
        # being wiped by the driver: no room for a second copy
        cuda = FakeCudaDevices(140 * GB)
        monkeypatch.setitem(sys.modules, "torch", types.SimpleNamespace(cuda=cuda))
        monkeypatch.setattr(ckmod, "streaming_writer", lambda path: None)  # spill complete
        monkeypatch.setattr(ckmod, "region_total", lambda path: 150 * GB)
        monkeypatch.setattr(placement, "device_vram_usage",
                            lambda dev: (cuda.TOTAL - cuda.free, cuda.TOTAL))

        def predecessor_exits():  # its memory comes back once it has gone
            pred.wait(30)
            cuda.free = cuda.TOTAL - 2 * GB

        threading.Thread(target=predecessor_exits, daemon=True).start()
        t0 = time.monotonic()
        preemption.wait_for_device_memory(spill, timeout=20)
        assert time.monotonic() - t0 < 10  # not the predecessor's 60 s linger
        out = pred.stdout.read()
        assert "exit: successor closed" in out, out
        codes = [e["code"] for e in _events(events)]
        assert "successor-hbm-declined" in codes
        rec = [e for e in _events(events) if e["code"] == "successor-hbm-wait"][-1]
        assert not any("timed out" in d for d in rec["description"])
        assert not os.path.exists(spill + ".hbm") and not os.path.exists(spill + ".hbm.claim")
    finally:
        if pred.poll() is None:
            pred.kill()
        pred.wait()


def test_a_parked_hot_standby_needs_no_room_for_its_context_again(tmp_path, monkeypatch):
    """A hot standby parks with its GPU context and engine made, so that memory is in the
    device's count already: the offer then needs the state + 1 % + 256 MiB next to it, not
    + 2 GiB (a 150 GB state on a 288 GiB MI355X: r6g/r6h took the host path for want of
    ~0.1 GB).  The marker of a dead process, or of this one, does not count."""
    import subprocess as sp

    from terraform_provider_iterative_amd.parallel import placement

    cuda = FakeCudaDevices(FakeCudaDevices.TOTAL - 156 * GB)  # 150 GB state + contexts + rest
    monkeypatch.setitem(sys.modules, "torch", types.SimpleNamespace(cuda=cuda))
    monkeypatch.delenv("TPI_EARLY_HANDOFF", raising=False)
    monkeypatch.setattr(placement, "device_vram_usage", lambda dev: None)
    spill = str(tmp_path / "spill")
    ck = types.SimpleNamespace(plan=types.SimpleNamespace(total=150 * GB), device_index=0,
                               path=spill)
    monkeypatch.setattr(preemption, "_registered", [ck])
    assert not preemption._handoff_safe()  # 153.2 GB free < 153.65 GB needed
    standby = sp.Popen([sys.executable, "-c", "import time; time.sleep(60)"])
    try:
        with open(spill + ".standby", "w") as handle:
            handle.write(str(standby.pid))
        assert preemption._standby_parked()
        assert preemption._handoff_safe()  # 153.2 GB free >= 151.8 GB needed
    finally:
        standby.kill()
        standby.wait()
    assert not preemption._standby_parked() and not preemption._handoff_safe()
    with open(spill + ".standby", "w") as handle:
        handle.write(str(os.getpid()))  # our own marker (a standby that became the rank)
    assert not preemption._standby_parked()
    preemption._mark_parked(spill)  # what a parked standby writes ...
    with open(spill + ".standby") as handle:
        assert int(handle.read()) == os.getpid()
    preemption._unmark_parked(spill)  # ... and removes when it is activated or discarded
    assert not os.path.exists(spill + ".standby")
