"""The hand-off protocol between a preempted rank, its successor and the supervisor.

Reference: a reclaimed spot VM is replaced and restores the bucket's ``data/`` (machine-script
.sh.tpl:89); the scaling group goes to 0 right after the task exits (tpl:10-15, 51;
resource_auto_scaling_group.go:188-199).  Here the successor copies the predecessor's HBM over
IPC, so the predecessor must outlive every mapping of its memory ("closed"), and the node's
resources go back as soon as the ranks are down -- not when the last released process has
finished its kernel teardown.

* supervisor: SIGUSR2 to the predecessor only after the successor's ``closed`` (or its
  death), never on ``restored hbm``; leases released before a slow released process is reaped;
  its exit traced (``exit-trace``);
* rank: :func:`preemption._await_successor` holds the exporter until the claim protocol says
  nobody maps its memory -- on the success path and after a failed spill;
* reclaim: a queued on-demand task starts while the victim's process is still exiting.
"""
import json
import os
import signal
import subprocess
import sys
import threading
import time

import pytest

from terraform_provider_iterative_amd import _build
from terraform_provider_iterative_amd.checkpoint import preemption
from terraform_provider_iterative_amd.checkpoint.checkpointer import CheckpointError, Checkpointer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def binary():
    return _build.build_supervisor()


def _spec(tmp_path, script, **extra):
    task = tmp_path / "task"
    for d in ("data", "reports", "supervisor"):
        (task / d).mkdir(parents=True, exist_ok=True)
    path = task / "supervisor" / "script"
    path.write_text(script)
    path.chmod(0o755)
    spec = {"task_id": "tpi-handoff-test", "task_dir": str(task), "workdir": str(task / "data"),
            "script": str(path), "env": {"PATH": os.environ["PATH"]}, "parallelism": 1,
            "ranks": [{"gpus": "", "rank_gpus": ""}], "grace_seconds": 20,
            "master_port": 29998}
    spec.update(extra)
    spec_path = task / "supervisor" / "spec.json"
    spec_path.write_text(json.dumps(spec))
    return task, str(spec_path)


def _events(task):
    with open(task / "supervisor" / "events.jsonl") as handle:
        return [json.loads(line) for line in handle if line.strip()]


def _wait_file(path, timeout=30):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if os.path.exists(path) and os.path.getsize(path):
            return
        time.sleep(0.01)
    raise AssertionError("%s never appeared" % path)


# A rank that speaks the notify protocol by hand (no torch): incarnation 0 is preempted,
# releases, waits for SIGUSR2 and records when it came; incarnation 1 "restores from its HBM"
# and, unless told to die first, closes the hand-off one second later.
PROTOCOL_RANK = r'''#!%(python)s
import os, signal, sys, time
out = %(out)r
def note(name):
    with open(os.path.join(out, name), "w") as f:
        f.write(repr(time.time()))
restart = int(os.environ["TPI_RESTART_COUNT"])
fd = int(os.environ["TPI_NOTIFY_FD"])
if restart == 0:
    signal.pthread_sigmask(signal.SIG_BLOCK, {signal.SIGTERM, signal.SIGUSR2})
    print("ready", flush=True)
    signal.sigwait({signal.SIGTERM})
    os.write(fd, b"released\n")
    signal.sigwait({signal.SIGUSR2})
    note("usr2")
    time.sleep(%(slow_exit)r)  # a slow teardown after the exit request
    os._exit(143)
os.write(fd, b"restored hbm\n")
time.sleep(1.0)
if %(die)r:
    note("successor-exit")
    os._exit(0)
note("closed")
os.write(fd, b"closed\n")
time.sleep(0.2)
print("successor done", flush=True)
'''


@pytest.mark.parametrize("die", [False, True], ids=["closed", "successor-dies"])
def test_predecessor_released_only_after_closed(binary, tmp_path, die):
    out = tmp_path / "out"
    out.mkdir()
    lease = tmp_path / "gpu-0.lease"
    lease.write_text("{}")
    script = PROTOCOL_RANK % {"python": sys.executable, "out": str(out), "die": die,
                              "slow_exit": 2.0}
    task, spec = _spec(tmp_path, script, leases=[str(lease)])
    sup = subprocess.Popen([binary, spec], stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    try:
        deadline = time.time() + 30
        while time.time() < deadline and not any(
                "ready" in (task / "reports" / n).read_text()
                for n in os.listdir(task / "reports") if n.startswith("task-")):
            time.sleep(0.02)
        sup.send_signal(signal.SIGUSR1)  # preempt
        _, err = sup.communicate(timeout=60)
    finally:
        if sup.poll() is None:
            sup.kill()
    for marker in (b"AddressSanitizer", b"LeakSanitizer", b"runtime error"):  # (ASan build)
        assert marker not in err, err[-3000:]
    assert sup.returncode == 0, err[-2000:]
    usr2 = float((out / "usr2").read_text())
    after = float((out / ("successor-exit" if die else "closed")).read_text())
    # "restored hbm" alone never lets the predecessor go: its memory is still mapped
    assert usr2 >= after, (usr2, after)
    events = _events(task)
    codes = [e["code"] for e in events]
    req = [e for e in events if e["code"] == "predecessor-exit-requested"]
    assert len(req) == 1, codes
    assert req[0]["description"][-1] == ("successor exited" if die else
                                         "successor closed the HBM hand-off")
    # the successor finished; the predecessor takes 2 s more to exit: the lease is released
    # before it is reaped, and its exit is traced meanwhile
    t = {c: next(e["time"] for e in events if e["code"] == c)
         for c in ("resources-released", "rank-released-exit", "supervisor-exit")}
    assert t["resources-released"] < t["rank-released-exit"] <= t["supervisor-exit"]
    assert t["rank-released-exit"] - t["resources-released"] > 0.5
    assert not lease.exists()
    traces = [e for e in events if e["code"] == "exit-trace"]
    assert traces and all(e["description"][3].startswith("+") for e in traces), traces[:3]
    released_exit = next(e for e in events if e["code"] == "rank-released-exit")
    assert released_exit["description"][-1].endswith("after the exit request")


# -- the exporter side: _await_successor / _save_and_exit with a stand-in checkpointer ----------

class _FakeHandoff:
    """The parts of a Checkpointer the hand-off protocol touches (the manifest is what
    export_hbm() would write; no GPU)."""

    def __init__(self, path):
        self.path = path
        self.region = None

    def _hbm_manifest_path(self):
        return self.path + ".hbm"

    _hbm_claim_path = Checkpointer._hbm_claim_path
    hbm_claim_owner = Checkpointer.hbm_claim_owner
    claim_hbm = Checkpointer.claim_hbm
    release_hbm_claim = Checkpointer.release_hbm_claim


def _claimer(path, hold, remove_manifest=True, die=False):
    """A "successor" process: claims the hand-off, holds it ``hold`` s, then closes (drops
    manifest + claim) -- or dies holding it."""
    code = ("import os, sys, time\nsys.path.insert(0, %r)\n"
            "from tests.test_handoff_protocol import _FakeHandoff\n"
            "ck = _FakeHandoff(%r)\nassert ck.claim_hbm()\nprint('claimed', flush=True)\n"
            "time.sleep(%r)\n"
            "if %r:\n    os._exit(0)\n"
            "if %r:\n    os.remove(ck._hbm_manifest_path())\n"
            "ck.release_hbm_claim()\n" % (ROOT, path, hold, die, remove_manifest))
    proc = subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE)
    assert proc.stdout.readline().strip() == b"claimed"
    return proc


@pytest.fixture()
def exporter(tmp_path, monkeypatch):
    ck = _FakeHandoff(str(tmp_path / "spill"))
    with open(ck._hbm_manifest_path(), "w") as f:
        f.write("{}")
    monkeypatch.setattr(preemption, "_usr2", type(preemption._usr2)())
    monkeypatch.setenv("TPI_LINGER_SECONDS", "30")
    monkeypatch.delenv("TPI_EVENTS_FILE", raising=False)
    return ck


def test_exporter_waits_for_the_claimer_to_close_even_after_sigusr2(exporter):
    proc = _claimer(exporter.path, hold=1.0)
    preemption._usr2.set()  # a supervisor that says "go" too early
    t0 = time.monotonic()
    how = preemption._await_successor(exporter)
    took = time.monotonic() - t0
    proc.wait(10)
    assert how == "successor closed" and took >= 0.8, (how, took)


def test_exporter_goes_when_the_claimer_dies(exporter):
    proc = _claimer(exporter.path, hold=0.5, die=True)
    how = preemption._await_successor(exporter)
    proc.wait(10)
    assert how == "successor died"


def test_exporter_withdraws_an_unclaimed_offer(exporter):
    preemption._usr2.set()
    assert preemption._await_successor(exporter) == "withdrawn"
    assert exporter.hbm_claim_owner() == os.getpid()
    # a successor arriving now cannot import any more: it restores from the host copy
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from tests.test_handoff_protocol import _FakeHandoff\n"
            "print(_FakeHandoff(%r).claim_hbm())" % (ROOT, exporter.path))
    assert subprocess.check_output([sys.executable, "-c", code]).strip() == b"False"


def test_exporter_withdraws_after_the_linger_timeout(exporter, monkeypatch):
    monkeypatch.setenv("TPI_LINGER_SECONDS", "0.3")
    t0 = time.monotonic()
    assert preemption._await_successor(exporter) == "withdrawn"
    assert time.monotonic() - t0 >= 0.3


def test_an_empty_claim_is_never_taken_for_a_dead_holder(exporter, monkeypatch):
    #  a claim file seen between its creation and its pid being written must not
    # read as "holder died": neither a second claimer nor the exporter may act on it
    with open(exporter._hbm_claim_path(), "w"):
        pass
    assert exporter.hbm_claim_owner() == 0
    assert not exporter.claim_hbm()
    assert os.path.exists(exporter._hbm_claim_path())
    monkeypatch.setenv("TPI_HANDOFF_CLOSE_TIMEOUT", "0.3")
    preemption._usr2.set()
    how = preemption._await_successor(exporter)
    assert how.startswith("timeout"), how


CLAIM_RACE = r'''
import os, sys, time
sys.path.insert(0, %(root)r)
from tests.test_handoff_protocol import _FakeHandoff
ck = _FakeHandoff(%(path)r)
while time.time() < %(start)r:
    pass
got = ck.claim_hbm()
owner = ck.hbm_claim_owner()
print(int(got), owner, flush=True)
time.sleep(0.5)  # stay alive: a live holder
'''


def test_concurrent_claims_have_exactly_one_winner_who_is_the_recorded_owner(tmp_path):
    path = str(tmp_path / "spill")
    start = time.time() + 1.5
    procs = [subprocess.Popen([sys.executable, "-c", CLAIM_RACE % {
        "root": ROOT, "path": path, "start": start}], stdout=subprocess.PIPE, text=True)
        for _ in range(8)]
    rows = [p.communicate(timeout=30)[0].split() for p in procs]
    winners = [p.pid for p, (got, _) in zip(procs, rows) if got == "1"]
    assert len(winners) == 1, rows
    # every loser already saw the winner's pid in the claim (never an empty file)
    assert all(int(owner) == winners[0] for _, owner in rows), (winners, rows)
    assert not [n for n in os.listdir(tmp_path) if n.endswith(".tmp")]


EXPORTER = r'''
import os, sys, time
sys.path.insert(0, %(root)r)
from terraform_provider_iterative_amd.checkpoint import preemption
from terraform_provider_iterative_amd.checkpoint.checkpointer import CheckpointError
from tests.test_handoff_protocol import _FakeHandoff

class Res:
    bytes = wire_bytes = 1000
    seconds = 0.1
    gbps = 1e-5

class Exporting(_FakeHandoff):
    def export_hbm(self, metadata=None):
        with open(self._hbm_manifest_path(), "w") as f:
            f.write("{}")
        return self._hbm_manifest_path()
    def save(self, metadata, on_stream=None, **kw):
        on_stream()  # "released": the successor starts and may import our HBM
        time.sleep(0.3)
        if %(fail)r:
            raise CheckpointError("host spill failed (injected)")
        return Res()

preemption.register(Exporting(%(path)r))
preemption.install()  # SIGUSR2 handler, as in every rank
preemption._save_and_exit("boundary")
'''


@pytest.mark.parametrize("fail", [False, True], ids=["spill-ok", "spill-failed"])
def test_preempted_rank_never_exits_while_its_hbm_is_claimed(tmp_path, fail):
    """_save_and_exit end to end with a fake notify pipe: after "released" a successor claims
    the export; the rank must stay alive until the claim is dropped (spill ok: code 143;
    spill failed: code 1 -- the HBM copy is the only good one, so it waits just the same)."""
    path = str(tmp_path / "spill")
    r, w = os.pipe()
    env = dict(os.environ, TPI_NOTIFY_FD=str(w), TPI_LINGER_SECONDS="30",
               TPI_EVENTS_FILE=str(tmp_path / "events.jsonl"))
    env.pop("TPI_REQUEUE_FILE", None)
    proc = subprocess.Popen([sys.executable, "-c", EXPORTER % {"root": ROOT, "path": path,
                                                                 "fail": fail}],
                            env=env, pass_fds=(w,))
    os.close(w)
    try:
        assert os.read(r, 64) == b"released\n"
        ck = _FakeHandoff(path)
        assert ck.claim_hbm()  # this test process is the successor
        os.kill(proc.pid, signal.SIGUSR2)  # an early "go" must not matter while claimed
        time.sleep(1.5)
        assert proc.poll() is None, "the exporter exited while its HBM was claimed"
        os.remove(ck._hbm_manifest_path())  # copy done ...
        ck.release_hbm_claim()              # ... and every mapping closed
        assert proc.wait(10) == (1 if fail else preemption.PREEMPTED_EXIT_CODE)
    finally:
        if proc.poll() is None:
            proc.kill()
        os.close(r)
    with open(tmp_path / "events.jsonl") as f:
        events = [json.loads(line) for line in f]
    exit_ev = [e for e in events if e["code"] == "predecessor-exit"]
    assert exit_ev and exit_ev[0]["description"][1] == "successor closed", events
    assert not os.path.exists(path + ".hbm") and not os.path.exists(path + ".hbm.claim")


# -- reclaim: the on-demand task starts while the victim is still exiting ----------------------

SPOT = r'''#!%(python)s
import os, sys, time
sys.path.insert(0, %(root)r)
import torch
from terraform_provider_iterative_amd.checkpoint import Checkpointer, preemption
state = {"w": torch.zeros(1000, dtype=torch.float64)}
ck = Checkpointer(state, path=os.path.join(os.environ["TPI_DATA_DIRECTORY"], ".spill"),
                  tile_bytes=4096)
meta = preemption.resume(ck)
start = (meta or {}).get("step", 0)
print("start", start, flush=True)
preemption.register(ck)
preemption.install()
_exit = preemption._teardown
def slow_teardown(code, release_device=True):  # a victim whose kernel teardown is slow
    time.sleep(3.0)
    _exit(code, release_device)
preemption._teardown = slow_teardown
for step in range(start, %(steps)d):
    state["w"] += 1
    time.sleep(0.05)
    preemption.step(step + 1)
print("final", int(state["w"][0]), flush=True)
'''


def test_reclaimed_gpu_goes_to_the_on_demand_task_before_the_victim_is_reaped(tmp_path,
                                                                                monkeypatch):
    from tests.test_scheduler import _cloud, _task

    monkeypatch.setenv("TPI_MI355X_GPUS", "0")
    monkeypatch.setenv("TPI_NODE_CPUS", "0-31")
    monkeypatch.setenv("TPI_NODE_MEMORY_MB", "512000")
    cloud = _cloud(tmp_path)
    spot = _task(cloud, "spot-slow", SPOT % {"python": sys.executable, "root": ROOT,
                                             "steps": 30}, spot=0)
    spot.create()
    deadline = time.time() + 60
    while time.time() < deadline and "start 0" not in "".join(spot.logs()):
        time.sleep(0.05)
    time.sleep(0.3)
    od = _task(cloud, "ondemand-fast", "#!/bin/sh\necho on-demand running\n")
    t_apply = time.time()
    od.create()
    deadline = time.time() + 60
    while time.time() < deadline and "on-demand running" not in "".join(od.logs()):
        time.sleep(0.01)
    t_first_log = time.time()
    deadline = time.time() + 120
    while time.time() < deadline and (spot.supervisor_running() or od.supervisor_running()
                                      or spot.status()["succeeded"] < 1):
        time.sleep(0.05)
    spot_ev = {e.code: e.time.timestamp() for e in reversed(spot.events())}  # first of each
    od_start = next(e.time.timestamp() for e in od.events() if e.code == "rank-start")
    assert spot.status()["succeeded"] == 1 and od.status()["succeeded"] == 1, spot.logs()
    # saved -> released (no linger, no hand-off) -> resources back -> on-demand starts,
    # all while the victim still sleeps in its teardown
    assert spot_ev["checkpoint-released"] <= spot_ev["resources-released"] < od_start
    assert od_start < spot_ev["rank-released-exit"], (od_start, spot_ev)
    assert t_first_log - t_apply < 3.0, t_first_log - t_apply
    codes = [e.code for e in spot.events()]
    assert "checkpoint-streaming" not in codes and "checkpoint-hbm-export" not in codes
    assert "exit-trace" in codes
    logs = spot.logs()
    assert "final 30" in logs[-1], logs
    od.delete()
    spot.delete()


RELEASING = r'''
import os, sys, time
sys.path.insert(0, %(root)r)
from terraform_provider_iterative_amd.checkpoint import preemption
from tests.test_handoff_protocol import _FakeHandoff

class Res:
    bytes = wire_bytes = 1000
    seconds = 0.1
    gbps = 1e-5
    released_bytes = 10 ** 9  # the save freed every tensor's HBM behind the spill

class ReleasingBehind(_FakeHandoff):
    def save(self, metadata, on_stream=None, release_behind=False, **kw):
        assert release_behind and on_stream is None
        return Res()

preemption.register(ReleasingBehind(%(path)r))
preemption.install()
preemption._save_and_exit("boundary")
'''


def test_a_save_that_released_behind_the_spill_still_says_released(tmp_path):
    """ a state too big for two copies (not safe) is freed by the save itself
    (release_behind); "released" must still go out, before the exit, so the supervisor hands
    the GPU on without waiting for the process to be reaped."""
    r, w = os.pipe()
    env = dict(os.environ, TPI_NOTIFY_FD=str(w), TPI_LINGER_SECONDS="1.0",
               TPI_EARLY_HANDOFF="0", TPI_EVENTS_FILE=str(tmp_path / "events.jsonl"))
    env.pop("TPI_REQUEUE_FILE", None)
    proc = subprocess.Popen([sys.executable, "-c", RELEASING % {
        "root": ROOT, "path": str(tmp_path / "spill")}], env=env, pass_fds=(w,))
    os.close(w)
    try:
        assert os.read(r, 64) == b"released\n"
        assert proc.poll() is None, "released must come before the exit"
        assert proc.wait(10) == preemption.PREEMPTED_EXIT_CODE
    finally:
        if proc.poll() is None:
            proc.kill()
        os.close(r)


def test_a_stuck_ipc_import_gives_up_the_hbm_route_and_the_claim(tmp_path, monkeypatch):
    """ hipIpcOpenMemHandle that never returns: restore_hbm raises after
    TPI_IPC_OPEN_TIMEOUT (the caller restores from the host copy) and drops its claim, so the
    predecessor is not kept waiting for a successor that will never close."""
    from terraform_provider_iterative_amd.checkpoint import checkpointer as ckmod
    from terraform_provider_iterative_amd.checkpoint import handoff as hmod

    stuck = threading.Event()

    class FakeLib:
        def tpi_ipc_open(self, handle, device, out):
            if handle == b"\x02":
                stuck.wait(60)  # the import that never returns
            return 0

        def tpi_ipc_close(self, ptr):
            return 0

        def check(self, rc, what):
            assert rc == 0, what

    import types

    import numpy as np

    from terraform_provider_iterative_amd.ops.packing import SEG_DTYPE

    class Successor(_FakeHandoff):
        device_index = 0
        plan = types.SimpleNamespace(segs=np.zeros(0, dtype=SEG_DTYPE))
        restore_hbm = Checkpointer.restore_hbm
        _restore_hbm = Checkpointer._restore_hbm

        def _hbm_doc(self):
            return {"allocations": [1 << 20] * 3, "ipc": {"0": "01", "1": "02", "2": "03"},
                    "where": [], "segs": ""}

    monkeypatch.setattr(hmod, "hip", lambda *a, **k: FakeLib())
    monkeypatch.setenv("TPI_IPC_OPEN_TIMEOUT", "0.5")
    ck = Successor(str(tmp_path / "spill"))
    t0 = time.monotonic()
    with pytest.raises(CheckpointError, match="did not return within"):
        ck.restore_hbm()
    assert time.monotonic() - t0 < 5.0
    assert ck.hbm_claim_owner() is None  # the claim is gone: the predecessor may go
    stuck.set()


# -- the hand-off state machine, one row per mode (docs/ARCHITECTURE.md "Hand-off modes") -------
# A rank that speaks the notify protocol for every supervisor-visible mode.  Incarnation 0 is
# preempted: "released", then it waits for the supervisor's exit request (SIGUSR2).  The
# successor -- a fresh process (cold), or a standby activated by "go" (warm: started at the
# preemption; hot: started with the rank) -- reports what a real successor reports.
MODE_RANK = r'''#!%(python)s
import os, signal, sys, time
out, mode = %(out)r, %(mode)r
fd = int(os.environ["TPI_NOTIFY_FD"])
def note(name):
    with open(os.path.join(out, name), "w") as f:
        f.write(repr(time.time()))
if mode in ("warm", "hot"):
    os.write(fd, b"standby\n")  # preemption.standby(): standbys are welcome
if os.environ.get("TPI_STANDBY") == "1":
    msg = os.read(int(os.environ["TPI_STANDBY_FD"]), 64)
    if not msg.startswith(b"go"):
        os._exit(0)  # discarded
    note("activated")
if int(os.environ["TPI_RESTART_COUNT"]) == 0:
    signal.pthread_sigmask(signal.SIG_BLOCK, {signal.SIGTERM, signal.SIGUSR2})
    print("ready", flush=True)
    signal.sigwait({signal.SIGTERM})
    os.write(fd, b"released\n")
    signal.sigwait({signal.SIGUSR2})
    note("usr2")
    os._exit(143)
if mode.startswith("hbm"):
    os.write(fd, b"restored hbm\n")
    time.sleep(0.5)
    if mode == "hbm-successor-dies":
        note("successor-exit")
        os._exit(0)
    note("closed")
    os.write(fd, b"closed\n")
else:
    note("restored")
    os.write(fd, b"restored\n")
time.sleep(0.2)
print("successor done", flush=True)
'''

# mode -> (spec extras, the predecessor's release reason, the successor's start, the note
# the predecessor's SIGUSR2 may not precede)
HANDOFF_MODES = {
    "cold": ({}, "successor restored", "fresh", "restored"),
    "warm": ({"standby": True}, "successor restored", "warm standby", "restored"),
    "hot": ({"standby": True, "standby_hot": True}, "successor restored", "warm standby",
            "restored"),
    "hbm": ({}, "successor closed the HBM hand-off",
            "fresh", "closed"),
    "hbm-successor-dies": ({}, "successor exited", "fresh", "successor-exit"),
}


@pytest.mark.parametrize("mode", sorted(HANDOFF_MODES))
def test_handoff_mode_row(binary, tmp_path, mode):
    extra, why, start, gate = HANDOFF_MODES[mode]
    out = tmp_path / "out"
    out.mkdir()
    script = MODE_RANK % {"python": sys.executable, "out": str(out), "mode": mode}
    task, spec = _spec(tmp_path, script, **extra)
    sup = subprocess.Popen([binary, spec], stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    try:
        deadline = time.time() + 30
        while time.time() < deadline and not any(
                "ready" in (task / "reports" / n).read_text()
                for n in os.listdir(task / "reports") if n.startswith("task-")):
            time.sleep(0.02)
        if mode == "hot":  # the hot standby is up before the preemption
            while time.time() < deadline and "standby-start" not in [
                    e["code"] for e in _events(task)]:
                time.sleep(0.02)
        sup.send_signal(signal.SIGUSR1)  # preempt
        _, err = sup.communicate(timeout=60)
    finally:
        if sup.poll() is None:
            sup.kill()
    assert sup.returncode == 0, err[-2000:]
    events = _events(task)
    codes = [e["code"] for e in events]
    t = lambda code: next(e["time"] for e in events if e["code"] == code)  # noqa: E731
    # released -> the successor runs -> it lets the predecessor go -> the task settles and ends
    for a, b in (("preempt-requested", "rank-released"),
                 ("rank-released", "predecessor-exit-requested"),
                 ("predecessor-exit-requested", "supervisor-settled"),
                 ("supervisor-settled", "supervisor-exit")):
        assert t(a) <= t(b), (a, b, codes)
    req = [e for e in events if e["code"] == "predecessor-exit-requested"]
    assert len(req) == 1 and req[0]["description"][-1] == why, req
    # the predecessor is never told to go before the successor is done with it
    assert float((out / "usr2").read_text()) >= float((out / gate).read_text())
    starts = [e for e in events if e["code"] == "rank-start"]
    assert len(starts) == 2, starts
    assert (starts[1]["description"][-1] == "warm standby") == (start == "warm standby"), starts
    if mode == "hot":
        assert t("standby-start") < t("preempt-requested")
    if mode == "warm":
        assert t("preempt-requested") <= t("standby-start")
    status = [n for n in os.listdir(task / "reports") if n.startswith("status-")]
    assert len(status) == 1, status  # the successor's; the predecessor's release is no status


def test_dmabuf_route_hands_every_allocation_over_the_socket(tmp_path, monkeypatch):
    """TPI_HBM_ROUTE=dmabuf (round 5): allocations below IPC_MAX_ALLOC travel as HIP IPC
    handles in the manifest, the larger ones as dma-buf descriptors the exporter serves over an
    abstract Unix socket (batches of FDS_PER_MESSAGE, SCM_RIGHTS), each buffer's size checked
    on both sides.  The successor maps each, points the source segments at base + offset + the
    tensor's place in the allocation, copies, and unmaps them all behind the restore.  Buffers
    are sparse memfds and mappings fake addresses: no GPU."""
    import numpy as np

    import torch

    from terraform_provider_iterative_amd.checkpoint import checkpointer as ckmod
    from terraform_provider_iterative_amd.checkpoint import handoff as hmod
    from terraform_provider_iterative_amd.ops.packing import SEG_DTYPE

    n_alloc = ckmod.FDS_PER_MESSAGE + 37  # two batches of dma-bufs ...
    n_small = 5                           # ... and a few IPC handles
    sizes = [(3 << 30) + i * 4096 for i in range(n_alloc)] + [1 << 20] * n_small
    imported, opened, unmapped, closed = {}, {}, [], []

    class FakeLib:
        def tpi_mem_range(self, ptr, base, size):
            i = (ptr.value - 0x1000_0000_0000) // (1 << 33)
            base._obj.value, size._obj.value = 0x1000_0000_0000 + i * (1 << 33), sizes[i]
            return 0

        def tpi_dmabuf_available(self):
            return 1

        def tpi_dmabuf_export(self, ptr, size, fd, off):
            f = os.memfd_create("fake-dmabuf")
            os.ftruncate(f, size + 4096)
            fd._obj.value = f
            off._obj.value = 4096
            return 0

        def tpi_ipc_export(self, ptr, handle, off, size):
            handle.raw = ("%064x" % ptr.value).encode()[:64]
            return 0

        def tpi_dmabuf_import(self, device, fd, ptr, size):
            ptr._obj.value = 0x7000_0000_0000 + len(imported) * (1 << 36)
            size._obj.value = os.lseek(fd, 0, os.SEEK_END)
            imported[ptr._obj.value] = fd
            return 0

        def tpi_ipc_open(self, handle, device, out):
            out._obj.value = 0x6000_0000_0000 + len(opened) * (1 << 30)
            opened[out._obj.value] = handle
            return 0

        def tpi_dmabuf_unmap(self, ptr):
            unmapped.append(ptr.value)
            return 0

        def tpi_ipc_close(self, ptr):
            closed.append(ptr.value)
            return 0

        def tpi_device_pci_bus_id(self, dev, buf, n):
            buf.value = b"0000:75:00.0"
            return 0

        def check(self, rc, what):
            assert rc == 0, what

    monkeypatch.setattr(hmod, "hip", lambda *a, **k: FakeLib())
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a: None)
    monkeypatch.setattr(torch.cuda, "current_stream",
                        lambda *a: type("S", (), {"cuda_stream": 0})())
    monkeypatch.setenv("TPI_HBM_ROUTE", "dmabuf")

    n = n_alloc + n_small
    segs = np.zeros(n, dtype=SEG_DTYPE)
    segs["ptr"] = [0x1000_0000_0000 + i * (1 << 33) + 512 * i for i in range(n)]
    segs["nbytes"] = 4096

    class Plan:
        pass

    Plan.segs, Plan.total, Plan.tile_bytes = segs, 1 << 30, 1 << 20

    class Exporter(_FakeHandoff):
        device_index = 0
        engine = object()
        plan = Plan
        _entries_digest = "d"
        export_hbm = Checkpointer.export_hbm
        _publish_hbm = Checkpointer._publish_hbm
        _free_relocated = Checkpointer._free_relocated
        _serve_dmabufs = Checkpointer._serve_dmabufs
        _close_dmabuf_server = Checkpointer._close_dmabuf_server

        def _target(self):
            return None, 3

    exporter = Exporter(str(tmp_path / "spill"))
    manifest = exporter.export_hbm({"step": 9})
    with open(manifest) as f:
        doc = json.load(f)
    assert len(doc["ipc"]) == n_small and len(doc["dmabuf"]) == n_alloc, doc.keys()
    assert sorted(int(i) for i in doc["ipc"]) == list(range(n_alloc, n))

    copied = {}

    class Engine:
        def copy_segments(self, src, plan, sig, dst=None):
            copied["src"] = src.copy()

            class Res:
                bad_tiles = 0
            return Res()

    class Successor(_FakeHandoff):
        device_index = 0
        engine = Engine()
        plan = Plan
        restore_hbm = Checkpointer.restore_hbm
        _restore_hbm = Checkpointer._restore_hbm

        def _hbm_doc(self):
            return doc

    ck = Successor(str(tmp_path / "spill"))
    ck.restore_hbm()
    ck._hbm_closer.join(10)
    src = copied["src"]
    maps = sorted(imported)
    for i in range(n_alloc):  # the dma-bufs, in the exporter's order
        assert int(src[i]["ptr"]) == maps[i] + 4096 + 512 * i
    ipc_bases = {int(h.decode(), 16): b for b, h in opened.items()}
    for i in range(n_alloc, n):
        assert int(src[i]["ptr"]) == ipc_bases[0x1000_0000_0000 + i * (1 << 33)] + 512 * i
    assert sorted(unmapped) == maps and sorted(closed) == sorted(opened)
    assert ck.hbm_claim_owner() is None
    exporter._close_dmabuf_server()


def test_auto_route_relocates_tensors_of_big_allocations(tmp_path, monkeypatch):
    """The default route (round 5): tensors in an allocation HIP IPC cannot open (>= 2 GiB) are
    copied device to device into plain blocks of at most RELOCATE_CHUNK bytes, which travel
    over HIP IPC like every other allocation; the successor splits those segments -- source and
    destination at the same stream offsets -- and copies as usual.  Fake device: no GPU."""
    import numpy as np

    import torch

    from terraform_provider_iterative_amd.checkpoint import checkpointer as ckmod
    from terraform_provider_iterative_amd.checkpoint import handoff as hmod
    from terraform_provider_iterative_amd.ops.packing import SEG_CONTIG, SEG_DTYPE

    G = 1 << 30
    # allocation 0: 5 GiB holding two tensors (3 GiB + 1.5 GiB); 1: a small one; 2: 2.5 GiB
    tensors = [(0x1000_0000_0000, 0, 3 * G), (0x1000_0000_0000, 3 * G, G + G // 2),
               (0x2000_0000_0000, 0, 1 << 20), (0x3000_0000_0000, 0, 5 * G // 2)]
    alloc_size = {0x1000_0000_0000: 5 * G, 0x2000_0000_0000: 4 << 20, 0x3000_0000_0000: 5 * G // 2}
    blocks, copies, opened = [], [], {}
    freed, fail_export = [], []

    class FakeLib:
        def tpi_mem_range(self, ptr, base, size):
            key = max(k for k in alloc_size if k <= ptr.value)
            base._obj.value, size._obj.value = key, alloc_size[key]
            return 0

        def tpi_dev_alloc(self, n, out):
            out._obj.value = 0x9000_0000_0000 + len(blocks) * (2 * G)
            blocks.append((out._obj.value, n))
            return 0

        def tpi_d2d(self, dst, src, n, stream):
            copies.append((dst.value, src.value, n))
            return 0

        def tpi_dev_free(self, ptr):
            freed.append(ptr.value)
            return 0

        def tpi_dmabuf_available(self):
            return 1

        def tpi_ipc_export(self, ptr, handle, off, size):
            if fail_export:
                return 1
            handle.raw = ("%064x" % ptr.value).encode()[:64]
            return 0

        def tpi_ipc_open(self, handle, device, out):
            out._obj.value = int(handle.decode(), 16) + 0x0100_0000_0000_0000  # "mapped" here
            opened[out._obj.value] = handle
            return 0

        def tpi_ipc_close(self, ptr):
            return 0

        def tpi_device_pci_bus_id(self, dev, buf, n):
            buf.value = b"0000:75:00.0"
            return 0

        def check(self, rc, what):
            assert rc == 0, what

    monkeypatch.setattr(hmod, "hip", lambda *a, **k: FakeLib())
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a: None)
    monkeypatch.setattr(torch.cuda, "mem_get_info", lambda *a: (200 * G, 288 * G))
    monkeypatch.setattr(torch.cuda, "current_stream",
                        lambda *a: type("S", (), {"cuda_stream": 0})())
    monkeypatch.delenv("TPI_HBM_ROUTE", raising=False)

    segs = np.zeros(len(tensors), dtype=SEG_DTYPE)
    off = 0
    for i, (key, o, n) in enumerate(tensors):
        segs[i]["ptr"], segs[i]["off"], segs[i]["nbytes"] = key + o, off, n
        segs[i]["kind"] = SEG_CONTIG
        off += n

    class Plan:
        pass

    Plan.segs, Plan.total, Plan.tile_bytes = segs, off, 1 << 20

    class Exporter(_FakeHandoff):
        device_index = 0
        engine = object()
        plan = Plan
        _entries_digest = "d"
        export_hbm = Checkpointer.export_hbm
        _publish_hbm = Checkpointer._publish_hbm
        _free_relocated = Checkpointer._free_relocated
        _relocate = Checkpointer._relocate

        def _target(self):
            return None, 1

    # an export that fails after the relocation frees the relocated blocks at
    # once (nothing was published), instead of holding them through the save
    freed.clear()
    fail_export.append(True)
    failing = Exporter(str(tmp_path / "spill-failing"))
    with pytest.raises(AssertionError, match="tpi_ipc_export"):
        failing.export_hbm()
    assert len(freed) == 8 and not failing._relocated
    assert not os.path.exists(str(tmp_path / "spill-failing") + ".hbm")
    fail_export.clear()
    copies.clear()

    with open(Exporter(str(tmp_path / "spill")).export_hbm()) as f:
        doc = json.load(f)
    # 3 + 2 + 3 blocks of <= 1 GiB; the small allocation stays itself; nothing >= 2 GiB left
    assert sorted(doc["pieces"]) == ["0", "1", "3"]
    assert [len(doc["pieces"][k]) for k in ("0", "1", "3")] == [3, 2, 3]
    assert max(doc["allocations"]) <= ckmod.RELOCATE_CHUNK and len(doc["ipc"]) == 9
    assert sum(n for _, _, n in copies) == 3 * G + G + G // 2 + 5 * G // 2
    assert doc["where"][2] is not None and doc["where"][0] is None

    dst_base = 0x5000_0000_0000
    alloc_size[dst_base] = off  # the successor's own allocation holding its tensors
    dsegs = segs.copy()
    dsegs["ptr"] = [dst_base + int(s["off"]) for s in segs]
    seen = {}

    class Engine:
        def copy_segments(self, src, plan, sig, dst=None):
            seen["src"], seen["dst"] = src.copy(), dst.copy()

            class Res:
                bad_tiles = 0
            return Res()

    class DstPlan:
        pass

    DstPlan.segs, DstPlan.total, DstPlan.tile_bytes = dsegs, off, 1 << 20

    class Successor(_FakeHandoff):
        device_index = 0
        engine = Engine()
        plan = DstPlan
        restore_hbm = Checkpointer.restore_hbm
        _restore_hbm = Checkpointer._restore_hbm

        def _hbm_doc(self):
            return doc

    ck = Successor(str(tmp_path / "spill"))
    ck.restore_hbm()
    ck._hbm_closer.join(10)
    src, dst = seen["src"], seen["dst"]
    assert len(src) == len(dst) == 3 + 2 + 1 + 3
    assert list(src["off"]) == list(dst["off"]) == sorted(src["off"])
    assert list(src["nbytes"]) == list(dst["nbytes"])
    assert all(int(d["ptr"]) == dst_base + int(d["off"]) for d in dst)  # split in place
    # every source piece is a mapped block (or the small allocation), never a big allocation
    mapped = set(opened)
    assert all(any(b <= int(p) < b + 2 * G for b in mapped) for p in src["ptr"])


def test_copy_ranges_are_checked_on_the_host_before_any_kernel():
    """A hand-off descriptor that would read past the mapped predecessor allocation, or write
    past the successor's own, is refused on the host (CheckpointError: restore from the host
    copy) -- the copy kernel never sees it."""
    import numpy as np

    from terraform_provider_iterative_amd.checkpoint.handoff import (_check_copy_ranges,
                                                                     _seg_extent)
    from terraform_provider_iterative_amd.ops.packing import SEG_CONTIG, SEG_DTYPE

    class Lib:
        def tpi_mem_range(self, ptr, base, size):
            base._obj.value, size._obj.value = 0x9000, 0x1000  # the successor's allocation
            return 0

    src = np.zeros(2, dtype=SEG_DTYPE)
    dst = np.zeros(2, dtype=SEG_DTYPE)
    src["kind"] = dst["kind"] = SEG_CONTIG
    src["ptr"], src["nbytes"] = [0x1000, 0x1800], [0x800, 0x800]
    dst["ptr"], dst["nbytes"] = [0x9000, 0x9800], [0x800, 0x800]
    owner = np.array([0, 0])
    _check_copy_ranges(src, owner, [0x1000], [0x1000], dst, Lib())  # fits exactly
    with pytest.raises(CheckpointError, match="source segment 1"):
        _check_copy_ranges(src, owner, [0x1000], [0xfff], dst, Lib())
    dst["nbytes"][1] = 0x801
    with pytest.raises(CheckpointError, match="destination segment 1"):
        _check_copy_ranges(src, owner, [0x1000], [0x1000], dst, Lib())
    # consecutive destinations in one allocation: one driver query for all of them
    from terraform_provider_iterative_amd.checkpoint.handoff import _check_destinations

    calls = []

    class CountingLib(Lib):
        def tpi_mem_range(self, ptr, base, size):
            calls.append(ptr.value)
            return Lib.tpi_mem_range(self, ptr, base, size)

    dst["nbytes"][1] = 0x800
    _check_destinations(dst, CountingLib())
    assert calls == [0x9000]
    # a strided view's extent runs from its lowest to its highest element
    v = np.zeros(1, dtype=SEG_DTYPE)[0]
    v["ptr"], v["nbytes"], v["kind"], v["elem"], v["ndim"] = 0x100, 64, 1, 4, 2
    v["sizes"][:2], v["strides"][:2] = [4, 4], [-8, 1]
    assert _seg_extent(v) == (0x100 - 3 * 8 * 4, 0x100 + 3 * 4 + 4)
