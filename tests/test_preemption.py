"""Preempt-recover on the node runtime (config 4 control flow, CPU tensors):
SIGTERM mid-task -> rank checkpoints (pack -> host region) -> supervisor respawns it with a
new machine identity -> successor restores and finishes.  The reference's equivalent is spot
recovery with the workdir restored from the bucket (machine-script.sh.tpl:89,118-124)."""
import os
import sys
import time

import pytest

from terraform_provider_iterative_amd import backends
from terraform_provider_iterative_amd.models.cloud import Cloud, Credentials, NodeCredentials
from terraform_provider_iterative_amd.models.values import Environment, Task, Variables
from terraform_provider_iterative_amd.utils.identifier import new_deterministic_identifier

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

TRAIN = r'''#!%(python)s
import os, sys, time
sys.path.insert(0, %(root)r)
import torch
from terraform_provider_iterative_amd.checkpoint import Checkpointer, preemption

state = {"w": torch.zeros(4096), "step": torch.zeros((), dtype=torch.int64),
         "m": torch.randn(64, 32).t()}
spill = os.path.join(os.environ["TPI_DATA_DIRECTORY"], ".spill")  # survives the rank
ck = Checkpointer(state, path=spill, tile_bytes=4096)
meta = preemption.resume(ck)
start = int(state["step"])
print(("resumed %%d %%s" %% (start, meta.get("reason"))) if meta else "fresh", flush=True)
preemption.register(ck)
preemption.on_preempt(lambda: {"step": int(state["step"])})
preemption.install()
for step in range(start, %(steps)d):
    state["w"].fill_(step + 1)
    state["step"].fill_(step + 1)
    print("step", step + 1, flush=True)
    time.sleep(0.05)
print("final", int(state["w"][0].item()), int(state["step"]), flush=True)
'''


@pytest.fixture()
def cloud(tmp_path):
    return Cloud(provider="local",
                 credentials=Credentials(node=NodeCredentials(state_root=str(tmp_path / "st"))))


def _wait_for(task, text, timeout=60, ranks=1):
    """Until ``text`` is in the logs of ``ranks`` ranks."""
    deadline = time.time() + timeout
    while time.time() < deadline:
        if sum(text in log for log in task.logs()) >= ranks:
            return True
        time.sleep(0.05)
    raise AssertionError("%r never appeared in logs: %s" % (text, task.logs()))


@pytest.mark.parametrize("how", ["supervisor", "rank-sigterm", "no-handoff"])
def test_preempt_checkpoint_respawn_resume(cloud, how):
    script = TRAIN % {"python": sys.executable, "root": ROOT, "steps": 40}
    env = {"TPI_TASK": "true"}
    if how == "no-handoff":  # successor waits for the old process to exit
        env["TPI_EARLY_HANDOFF"] = "0"
    spec = Task(environment=Environment(script=script, timeout=300, variables=Variables(env)))
    task = backends.new(cloud, new_deterministic_identifier("preempt-" + how), spec)
    task.create()
    _wait_for(task, "step 5")
    if how != "rank-sigterm":
        task.preempt()  # leo preempt: SIGUSR1 -> supervisor SIGTERMs the ranks
    else:  # an external agent SIGTERMs the rank process directly
        import json
        import signal

        state = json.load(open(os.path.join(task.root, "supervisor", "state.json")))
        os.kill(state["ranks"][0]["pid"], signal.SIGTERM)
    status = task.wait(90)
    logs = task.logs()
    assert status["succeeded"] == 1 and status["failed"] == 0, (status, logs)
    assert len(logs) == 2, logs  # one log per machine identity, like the reference
    assert "preemption checkpoint saved" in logs[0]
    assert "resumed" in logs[1] and "preempted" in logs[1]
    resumed_at = int(logs[1].split("resumed ")[1].split()[0])
    assert resumed_at >= 5
    assert "final 40 40" in logs[1]
    codes = [e.code for e in task.events()]
    assert "respawn" in codes
    if how == "no-handoff":
        assert "rank-preempted" in codes and "rank-released" not in codes
    else:  # early hand-off: respawned on "released", the old process reaped afterwards
        assert "rank-released" in codes and "rank-released-exit" in codes
        # streamed hand-off (default): released when the spill starts, the successor
        # restores behind it
        assert "checkpoint-streaming" in codes and "checkpoint-released" not in codes
        assert codes.index("rank-released") < codes.index("respawn")
        # the supervisor's SIGUSR2 ("successor restored") ends the predecessor's linger; it
        # must not kill it: the spill finishes (checkpoint-saved) and the exit is 143
        exits = [e for e in task.events() if e.code == "rank-released-exit"]
        assert exits and "code 143" in exits[0].description, exits[0].description
        assert "predecessor-exit" in codes
        assert codes.index("checkpoint-saved") < codes.index("rank-released-exit")
    # phase journal: start -> first output -> preempt -> saved / respawn -> restored
    for phase in ("rank-start", "rank-first-output", "preempt-signal", "checkpoint-saved",
                  "checkpoint-restored"):
        assert phase in codes, (phase, codes)
    assert codes.index("checkpoint-saved") < codes.index("checkpoint-restored")
    assert codes.index("respawn") < codes.index("checkpoint-restored")
    saved = [e for e in task.events() if e.code == "checkpoint-saved"][0]
    assert saved.description[0] == "rank 0" and saved.description[-1].endswith("GB/s")
    task.delete()


def test_successor_starts_while_released_rank_exits(cloud):
    # the released rank lingers 2 s after "released" (a slow teardown): its successor must
    # already be running, and the old process is still reaped and journalled
    slow = TRAIN.replace("preemption.install()", "_orig = preemption.notify_released\n"
                         "def _slow():\n    sent = _orig()\n    time.sleep(2)\n    return sent\n"
                         "preemption.notify_released = _slow\npreemption.install()")
    script = slow % {"python": sys.executable, "root": ROOT, "steps": 30}
    spec = Task(environment=Environment(script=script, timeout=300,
                                        variables=Variables({"TPI_TASK": "true"})))
    task = backends.new(cloud, new_deterministic_identifier("preempt-overlap"), spec)
    task.create()
    _wait_for(task, "step 3")
    task.preempt()
    status = task.wait(90)
    assert status["succeeded"] == 1, task.logs()
    events = task.events()
    released_exit = [e.time for e in events if e.code == "rank-released-exit"]
    starts = [e.time for e in events if e.code == "rank-start"]
    assert len(starts) == 2 and released_exit
    assert starts[1] < released_exit[0]
    assert "final 30 30" in task.logs()[1]
    task.delete()


STANDBY = TRAIN.replace("spill = os.path.join(", "activated = preemption.standby()\nspill = os.path.join(")
STANDBY = STANDBY.replace('print(("resumed', 'print("activated" if activated else "cold", flush=True)\nprint(("resumed')


def test_warm_standby_takes_over(cloud, monkeypatch):
    monkeypatch.setenv("TPI_WARM_STANDBY", "1")
    script = STANDBY % {"python": sys.executable, "root": ROOT, "steps": 30}
    spec = Task(environment=Environment(script=script, timeout=300,
                                        variables=Variables({"TPI_TASK": "true"})))
    task = backends.new(cloud, new_deterministic_identifier("preempt-standby"), spec)
    task.create()
    _wait_for(task, "step 3")
    task.preempt()
    status = task.wait(90)
    logs = task.logs()
    assert status["succeeded"] == 1 and len(logs) == 2, (status, logs)
    assert "cold" in logs[0] and "activated" in logs[1] and "final 30 30" in logs[1]
    events = task.events()
    codes = [e.code for e in events]
    for code in ("standby-start", "standby-activated", "rank-released", "respawn"):
        assert code in codes, (code, codes)
    assert "standby-discarded" not in codes
    starts = [e for e in events if e.code == "rank-start"]
    assert len(starts) == 2 and "warm standby" in starts[1].description
    task.delete()


def test_hot_standby_restores_behind_the_streamed_spill(cloud, monkeypatch):
    """TPI_WARM_STANDBY=hot: the successor runs (imports done) before any preemption; the
    preempted rank releases it when its spill *starts* and it resumes from the stream."""
    monkeypatch.setenv("TPI_WARM_STANDBY", "hot")
    script = STANDBY % {"python": sys.executable, "root": ROOT, "steps": 30}
    spec = Task(environment=Environment(script=script, timeout=300,
                                        variables=Variables({"TPI_TASK": "true"})))
    task = backends.new(cloud, new_deterministic_identifier("preempt-hot"), spec)
    task.create()
    _wait_for(task, "step 3")
    deadline = time.time() + 30
    while time.time() < deadline and "standby-start" not in [e.code for e in task.events()]:
        time.sleep(0.05)
    task.preempt()
    status = task.wait(90)
    logs = task.logs()
    assert status["succeeded"] == 1, (status, logs)
    assert any("activated" in l and "final 30 30" in l for l in logs), logs
    codes = [e.code for e in task.events()]
    assert codes.index("standby-start") < codes.index("preempt-requested")
    for code in ("standby-activated", "checkpoint-streaming", "rank-released", "respawn",
                 "checkpoint-restored"):
        assert code in codes, (code, codes)
    # the successor's own hot standby waits until it restored (no start-up next to a restore)
    starts = [i for i, c in enumerate(codes) if c == "standby-start"]
    assert all(i > codes.index("checkpoint-restored") for i in starts[1:]), codes
    task.delete()


def test_hot_standby_gang_of_two(cloud, monkeypatch):
    """Two coupled ranks, each with a hot standby: preempting rank 1 takes the gang down,
    both stream their spills, both standbys take over and finish from their own spill."""
    monkeypatch.setenv("TPI_WARM_STANDBY", "hot")
    script = STANDBY.replace('".spill")', '".spill-" + os.environ["RANK"])') % {
        "python": sys.executable, "root": ROOT, "steps": 30}
    spec = Task(parallelism=2,
                environment=Environment(script=script, timeout=300,
                                        variables=Variables({"TPI_TASK": "true"})))
    task = backends.new(cloud, new_deterministic_identifier("preempt-hot-gang"), spec)
    task.create()
    # both ranks in their loops (handler installed): a rank still starting up when the gang
    # is preempted dies without a save, and its standby rightly starts fresh
    _wait_for(task, "step 3", ranks=2)
    # each rank's hot standby starts once the rank has announced itself from standby(); under
    # a loaded machine (the suite on 8 workers) that can take longer than the steps do
    deadline = time.time() + 120
    while time.time() < deadline and \
            sum(e.code == "standby-start" for e in task.events()) < 2:
        time.sleep(0.05)
    assert sum(e.code == "standby-start" for e in task.events()) == 2, \
        [e.code for e in task.events()]
    task.preempt(rank=1)
    status = task.wait(180)
    logs = task.logs()
    assert status["succeeded"] == 2, (status, logs)
    finished = [l for l in logs if "activated" in l and "final 30 30" in l]
    assert len(finished) == 2, logs
    codes = [e.code for e in task.events()]
    trail = "\n".join("%s %s" % (e.code, " ".join(e.description)) for e in task.events())
    assert codes.count("standby-activated") == 2, trail
    assert codes.count("checkpoint-streaming") + codes.count("checkpoint-released") >= 2, trail
    task.delete()


def test_unused_standby_is_discarded(cloud, monkeypatch):
    monkeypatch.setenv("TPI_WARM_STANDBY", "1")
    # stop arrives while the preempted rank is still releasing: its standby must not run
    slow = STANDBY.replace("preemption.install()", "_orig = preemption.notify_released\n"
                           "def _slow():\n    time.sleep(3)\n    return _orig()\n"
                           "preemption.notify_released = _slow\npreemption.install()")
    script = slow % {"python": sys.executable, "root": ROOT, "steps": 30}
    spec = Task(environment=Environment(script=script, timeout=300,
                                        variables=Variables({"TPI_TASK": "true"})))
    task = backends.new(cloud, new_deterministic_identifier("preempt-standby-stop"), spec)
    task.create()
    _wait_for(task, "step 3")
    task.preempt()
    deadline = time.time() + 30
    while time.time() < deadline and "standby-start" not in [e.code for e in task.events()]:
        time.sleep(0.05)
    task.stop()
    task.wait(60)
    codes = [e.code for e in task.events()]
    assert "standby-start" in codes and "standby-discarded" in codes, codes
    assert "standby-activated" not in codes and not task.supervisor_running()
    task.delete()


def test_machine_logs_journal(cloud):
    # TPI_MACHINE_LOGS (machine-script.sh.tpl:109): reports/machine-<uuid> next to task-<uuid>
    spec = Task(environment=Environment(script="#!/bin/sh\necho hi\n", timeout=60,
                                        variables=Variables({"TPI_MACHINE_LOGS": "1"})))
    task = backends.new(cloud, new_deterministic_identifier("machine-logs"), spec)
    task.create()
    status = task.wait(60)
    assert status["succeeded"] == 1
    names = os.listdir(task.reports_dir)
    machine = [n for n in names if n.startswith("machine-")]
    assert machine and ("task-" + machine[0][len("machine-"):]) in names
    text = open(os.path.join(task.reports_dir, machine[0])).read()
    assert "tpi-supervisor: rank-start rank 0" in text
    assert len(task.logs()) == 1 and "hi" in task.logs()[0]  # machine-* is not a task log
    task.delete()


@pytest.fixture()
def fresh_preemption(monkeypatch):
    from terraform_provider_iterative_amd.checkpoint import preemption

    monkeypatch.setattr(preemption, "_registered", [])
    monkeypatch.setattr(preemption, "_callbacks", [])
    monkeypatch.setattr(preemption, "_tick_pending", {})
    monkeypatch.setattr(preemption, "_tick_last", None)
    monkeypatch.setattr(preemption, "_agreement", None)
    monkeypatch.setattr(preemption, "_boundary_seen", False)
    monkeypatch.setattr(preemption, "_last_step", None)
    return preemption


@pytest.mark.parametrize("mode", ["async", "sync"])
def test_periodic_tick_checkpoints_at_the_interval(tmp_path, monkeypatch, fresh_preemption, mode):
    """TPI_SYNC_INTERVAL cadence (machine-script.sh.tpl:118-124): a rank that dies without a
    SIGTERM still leaves the last periodic checkpoint behind."""
    import json

    import torch

    from terraform_provider_iterative_amd.checkpoint import Checkpointer

    pre = fresh_preemption
    events = tmp_path / "events.jsonl"
    monkeypatch.setenv("TPI_SYNC_INTERVAL", "0.1")
    monkeypatch.setenv("TPI_SYNC_MODE", mode)
    monkeypatch.setenv("TPI_EVENTS_FILE", str(events))
    state = {"w": torch.zeros(5000), "step": torch.zeros((), dtype=torch.int64)}
    spill = str(tmp_path / "spill")
    ck = Checkpointer(state, path=spill, tile_bytes=4096)
    pre.register(ck)
    pre.on_preempt(lambda: {"step": int(state["step"])})
    assert pre.tick() is False  # arms the timer
    state["w"].fill_(3)
    state["step"].fill_(1)
    assert pre.tick() is False  # not due yet
    time.sleep(0.12)
    assert pre.tick({"extra": "x"}) is True
    ck.wait_pending()
    meta = ck.header()["metadata"]
    assert meta["step"] == 1 and meta["reason"] == "periodic" and meta["extra"] == "x"
    assert pre.tick() is False  # interval restarts
    monkeypatch.setenv("TPI_SYNC_INTERVAL", "0")
    time.sleep(0.12)
    assert pre.tick() is False  # 0 disables the cadence
    assert pre.tick(force=True) is True
    ck.wait_pending()
    ck.close()
    # the "crashed" rank's successor finds the periodic checkpoint
    fresh = {"w": torch.zeros(5000), "step": torch.zeros((), dtype=torch.int64)}
    ck2 = Checkpointer(fresh, path=spill, tile_bytes=4096)
    assert pre.resume(ck2)["reason"] == "periodic"
    assert torch.equal(fresh["w"], state["w"]) and int(fresh["step"]) == 1
    ck2.close()
    lines = [json.loads(l) for l in events.read_text().splitlines()]
    synced = [l for l in lines if l["code"] == "checkpoint-synced"]
    assert len(synced) == 2
    assert synced[0]["description"][1] == ("incremental" if mode == "sync" else "async")
