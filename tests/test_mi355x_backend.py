"""mi355x provider on a fake 8-GPU inventory (CPU-only scripts): placement, rank env,
concurrency (config 5: 4 concurrent 2-GPU tasks), auto-cleanup of leases, stop/start."""
import json
import os
import time

import pytest

from terraform_provider_iterative_amd import backends
from terraform_provider_iterative_amd.models.cloud import Cloud, Credentials, NodeCredentials
from terraform_provider_iterative_amd.models.machine_types import (MachineTypeError,
                                                                   parse_node_machine)
from terraform_provider_iterative_amd.models.values import (Environment, NotFoundError, Size, Task,
                                                            Variables)
from terraform_provider_iterative_amd.parallel.placement import (GPU, Placement,
                                                                 PlacementError, discover)
from terraform_provider_iterative_amd.utils.identifier import new_deterministic_identifier


@pytest.fixture()
def cloud(tmp_path, monkeypatch):
    # an 8-GPU MI355X node: 8 GPUs, 128 cores, 2 TB of reservable host memory
    monkeypatch.setenv("TPI_MI355X_GPUS", "0,1,2,3,4,5,6,7")
    monkeypatch.setenv("TPI_NODE_CPUS", "0-127")
    monkeypatch.setenv("TPI_NODE_MEMORY_MB", "2000000")
    return Cloud(provider="mi355x",
                 credentials=Credentials(node=NodeCredentials(state_root=str(tmp_path / "st"))))


def _task(cloud, name, script, machine="m+mi355x", parallelism=1, timeout=60):
    spec = Task(size=Size(machine=machine), parallelism=parallelism,
                environment=Environment(script=script, variables=Variables({"TPI_TASK": "true"}),
                                        timeout=timeout))
    return backends.new(cloud, new_deterministic_identifier(name), spec)


ENV_SCRIPT = "#!/bin/sh\necho \"rank=$RANK world=$WORLD_SIZE hip=$HIP_VISIBLE_DEVICES mine=$TPI_RANK_GPUS port=$MASTER_PORT\"\n"


def test_machine_types():
    assert parse_node_machine("m").gpus == 0
    assert parse_node_machine("m+mi355x").gpus == 1
    assert parse_node_machine("l+mi355x").gpus == 4
    assert parse_node_machine("xl+mi355x").gpus == 8
    assert parse_node_machine("xl+v100").gpus == 8
    mt = parse_node_machine("16-64000+mi355x*2")
    assert (mt.cpus, mt.memory_mb, mt.gpus) == (16, 64000, 2)
    with pytest.raises(MachineTypeError):
        parse_node_machine("64-1000+mi355x*9")
    with pytest.raises(MachineTypeError):
        parse_node_machine("bogus")


def test_rank_env_and_gpu_assignment(cloud):
    task = _task(cloud, "envtest", ENV_SCRIPT, machine="m+mi355x", parallelism=2)
    task.create()
    status = task.wait(20)
    assert status["succeeded"] == 2
    logs = sorted(l.split(" ", 1)[1].strip() for l in task.logs())
    gpus = task.gpus()
    assert len(gpus) == 2
    visible = ",".join(str(g) for g in gpus)
    assert logs[0].startswith("rank=0 world=2 hip=%s mine=0 " % visible)
    assert logs[1].startswith("rank=1 world=2 hip=%s mine=1 " % visible)
    # supervisor exited -> leases released
    assert Placement(cloud.state_root()).free() and len(Placement(cloud.state_root()).free()) == 8
    task.delete()


def test_four_concurrent_two_gpu_tasks(cloud, tmp_path):
    # the four tasks hold their GPUs until the test opens the gate (a fixed sleep could run
    # out under a loaded `pytest -n 8` before the fifth task was applied)
    gate = tmp_path / "gate"
    hold = ("#!/bin/sh\ni=0\nwhile [ ! -e %s ] && [ $i -lt 600 ]; do sleep 0.05; i=$((i+1)); "
            "done\necho done\n" % gate)
    tasks = [_task(cloud, "conc-%d" % i, hold, machine="16-64000+mi355x*2") for i in range(4)]
    for t in tasks:
        t.create()
    sets = [set(t.gpus()) for t in tasks]
    assert all(len(s) == 2 for s in sets)
    assert len(set().union(*sets)) == 8  # disjoint
    # a fifth task does not fit: it is queued (create succeeds, like a scaling group
    # without capacity) and starts when a GPU frees up
    extra = _task(cloud, "conc-extra", "#!/bin/sh\necho hi\n", machine="m+mi355x")
    extra.create()
    assert extra.status() == {"running": 0, "succeeded": 0, "failed": 0}  # leo read: queued
    assert extra.supervisor_running() and not extra.gpus()
    gate.write_text("go")
    for t in tasks:
        assert t.wait(30)["succeeded"] == 1
    assert extra.wait(30)["succeeded"] == 1
    codes = [e.code for e in extra.events()]
    assert codes.index("queued") < codes.index("dequeued") < codes.index("placed")
    extra.delete()
    # auto-cleanup: all GPUs free again, a new task fits
    again = _task(cloud, "after", "#!/bin/sh\necho ok\n", machine="xl+mi355x")
    again.create()
    assert sorted(again.gpus()) == list(range(8))
    assert again.wait(20)["succeeded"] == 1
    for t in tasks + [again]:
        t.delete()


def test_stop_and_start(cloud):
    task = _task(cloud, "stopstart", "#!/bin/sh\necho started\nsleep 30\n")
    task.create()
    deadline = time.time() + 10
    while not task.logs() and time.time() < deadline:
        time.sleep(0.05)
    assert task.status()["running"] == 1
    task.stop()
    st = task.status()
    assert st["running"] == 0 and st["succeeded"] == 0 and st["failed"] == 0  # no status
    assert len(Placement(cloud.state_root()).free()) == 8
    codes = [e.code for e in task.events()]
    assert "stop-requested" in codes and "rank-stopped" in codes
    task.delete()


def test_deadline_marks_failed(cloud, monkeypatch):
    monkeypatch.setenv("TPI_GRACE_SECONDS", "1")
    task = _task(cloud, "deadline", "#!/bin/sh\necho start\nsleep 30\n", timeout=1)
    task.create()
    st = task.wait(15)
    assert st["failed"] == 1
    status_files = [n for n in os.listdir(os.path.join(task.root, "reports"))
                    if n.startswith("status-")]
    report = json.load(open(os.path.join(task.root, "reports", status_files[0])))
    assert report["result"] == "timeout"
    task.delete()


def test_discover_kfd_does_not_crash(monkeypatch):
    monkeypatch.delenv("TPI_MI355X_GPUS", raising=False)
    assert isinstance(discover(), list)


def test_numa_preference(tmp_path):
    gpus = [GPU(i, numa_node=0 if i < 4 else 1) for i in range(8)]
    p = Placement(str(tmp_path), gpus)
    a = p.allocate("t1", 3)
    assert {g.numa_node for g in a} == {0}
    b = p.allocate("t2", 4)
    assert {g.numa_node for g in b} == {1}
    assert p.allocate("t1", 3) == a  # idempotent
    assert p.release("t1") == 3


def test_control_socket(cloud):
    """Supervisor control API: ping / live state / unknown / stop."""
    task = _task(cloud, "control", "#!/bin/sh\necho started\nsleep 30\n", parallelism=2)
    task.create()
    deadline = time.time() + 10
    while not task.logs() and time.time() < deadline:
        time.sleep(0.05)
    pong = task.control("ping")
    assert pong["ok"] and pong["pid"] > 0 and pong["task_id"] == task.id
    assert os.stat(os.path.join(task.sup_dir, "control.sock")).st_mode & 0o077 == 0
    state = task.control("state")
    assert [r["rank"] for r in state["ranks"]] == [0, 1]
    assert all(r["state"] == "running" and r["pid"] > 0 for r in state["ranks"])
    assert task.control("bogus")["ok"] is False
    task.stop()  # goes through the socket
    assert task.control("ping") is None  # socket removed at exit
    assert not os.path.exists(os.path.join(task.sup_dir, "control.sock"))
    codes = [(e.code, e.description) for e in task.events()]
    assert any(c == "stop-requested" and "control socket" in d for c, d in codes)
    task.delete()


def test_preempt_one_rank_over_control_socket(cloud):
    """`leo preempt --rank 1`: only rank 1 is signalled; the coupled gang is respawned."""
    script = "#!/bin/sh\necho \"up $RANK $TPI_MACHINE_IDENTITY\"\nsleep 30\n"
    task = _task(cloud, "preemptone", script, parallelism=2)
    task.create()
    deadline = time.time() + 10
    while sum(log.count("up ") for log in task.logs()) < 2 and time.time() < deadline:
        time.sleep(0.05)
    with pytest.raises(NotFoundError):
        task.preempt(rank=7)  # no such rank
    task.preempt(rank=1)
    deadline = time.time() + 15
    state = {}
    while time.time() < deadline:
        state = task.control("state") or {}
        if state.get("ranks") and all(r["restarts"] == 1 and r["state"] == "running"
                                      for r in state["ranks"]):
            break
        time.sleep(0.05)
    assert [r["restarts"] for r in state["ranks"]] == [1, 1], state
    events = [(e.code, e.description) for e in task.events()]
    assert ("preempt-requested", ["rank 1", "control socket"]) in events
    task.stop()
    task.delete()


def test_bench_concurrent_config5(monkeypatch, tmp_path):
    """bench/bench_concurrent.py (config 5) on 8 logical slots: disjoint sets, refusal,
    lease auto-cleanup."""
    import importlib.util

    monkeypatch.setenv("TPI_MI355X_GPUS", "0,1,2,3,4,5,6,7")
    monkeypatch.setenv("TMPDIR", str(tmp_path))
    spec = importlib.util.spec_from_file_location(
        "bench_concurrent", os.path.join(os.path.dirname(os.path.dirname(__file__)), "bench",
                                         "bench_concurrent.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    out = mod.run(tasks=4, gpus_per_task=2, sleep=0.2)
    assert out["disjoint"] and out["cpus_disjoint"] and out["all_succeeded"]
    assert out["fifth_queued"] and out["fifth_succeeded"] and out["queued_start_s"] < 5
    assert out["reused_all_gpus"]
    assert len(out["first_log_s"]) == 4
