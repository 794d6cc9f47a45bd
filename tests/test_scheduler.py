"""Node scheduling: reservations of GPUs + cores + memory, the queue, spot reclaim, and the
machine-type limits the supervisor enforces.

Reference behaviour being mapped: a scaling group keeps ``desired = parallelism`` until the
cloud has capacity and consumers show ``queued`` meanwhile
(``resource_auto_scaling_group.go:51-106,188-199``; ``cmd/leo/read/read.go:164-176``); spot
capacity (``spot >= 0``) is reclaimable and replaced when capacity returns; the k8s Job turns
the machine type's cpu/memory/disk into pod limits (``resource_job.go:107-118``).
"""
import os
import sys
import time

import pytest

from terraform_provider_iterative_amd import backends
from terraform_provider_iterative_amd.models.cloud import Cloud, Credentials, NodeCredentials
from terraform_provider_iterative_amd.models.values import (Environment, Size, Task,
                                                            Variables)
from terraform_provider_iterative_amd.parallel.placement import (GPU, Placement,
                                                                 PlacementBusy, Request)
from terraform_provider_iterative_amd.utils.identifier import new_deterministic_identifier
from terraform_provider_iterative_amd.utils.logger import reduce_status

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cloud(tmp_path, provider="mi355x"):
    return Cloud(provider=provider,
                 credentials=Credentials(node=NodeCredentials(state_root=str(tmp_path / "st"))))


def _task(cloud, name, script, machine="m+mi355x", parallelism=1, spot=-1.0, env=None,
          disk=-1, timeout=120):
    spec = Task(size=Size(machine=machine, storage=disk), parallelism=parallelism, spot=spot,
                environment=Environment(script=script, timeout=timeout,
                                        variables=Variables(dict(env or {}, TPI_TASK="true"))))
    return backends.new(cloud, new_deterministic_identifier(name), spec)


@pytest.fixture()
def node(monkeypatch):
    """An 8-GPU node with 2 sockets (GPUs 0-3 on node 0), 128 cores, 1 TB for tasks."""
    monkeypatch.setenv("TPI_NODE_CPUS", "0-127")
    monkeypatch.setenv("TPI_NODE_MEMORY_MB", "1000000")
    gpus = [GPU(i, gfx="gfx950", numa_node=0 if i < 4 else 1,
                cpus=list(range(0, 64)) if i < 4 else list(range(64, 128))) for i in range(8)]
    return gpus


def test_reservations_give_disjoint_numa_local_cores(tmp_path, node):
    p = Placement(str(tmp_path), node)
    allocs = [p.reserve(Request(task="t%d" % i, parallelism=2, gpus_per_rank=1,
                                cpus_per_rank=16, memory_mb_per_rank=100000))
              for i in range(4)]
    cores = [c for a in allocs for rank in a.rank_cpus for c in rank]
    assert len(cores) == len(set(cores)) == 4 * 2 * 16  # config 5: disjoint core sets
    for a in allocs:
        for rank, gpu in enumerate(a.gpus):  # each rank on its GPU's socket
            local = set(node[gpu].cpus)
            assert set(a.rank_cpus[rank]) <= local, (a, rank)
    assert sum(a.memory_mb for a in allocs) == 800000
    # GPUs are all taken: a fifth waits; over-memory would wait too
    with pytest.raises(PlacementBusy, match="GPUs"):
        p.reserve(Request(task="t4", gpus_per_rank=1))
    p.release("t0")
    with pytest.raises(PlacementBusy, match="memory"):
        p.reserve(Request(task="big", parallelism=1, gpus_per_rank=1,
                          memory_mb_per_rank=500000))
    assert p.reserve(Request(task="small", gpus_per_rank=1, memory_mb_per_rank=100000)).gpus
    # idempotent
    assert p.reserve(Request(task="t1", parallelism=2, gpus_per_rank=1)).gpus == allocs[1].gpus


def test_queue_order_on_demand_before_spot_then_fifo(tmp_path, node):
    p = Placement(str(tmp_path), node)
    p.reserve(Request(task="holder", parallelism=8, gpus_per_rank=1))
    p.enqueue(Request(task="spot-a", gpus_per_rank=1, spot=True), waiter_pid=os.getpid())
    time.sleep(0.01)
    p.enqueue(Request(task="od-b", gpus_per_rank=1), waiter_pid=os.getpid())
    time.sleep(0.01)
    p.enqueue(Request(task="od-c", gpus_per_rank=1), waiter_pid=os.getpid())
    assert [e["task"] for e in p.queue()] == ["od-b", "od-c", "spot-a"]
    p.release("holder")
    with pytest.raises(PlacementBusy, match="queued behind od-b"):
        p.reserve(Request(task="od-c", gpus_per_rank=1))  # free GPUs, but not its turn
    assert p.reserve(Request(task="od-b", gpus_per_rank=1)).gpus
    assert p.reserve(Request(task="od-c", gpus_per_rank=1)).gpus
    assert p.reserve(Request(task="spot-a", gpus_per_rank=1, spot=True)).gpus
    assert p.queue() == []


def test_victims_are_the_fewest_spot_tasks_that_make_room(tmp_path, node):
    p = Placement(str(tmp_path), node)
    p.reserve(Request(task="od", parallelism=4, gpus_per_rank=1))
    p.reserve(Request(task="spot-small", gpus_per_rank=1, spot=True))
    p.reserve(Request(task="spot-big", parallelism=3, gpus_per_rank=1, spot=True))
    want = Request(task="new", parallelism=3, gpus_per_rank=1)
    assert [v["task"] for v in p.victims(want)] == ["spot-big"]
    want4 = Request(task="new4", parallelism=4, gpus_per_rank=1)
    assert sorted(v["task"] for v in p.victims(want4)) == ["spot-big", "spot-small"]
    assert p.victims(Request(task="x", parallelism=5, gpus_per_rank=1)) == []  # od holds 4
    assert p.victims(Request(task="s", gpus_per_rank=4, spot=True)) == []  # spot never reclaims


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
print("start", start, "gpus", os.environ.get("HIP_VISIBLE_DEVICES"), flush=True)
preemption.register(ck)
preemption.install()
for step in range(start, %(steps)d):
    state["w"] += 1  # not idempotent: a torn or repeated step shows in the final value
    time.sleep(0.05)
    preemption.step(step + 1)
print("final", int(state["w"][0]), flush=True)
'''


def test_on_demand_task_reclaims_a_spot_task_which_resumes_later(tmp_path, monkeypatch):
    """1-GPU node: a spot task runs; an on-demand task arrives, is queued, reclaims the GPU
    (the spot task checkpoints at a step boundary and goes back to the queue), runs, and the
    spot task resumes from its checkpoint once the GPU is free.  leo read's status goes
    running -> queued -> running -> succeeded for the spot task, queued -> running ->
    succeeded for the on-demand one."""
    monkeypatch.setenv("TPI_MI355X_GPUS", "0")
    monkeypatch.setenv("TPI_NODE_CPUS", "0-31")
    monkeypatch.setenv("TPI_NODE_MEMORY_MB", "512000")
    cloud = _cloud(tmp_path)
    spot = _task(cloud, "spot", SPOT % {"python": sys.executable, "root": ROOT, "steps": 40},
                 spot=0)
    spot.create()
    deadline = time.time() + 60
    while time.time() < deadline and "start 0" not in "".join(spot.logs()):
        time.sleep(0.05)
    time.sleep(0.3)
    od = _task(cloud, "ondemand", "#!/bin/sh\necho on-demand on GPU $HIP_VISIBLE_DEVICES\n"
                                  "sleep 1\necho done\n")
    # the spot task is handed back within ~0.1 s of the reclaim (save, release, requeue):
    # observe its "running" before the on-demand task is applied
    seen = {"spot": [reduce_status(spot.status(), 1)], "od": []}
    od.create()
    deadline = time.time() + 120
    while time.time() < deadline:
        for name, task in (("spot", spot), ("od", od)):
            st = reduce_status(task.status(), 1)
            if not seen[name] or seen[name][-1] != st:
                seen[name].append(st)
        if not spot.supervisor_running() and not od.supervisor_running():
            break
        time.sleep(0.02)
    assert spot.status()["succeeded"] == 1 and od.status()["succeeded"] == 1, (
        seen, spot.logs(), od.logs())
    assert seen["od"] == ["queued", "running", "succeeded"], seen
    assert seen["spot"] == ["running", "queued", "running", "succeeded"], seen
    logs = spot.logs()
    assert len(logs) == 2, logs
    resumed = int(logs[1].split("start ")[1].split()[0])
    assert 0 < resumed < 40 and "final 40" in logs[1], logs
    spot_codes = [e.code for e in spot.events()]
    for code in ("requeue-requested", "preempt-boundary", "rank-requeued", "requeued",
                 "queued", "dequeued"):
        assert code in spot_codes, (code, spot_codes)
    od_codes = [e.code for e in od.events()]
    assert od_codes.index("queued") < od_codes.index("reclaim") < od_codes.index("placed")
    # the on-demand task ran while the spot task was waiting
    t_od = [e.time for e in od.events() if e.code == "rank-exit"][0]
    t_spot2 = [e.time for e in spot.events() if e.code == "dequeued"][0]
    assert t_od <= t_spot2
    assert Placement(cloud.state_root()).queue() == []
    od.delete()
    spot.delete()


def test_stop_a_queued_task_leaves_the_queue(tmp_path, monkeypatch):
    monkeypatch.setenv("TPI_MI355X_GPUS", "0")
    monkeypatch.setenv("TPI_NODE_CPUS", "0-31")
    monkeypatch.setenv("TPI_NODE_MEMORY_MB", "512000")
    cloud = _cloud(tmp_path)
    first = _task(cloud, "holder", "#!/bin/sh\nsleep 30\n")
    first.create()
    second = _task(cloud, "waiting", "#!/bin/sh\necho never\n")
    second.create()
    assert Placement(cloud.state_root()).position(second.id) == 0
    second.stop()
    assert not second.supervisor_running()
    assert Placement(cloud.state_root()).queue() == []
    first.delete()
    second.delete()
    assert "never" not in "".join(second.logs())


def test_memory_limit_kills_the_rank_like_an_oom(tmp_path):
    """machine 1-200 (200 MB): a rank that allocates 600 MB is killed and fails."""
    cloud = _cloud(tmp_path, "local")
    script = ("#!%s\nimport time\nprint('up', flush=True)\nx = bytearray(600 << 20)\n"
              "time.sleep(30)\nprint('survived')\n" % sys.executable)
    task = _task(cloud, "oom", script, machine="1-200")
    task.create()
    status = task.wait(30)
    assert status["failed"] == 1, (status, task.logs())
    assert "survived" not in "".join(task.logs())
    codes = [e.code for e in task.events()]
    assert "rank-oom-killed" in codes and "rank-oom" in codes
    import json

    reports = [f for f in os.listdir(task.reports_dir) if f.startswith("status-")]
    assert json.load(open(os.path.join(task.reports_dir, reports[0])))["result"] == "oom"
    task.delete()


def test_disk_limit_fails_the_task(tmp_path):
    """disk_size: the workdir may not outgrow it (ephemeral-storage eviction)."""
    cloud = _cloud(tmp_path, "local")
    script = ("#!/bin/sh\necho writing\nhead -c 3000000 /dev/urandom > big.bin\nsync\n"
              "sleep 20\necho survived\n")
    task = _task(cloud, "disk", script, machine="s", disk=1,
                 env={"TPI_DISK_LIMIT_MB": "2", "TPI_DISK_CHECK_INTERVAL": "0.2"})
    task.create()
    status = task.wait(30)
    assert status["failed"] == 1, (status, task.logs())
    assert "survived" not in "".join(task.logs())
    assert "disk-limit" in [e.code for e in task.events()]
    task.delete()


def test_limit_mode_caps_affinity_to_the_machine_cores(tmp_path, monkeypatch):
    monkeypatch.setenv("TPI_NODE_CPUS", "0-7")
    cloud = _cloud(tmp_path, "local")
    task = _task(cloud, "affinity", "#!%s\nimport os\nprint(sorted(os.sched_getaffinity(0)))\n"
                 % sys.executable, machine="2-1000", parallelism=2)
    task.create()
    assert task.wait(30)["succeeded"] == 2
    sets = [eval(l.split("Z ", 1)[1]) for l in task.logs()]
    available = sorted(os.sched_getaffinity(0))
    for s in sets:
        assert len(s) == min(2, len(available)) or s == available, sets
    task.delete()


def test_memory_shared_with_forked_workers_counts_once(tmp_path):
    """machine 1-400 (400 MB): a rank touches 250 MB and forks three workers that share those
    pages copy-on-write.  Their resident sets add up to ~1 GB, over the limit, but the
    proportional set size that decides the kill counts the shared pages once: no OOM."""
    cloud = _cloud(tmp_path, "local")
    script = ("#!%s\nimport os, time\nx = bytearray(250 << 20)\nfor i in range(0, len(x), 4096):\n"
              "    x[i] = 1\nkids = []\nfor _ in range(3):\n    pid = os.fork()\n"
              "    if pid == 0:\n        time.sleep(2.5)\n        os._exit(0)\n"
              "    kids.append(pid)\n"
              "print('up', flush=True)\ntime.sleep(2.5)\n"
              "for k in kids:\n    os.waitpid(k, 0)\nprint('survived', flush=True)\n"
              % sys.executable)
    task = _task(cloud, "shared", script, machine="1-400")
    task.create()
    status = task.wait(30)
    assert status["succeeded"] == 1, (status, task.logs())
    assert "survived" in "".join(task.logs())
    assert "rank-oom-killed" not in [e.code for e in task.events()]
    task.delete()


REGION_RANK = r'''#!%(python)s
import os, sys, time
sys.path.insert(0, %(root)r)
if not %(announce)r:
    os.environ.pop("TPI_REGIONS_FILE", None)  # an unannounced mapping is working set
from terraform_provider_iterative_amd.checkpoint.host import HostRegion
region = HostRegion(%(mb)d << 20, os.path.join(os.environ["TPI_DATA_DIRECTORY"], ".spill"))
region.array()[:] = 7  # resident: every page touched
print("up", flush=True)
time.sleep(2.5)  # > 2 polls of the limit
print("survived", flush=True)
'''


@pytest.mark.parametrize("announce", [True, False], ids=["region", "working-set"])
def test_checkpoint_region_larger_than_the_memory_limit_survives(tmp_path, monkeypatch,
                                                                 announce):
    """a GPU machine type's memory (e.g. m+t4 -> 16 GB) is smaller than one GPU's
    checkpoint.  A spill region the rank announced (checkpoint/host.py does for every region)
    is not counted against the limit; the same mapping unannounced is, and is killed."""
    monkeypatch.setenv("TPI_MI355X_GPUS", "0")
    monkeypatch.setenv("TPI_NODE_CPUS", "0-31")
    monkeypatch.setenv("TPI_NODE_MEMORY_MB", "512000")
    cloud = _cloud(tmp_path)
    script = REGION_RANK % {"python": sys.executable, "root": ROOT, "mb": 700,
                            "announce": announce}
    task = _task(cloud, "region-" + str(announce), script, machine="1-400+mi355x*1",
                 env={"TPI_MEMORY_CHECK_INTERVAL": "0.2"})
    task.create()
    status = task.wait(60)
    logs = "".join(task.logs())
    codes = [e.code for e in task.events()]
    if announce:
        assert status["succeeded"] == 1 and "survived" in logs, (status, logs, codes)
        assert "rank-oom-killed" not in codes
    else:
        assert status["failed"] == 1 and "survived" not in logs, (status, logs)
        assert "rank-oom-killed" in codes
    task.delete()


def test_supervisor_puts_each_rank_in_a_memory_cgroup(tmp_path):
    """The hard cap: a cgroup per rank with memory.max = limit + headroom, the rank inside it
    before exec (a directory standing in for the cgroup hierarchy)."""
    from tests.test_supervisor import _events, _run, _spec

    from terraform_provider_iterative_amd import _build

    root = tmp_path / "cgroot"
    root.mkdir()
    (root / "cgroup.controllers").write_text("memory\n")  # looks like cgroup v2
    task, spec = _spec(tmp_path, "#!/bin/sh\necho pid $$\n", parallelism=2,
                       limits={"rank_memory_mb": 1000, "cgroup": str(root),
                               "cgroup_headroom_mb": 24})
    _run(_build.build_supervisor(), spec)
    events = _events(task)
    cg = [e for e in events if e["code"] == "memory-cgroup"]
    assert cg and cg[0]["description"][:2] == ["v2", str(root)], events
    dirs = sorted(d for d in os.listdir(root) if d.startswith("tpi-"))
    assert len(dirs) == 2 and dirs[0].endswith("-r0") and dirs[1].endswith("-r1")
    for d in dirs:
        assert (root / d / "memory.max").read_text() == str((1000 + 24) << 20)
    pids = {int(l.split()[-1]) for f in os.listdir(task / "reports") if f.startswith("task-")
            for l in (task / "reports" / f).read_text().splitlines()}
    joined = {int((root / d / "cgroup.procs").read_text().split()[0]) for d in dirs}
    assert joined == pids, (joined, pids)


def _cgroup_writable() -> bool:
    if os.geteuid() != 0:
        return False
    probe = None
    if os.path.exists("/sys/fs/cgroup/memory/memory.limit_in_bytes"):
        probe = "/sys/fs/cgroup/memory/tpi-probe-%d" % os.getpid()
    if probe is None:
        return False
    try:
        os.mkdir(probe)
        os.rmdir(probe)
        return True
    except OSError:
        return False


@pytest.mark.skipif(not _cgroup_writable(), reason="no writable memory cgroup hierarchy")
def test_fast_allocation_over_the_limit_is_stopped_by_the_kernel(tmp_path):
    """machine 1-1000 (1 GB): a rank that writes 2 GB in well under a poll interval is stopped
    by its memory cgroup (the poll is set to 30 s here, so only the kernel can act)."""
    cloud = _cloud(tmp_path, "local")
    script = ("#!%s\nimport time\nprint('up', flush=True)\nt = time.time()\n"
              "x = b'\\x01' * (2 << 30)\nprint('survived %%.3f s' %% (time.time() - t), flush=True)\n"
              "time.sleep(5)\n" % sys.executable)
    task = _task(cloud, "cg-oom", script, machine="1-1000",
                 env={"TPI_MEMORY_CHECK_INTERVAL": "30"})
    task.create()
    status = task.wait(30)
    logs = "".join(task.logs())
    assert status["failed"] == 1 and "survived" not in logs, (status, logs)
    events = task.events()
    assert "memory-cgroup" in [e.code for e in events]
    kills = [e for e in events if e.code == "rank-oom-killed"]
    assert kills and "memory cgroup cap" in kills[0].description, kills
    import json

    reports = [f for f in os.listdir(task.reports_dir) if f.startswith("status-")]
    assert json.load(open(os.path.join(task.reports_dir, reports[0])))["result"] == "oom"
    task.delete()
    assert not [d for d in os.listdir("/sys/fs/cgroup/memory") if d.startswith("tpi-" + task.id)]


def test_fast_allocation_is_stopped_by_the_fast_poll_without_a_cgroup(tmp_path):
    """where the kernel cap is refused (the MI355X box), the statm poll of each
    rank's process tree (20 ms) is the guard.  machine 1-1000 (1 GB), cgroup forced off: a rank
    writing 2 GB as fast as it can is killed before it passes 1.5 GB."""
    cloud = _cloud(tmp_path, "local")
    progress = tmp_path / "progress"
    script = ("#!%s\nimport os, time\nfd = os.open(%r, os.O_WRONLY | os.O_CREAT, 0o644)\n"
              "print('up', flush=True)\nkeep, t = [], time.time()\n"
              "for i in range(32):\n"
              "    keep.append(b'\\x01' * (64 << 20))\n"
              "    os.pwrite(fd, b'%%012d' %% ((i + 1) * (64 << 20)), 0)\n"
              "print('survived %%.3f s' %% (time.time() - t), flush=True)\ntime.sleep(5)\n"
              % (sys.executable, str(progress)))
    task = _task(cloud, "poll-oom", script, machine="1-1000",
                 env={"TPI_MEMORY_CGROUP": "off"})
    task.create()
    status = task.wait(30)
    logs = "".join(task.logs())
    assert status["failed"] == 1 and "survived" not in logs, (status, logs)
    reached = int(progress.read_text())
    print("reached %.2f GB" % (reached / 1e9))
    assert reached < 1.5e9, reached
    events = task.events()
    guard = [e for e in events if e.code == "memory-guard"]
    assert guard and guard[0].description[0] == "poll 20 ms", guard
    assert task._state().get("memory_guard") == "poll 20 ms"
    assert [e for e in events if e.code == "rank-oom-killed"]
    task.delete()
