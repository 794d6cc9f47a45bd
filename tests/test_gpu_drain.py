"""A GPU changes hands only once the driver has the previous holder's memory back
(VERDICT r5 next #1).  The amdgpu driver's ``mem_info_vram_used`` is faked with a sysfs tree
(``TPI_SYSFS_PCI``), so these run on CPU: the lease the previous holder releases becomes a
drain marker carrying the count at its reservation, and the next holder's start waits for the
count to come back to it (bounded, journalled as ``gpu-drain``).

Reference: a replacement machine is a fresh VM that never inherits the old one's memory
(``task/aws/resources/resource_auto_scaling_group.go:51-106``)."""
import json
import os
import threading
import time

import pytest

from terraform_provider_iterative_amd import backends
from terraform_provider_iterative_amd.models.cloud import Cloud, Credentials, NodeCredentials
from terraform_provider_iterative_amd.models.values import Environment, Size, Task, Variables
from terraform_provider_iterative_amd.parallel.placement import GPU, Placement, vram_usage
from terraform_provider_iterative_amd.utils.identifier import new_deterministic_identifier

GB = 10 ** 9
TOTAL = 288 * 2 ** 30
PCI = "0000:fa:00.0"


class FakeVram:
    def __init__(self, root):
        self.dir = root / PCI
        self.dir.mkdir(parents=True)
        (self.dir / "mem_info_vram_total").write_text("%d\n" % TOTAL)
        self.set(1 * GB)

    def set(self, used: int) -> None:
        tmp = self.dir / "mem_info_vram_used.tmp"
        tmp.write_text("%d\n" % used)
        os.replace(tmp, self.dir / "mem_info_vram_used")


class FakeKfd:
    """KFD's topology node of the fake GPU (gpu_id 4242 at PCI_LOC) and its per-process VRAM
    accounting (``proc/<pid>/vram_<gpu_id>``)."""

    GPU_ID = 4242

    def __init__(self, root):
        self.root = root
        node = root / "topology" / "nodes" / "3"
        node.mkdir(parents=True)
        (node / "properties").write_text("gfx_target_version 90500\ndomain 0\nlocation_id %d\n"
                                         % (0xfa << 8))
        (node / "gpu_id").write_text("%d\n" % self.GPU_ID)
        (root / "proc").mkdir()

    def live(self, pid: int, used: int) -> None:
        d = self.root / "proc" / str(pid)
        d.mkdir(exist_ok=True)
        (d / ("vram_%d" % self.GPU_ID)).write_text("%d\n" % used)

    def exit(self, pid: int) -> None:
        import shutil

        shutil.rmtree(self.root / "proc" / str(pid))


@pytest.fixture()
def vram(tmp_path, monkeypatch):
    monkeypatch.setenv("TPI_SYSFS_PCI", str(tmp_path / "pci"))
    monkeypatch.setenv("TPI_SYSFS_KFD", str(tmp_path / "no-kfd"))  # no accounting by default
    return FakeVram(tmp_path / "pci")


@pytest.fixture()
def kfd(tmp_path, monkeypatch):
    monkeypatch.setenv("TPI_SYSFS_KFD", str(tmp_path / "kfd"))
    return FakeKfd(tmp_path / "kfd")


def _placement(tmp_path):
    return Placement(str(tmp_path / "state"), gpus=[GPU(index=0, gfx="gfx950", pci=PCI)])


def test_released_lease_becomes_a_drain_marker_and_the_next_start_waits(tmp_path, vram):
    assert vram_usage(PCI) == (1 * GB, TOTAL)
    placement = _placement(tmp_path)
    placement.allocate("task-a", 1)
    assert placement._read_lease(0)["vram_baseline"] == 1 * GB
    vram.set(150 * GB)  # task A's ranks hold 149 GB
    placement.release("task-a")
    marker = json.loads(open(placement.drain_path(0)).read())
    assert marker["task"] == "task-a" and marker["vram_baseline"] == 1 * GB
    placement.allocate("task-b", 1)  # the GPU is free for placement at once ...
    assert placement._read_lease(0)["vram_baseline"] == 1 * GB  # ... baseline carried over
    timer = threading.Timer(0.5, vram.set, (2 * GB,))  # the driver gives it back later
    timer.start()
    t0 = time.monotonic()
    recs = placement.settle_gpus([0], timeout=10)
    waited = time.monotonic() - t0
    timer.join()
    assert 0.4 < waited < 5
    assert len(recs) == 1 and recs[0]["previous"] == "task-a" and not recs[0]["timed_out"]
    assert recs[0]["used_gb_at_start"] == 150.0 and recs[0]["used_gb"] == 2.0
    assert not os.path.exists(placement.drain_path(0))
    assert placement._read_lease(0)["vram_baseline"] == 2 * GB  # rebased on the settled count
    assert placement.settle_gpus([0], timeout=10) == []  # nothing left to wait for


def test_the_wait_is_bounded(tmp_path, vram):
    placement = _placement(tmp_path)
    placement.allocate("task-a", 1)
    vram.set(100 * GB)
    placement.release("task-a")
    placement.allocate("task-b", 1)
    t0 = time.monotonic()
    recs = placement.settle_gpus([0], timeout=0.3)
    assert time.monotonic() - t0 < 2
    assert recs[0]["timed_out"] and recs[0]["used_gb"] == 100.0


def test_memory_freed_by_a_process_that_held_no_lease_is_waited_for(tmp_path, vram):
    """No drain marker (say a benchmark freed its own tensors): a count above the idle
    fraction that is still falling is waited for until it stops falling."""
    placement = _placement(tmp_path)
    placement.allocate("task-b", 1)
    steps = [200 * GB, 150 * GB, 90 * GB, 40 * GB, 3 * GB]
    vram.set(steps[0])

    def drain():
        for used in steps[1:]:
            time.sleep(0.1)
            vram.set(used)

    thread = threading.Thread(target=drain)
    thread.start()
    recs = placement.settle_gpus([0], timeout=10)
    thread.join()
    assert recs and recs[0]["previous"] is None and recs[0]["used_gb"] == 3.0
    assert recs[0]["waited_s"] >= 0.35
    # a GPU busy with something that does not go away costs one flat period (as long as a
    # wipe of that much memory could take), not the bound
    vram.set(60 * GB)
    t0 = time.monotonic()
    recs = placement.settle_gpus([0], timeout=10)
    assert time.monotonic() - t0 < 3 + 1.5 and not recs[0]["timed_out"] and recs[0]["floor"]


def test_orphaned_memory_is_what_the_start_waits_for(tmp_path, vram, kfd):
    """With KFD's per-process accounting the gate waits for memory no live process holds
    (exited processes, frees being wiped) -- never for what live processes use -- and learns
    a GPU's idle level when orphaned memory stops falling above the limit."""
    from terraform_provider_iterative_amd.parallel.placement import orphaned_vram

    placement = _placement(tmp_path)
    placement.allocate("task-b", 1)
    kfd.live(111, 100 * GB)  # another user's live process: 100 GB, not ours to wait for
    vram.set(101 * GB)
    assert orphaned_vram(PCI)["orphaned"] == 1 * GB
    t0 = time.monotonic()
    assert placement.settle_gpus([0], timeout=10) == []
    assert time.monotonic() - t0 < 0.5


def test_memory_turning_orphaned_is_no_idle_level(tmp_path, vram, kfd):
    """Processes still exiting move their memory from "live" to "orphaned" (the orphaned
    count rises while the driver's total stays): that is a drain in progress, never the GPU's
    idle level (round 6, r6c: 62 -> 80 GB was taken for a floor)."""
    placement = _placement(tmp_path)
    placement.allocate("task-b", 1)
    vram.set(170 * GB)
    kfd.live(222, 110 * GB)  # an exiting predecessor still holds 110 GB; 60 GB orphaned

    def exit_then_wipe():
        time.sleep(1.0)
        kfd.live(222, 40 * GB)   # tearing down: orphaned rises to 130 GB
        time.sleep(1.0)
        kfd.exit(222)            # gone: 170 GB orphaned
        time.sleep(1.5)
        vram.set(90 * GB)        # the wipe frees it in steps
        time.sleep(1.0)
        vram.set(3 * GB)

    thread = threading.Thread(target=exit_then_wipe)
    thread.start()
    recs = placement.settle_gpus([0], timeout=20)
    thread.join()
    assert recs[0]["orphaned_gb"] == 3.0 and not recs[0]["floor"], recs
    assert recs[0]["waited_s"] > 4.0
    assert placement._orphan_floor(0) is None
    kfd.live(333, 100 * GB)  # a live 100 GB process ...
    vram.set(250 * GB)  # ... plus 150 GB that a process freed and the driver still wipes
    timer = threading.Timer(0.6, vram.set, (102 * GB,))
    timer.start()
    recs = placement.settle_gpus([0], timeout=10)
    timer.join()
    assert recs[0]["orphaned_gb_at_start"] == 150.0 and recs[0]["orphaned_gb"] == 2.0
    assert 0.5 < recs[0]["waited_s"] < 3 and not recs[0]["floor"]
    # 10 GB the driver never gives back (its own): waited for once, then remembered
    vram.set(110 * GB)
    recs = placement.settle_gpus([0], timeout=10)
    assert recs[0]["floor"] and 2.9 < recs[0]["waited_s"] < 4.5
    t0 = time.monotonic()
    assert placement.settle_gpus([0], timeout=10) == []
    assert time.monotonic() - t0 < 0.5


def test_a_big_buffer_wiped_in_one_step_is_no_idle_level(tmp_path, vram, kfd):
    """The driver gives a freed buffer back in one step at the end of its wipe (~35 GB/s): 150
    GB show no fall for ~4.3 s.  A 3 s window took that for the GPU's idle level and started
    the next task on top of it (round 6, r6f); the window scales with the count."""
    from terraform_provider_iterative_amd.parallel.placement import flat_window

    assert flat_window(2 * GB) == 3.0 and flat_window(150 * GB) == 7.5
    placement = _placement(tmp_path)
    placement.allocate("task-b", 1)
    vram.set(152 * GB)  # 150 GB freed by an exited process, still being wiped
    timer = threading.Timer(4.3, vram.set, (2 * GB,))
    timer.start()
    recs = placement.settle_gpus([0], timeout=20)
    timer.join()
    assert recs[0]["orphaned_gb"] == 2.0 and not recs[0]["floor"], recs
    assert 4.2 < recs[0]["waited_s"] < 6
    assert placement._orphan_floor(0) is None


def test_unreadable_counters_are_not_waited_for(tmp_path, monkeypatch):
    monkeypatch.setenv("TPI_SYSFS_PCI", str(tmp_path / "nothing-here"))
    placement = _placement(tmp_path)
    placement.allocate("task-a", 1)
    assert "vram_baseline" not in placement._read_lease(0)
    assert placement.settle_gpus([0], timeout=10) == []


def _task(cloud, name, script):
    spec = Task(size=Size(machine="m+mi355x"), parallelism=1,
                environment=Environment(script=script, variables=Variables({"TPI_TASK": "true"}),
                                        timeout=120))
    return backends.new(cloud, new_deterministic_identifier(name), spec)


def test_a_queued_task_starts_only_once_the_previous_holders_memory_is_back(
        tmp_path, vram, monkeypatch):
    monkeypatch.setenv("TPI_MI355X_GPUS", "0=%s" % PCI)
    monkeypatch.setenv("TPI_NODE_CPUS", "0-7")
    monkeypatch.setenv("TPI_NODE_MEMORY_MB", "64000")
    monkeypatch.setenv("TPI_PRELOAD", "0")
    cloud = Cloud(provider="mi355x",
                  credentials=Credentials(node=NodeCredentials(state_root=str(tmp_path / "st"))))
    gate = tmp_path / "gate"
    holder = _task(cloud, "drain-holder",
                   "#!/bin/sh\necho holding\ni=0\nwhile [ ! -e %s ] && [ $i -lt 1200 ]; do "
                   "sleep 0.05; i=$((i+1)); done\n" % gate)
    holder.create()
    deadline = time.time() + 30
    while time.time() < deadline and "holding" not in "".join(holder.logs()):
        time.sleep(0.05)
    vram.set(120 * GB)  # the holder's ranks fill the GPU
    nxt = _task(cloud, "drain-next", "#!/bin/sh\necho next started\n")
    nxt.create()
    assert [e.code for e in nxt.events()].count("queued") == 1
    gate.write_text("go")  # the holder finishes; its supervisor hands the GPU on
    assert holder.wait(30)["succeeded"] == 1
    time.sleep(1.0)  # ... but the driver still holds its memory
    assert "next started" not in "".join(nxt.logs())
    assert not any(e.code == "rank-start" for e in nxt.events())
    t_back = time.time()
    vram.set(1 * GB)
    assert nxt.wait(30)["succeeded"] == 1
    events = {e.code: e for e in nxt.events()}
    assert "gpu-drain" in events, [e.code for e in nxt.events()]
    desc = events["gpu-drain"].description
    assert "previous holder %s" % holder.id in desc and "timed out" not in " ".join(desc)
    waited = float(desc[1].split()[1])
    assert waited >= 0.9
    start = events["rank-start"].time
    start = start.timestamp() if hasattr(start, "timestamp") else start
    assert start >= t_back - 0.05
    nxt.delete()
    holder.delete()
