"""Off-node ``storage.container`` (storage/remote.py) over the SSH command transport, with the
fake ``ssh`` of the remote-node tests (it runs the command locally: the "storage node" is a
directory of this machine).

Reference: a pre-allocated bucket/volume holds the task's data and reports and outlives the
machine (``iterative/resource_task.go:380-397``, ``task/common/machine/storage.go:236-263``,
``task/aws/resources/data_source_bucket.go:15-62``); Delete pulls the output and leaves a
bucket it did not create in place (``task/aws/task.go:245-299``).
"""
import os
import sys

import pytest

from terraform_provider_iterative_amd import backends
from terraform_provider_iterative_amd.models.cloud import Cloud, Credentials, NodeCredentials
from terraform_provider_iterative_amd.models.values import (Environment, RemoteStorage, Task,
                                                            Variables)
from terraform_provider_iterative_amd.storage import remote
from terraform_provider_iterative_amd.utils.identifier import new_deterministic_identifier

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture()
def fake_ssh(tmp_path, monkeypatch):
    node = tmp_path / "storage-node-state"
    node.mkdir()
    monkeypatch.setenv("FAKE_SSH_STATE_ROOT", str(node))
    monkeypatch.setenv("TPI_SSH_COMMAND", "%s %s" % (sys.executable,
                                                     os.path.join(ROOT, "tests", "fake_ssh.py")))
    return node


def test_container_forms():
    c = remote.parse("ssh://alice@store-1:2222/srv/tpi")
    assert (c.backend, c.container, c.path, c.config["port"], c.config["user"]) == \
        ("ssh", "store-1", "/srv/tpi", "2222", "alice")
    c = remote.parse("store-1:/srv/tpi", "proj/run1")
    assert c.path == "/srv/tpi/proj/run1" and c.config["host"] == "store-1"
    c = remote.parse("bucket-dir", opts={"host": "store-2", "root": "/data", "port": "22"})
    assert (c.container, c.path, c.config["port"]) == ("store-2", "/data/bucket-dir", "22")
    c2 = remote.parse(str(c))  # the rclone form Connection renders parses back
    assert (c2.container, c2.path, c2.config["port"]) == ("store-2", "/data/bucket-dir", "22")
    assert remote.parse("/local/dir") is None and remote.parse("relative") is None
    assert remote.is_remote("ssh://h/x") and remote.is_remote("h:/x")
    assert not remote.is_remote("/dev/shm/spill")
    with pytest.raises(ValueError):  # nothing reaches ssh's argv as an option
        remote.SSHRemote(remote.parse(":ssh,host=-oProxyCommand:/srv"))
    assert remote.parse("ssh://-oProxy/srv") is None


SCRIPT = r'''#!%(python)s
import os, sys
sys.path.insert(0, %(root)r)
import torch
from terraform_provider_iterative_amd.checkpoint import Checkpointer
os.makedirs("output", exist_ok=True)
seen = open("input.txt").read().strip()
earlier = open("output/result.txt").read().strip() if os.path.exists("output/result.txt") else "-"
with open("output/result.txt", "w") as f:
    f.write("run %%s saw %%s after %%s\n" %% (os.environ["RUN"], seen, earlier))
open("cache.tmp", "w").write("scratch")
state = {"w": torch.arange(5000, dtype=torch.float64) * int(os.environ["RUN"])}
ck = Checkpointer(state, path=os.path.join(os.environ["TPI_DATA_DIRECTORY"], ".spill"),
                  tile_bytes=4096)
ck.save({"run": os.environ["RUN"]})
ck.persist(os.environ["CKPT_URL"])  # straight into the container, on the storage node
print("run", os.environ["RUN"], "done", flush=True)
'''


def _task(tmp_path, name, container, run, workdir, out="output"):
    cloud = Cloud(provider="local",
                  credentials=Credentials(node=NodeCredentials(state_root=str(tmp_path / "st"))))
    url = "ssh://storage-node%s/ckpt-%s.bin" % (container.split("storage-node:", 1)[1], run)
    spec = Task(
        environment=Environment(
            script=SCRIPT % {"python": sys.executable, "root": ROOT}, timeout=120,
            directory=str(workdir), directory_out=out, exclude_list=["cache.tmp"],
            variables=Variables({"TPI_TASK": "true", "RUN": str(run), "CKPT_URL": url,
                                 "FAKE_SSH_STATE_ROOT": os.environ["FAKE_SSH_STATE_ROOT"],
                                 "TPI_SYNC_INTERVAL": "0.3"})),
        remote_storage=RemoteStorage(container, "", {}))
    return backends.new(cloud, new_deterministic_identifier(name), spec), url


def test_task_data_lives_in_the_container_and_survives_delete(tmp_path, fake_ssh):
    bucket = tmp_path / "bucket"  # the storage node's directory
    container = "storage-node:%s" % bucket
    work = tmp_path / "work"
    work.mkdir()
    (work / "input.txt").write_text("hello\n")
    (work / "main.tf").write_text("# never uploaded (default exclude)\n")

    task, url = _task(tmp_path, "remote-1", container, 1, work)
    task.create()
    status = task.wait(60)
    assert status["succeeded"] == 1, task.logs()
    # the container holds the data, the output, the persisted checkpoint and the reports
    assert (bucket / "data" / "input.txt").read_text() == "hello\n"
    assert not (bucket / "data" / "main.tf").exists()
    assert (bucket / "data" / "output" / "result.txt").read_text() == "run 1 saw hello after -\n"
    assert (bucket / "ckpt-1.bin").stat().st_size > 40000
    reports = sorted(p.name for p in (bucket / "reports").iterdir())
    assert any(n.startswith("task-") for n in reports) and any(n.startswith("status-")
                                                               for n in reports)
    codes = [e.code for e in task.events()]
    assert "container-restored" in codes and "remote-synced" in codes
    task.delete()
    # delete pulled storage.output into the workdir and left the container in place
    assert (work / "output" / "result.txt").read_text() == "run 1 saw hello after -\n"
    assert not (work / "cache.tmp").exists()
    assert (bucket / "data" / "output" / "result.txt").exists()
    assert not os.path.exists(task.root)

    # a second task on the same container starts from what the first one left there
    (work / "input.txt").write_text("again\n")
    import shutil

    shutil.rmtree(work / "output")
    task2, _ = _task(tmp_path, "remote-2", container, 2, work)
    task2.create()
    assert task2.wait(60)["succeeded"] == 1, task2.logs()
    assert (bucket / "data" / "output" / "result.txt").read_text() == \
        "run 2 saw again after run 1 saw hello after -\n"
    task2.delete()

    # and a checkpoint persisted there loads from the container on any node
    import torch

    from terraform_provider_iterative_amd.checkpoint import Checkpointer

    state = {"w": torch.zeros(5000, dtype=torch.float64)}
    with Checkpointer(state, path=str(tmp_path / "spill"), tile_bytes=4096) as ck:
        res = ck.load(url)
        assert res.bad_tiles == 0 and ck.header()["metadata"] == {"run": "1"}
    assert torch.equal(state["w"], torch.arange(5000, dtype=torch.float64))


# A rank that is preempted, releases its GPU ("released" on the notify pipe) and then takes 20 s
# to exit after the supervisor's exit request -- the kernel teardown of a 100 GB pinned region
# after a hot hand-off took 10-18 s on MI355X.  Its successor finishes
# at once.  Reference: the status is written and the group scaled to 0 right after the task's
# exit (machine-script.sh.tpl:10-15,51).
LINGERING = r'''#!%(python)s
import os, signal, sys, time
restart = int(os.environ["TPI_RESTART_COUNT"])
fd = int(os.environ["TPI_NOTIFY_FD"])
if restart == 0:
    signal.pthread_sigmask(signal.SIG_BLOCK, {signal.SIGTERM, signal.SIGUSR2})
    open(os.environ["PRED_PID_FILE"], "w").write(str(os.getpid()))
    print("ready", flush=True)
    signal.sigwait({signal.SIGTERM})
    os.write(fd, b"released\n")
    signal.sigwait({signal.SIGUSR2})
    time.sleep(20.0)
    os._exit(143)
os.makedirs("output", exist_ok=True)
with open("output/result.txt", "w") as f:
    f.write("successor done\n")
print("successor done", flush=True)
'''


def test_delete_does_not_wait_for_a_lingering_released_process(tmp_path, fake_ssh):
    import time

    from terraform_provider_iterative_amd.parallel.placement import pid_alive

    bucket = tmp_path / "bucket"
    container = "storage-node:%s" % bucket
    work = tmp_path / "work"
    work.mkdir()
    pid_file = tmp_path / "pred.pid"
    cloud = Cloud(provider="local",
                  credentials=Credentials(node=NodeCredentials(state_root=str(tmp_path / "st"))))
    spec = Task(environment=Environment(
        script=LINGERING % {"python": sys.executable}, timeout=120, directory=str(work),
        directory_out="output",
        variables=Variables({"TPI_TASK": "true", "PRED_PID_FILE": str(pid_file),
                             "FAKE_SSH_STATE_ROOT": os.environ["FAKE_SSH_STATE_ROOT"],
                             "TPI_SYNC_INTERVAL": "0"})),
        remote_storage=RemoteStorage(container, "", {}))
    task = backends.new(cloud, new_deterministic_identifier("lingering"), spec)
    task.create()
    deadline = time.time() + 60
    while time.time() < deadline and "ready" not in "".join(task.logs()):
        time.sleep(0.05)
    pred = int(pid_file.read_text())
    task.preempt()
    status = task.wait(30)  # returns when the task is over for its users
    t_over = time.time()
    assert status["succeeded"] == 1, task.logs()
    assert pid_alive(pred), "the released predecessor should still be exiting"
    events = task.events()
    codes = [e.code for e in events]
    # the final awaited sync ran at the ranks' exit, before the released process was reaped
    synced = [e for e in events if e.code == "remote-synced" and "final" in e.description]
    assert synced and "supervisor-settled" in codes and "rank-released-exit" not in codes, codes
    assert (bucket / "data" / "output" / "result.txt").read_text() == "successor done\n"
    assert any(p.name.startswith("status-") for p in (bucket / "reports").iterdir())
    t0 = time.time()
    task.delete()
    took = time.time() - t0
    assert took < 3.0, took
    assert pid_alive(pred), "delete must not wait for (or need) the predecessor's exit"
    assert (work / "output" / "result.txt").read_text() == "successor done\n"
    assert not os.path.exists(task.root)
    assert time.time() - t_over < 10.0  # everything above, well inside the 20 s linger
    os.kill(pred, 9)
