"""Remote-node backend (``region = "host=..."``): the client drives another node's runtime
through a command transport; the reference's laptop -> remote machine flow
(task/task_smoke_test.go:63-237: create twice, logs carry the workdir's data, delete twice,
output downloaded, excluded files never uploaded).  ``tests/fake_ssh.py`` plays ssh, running
the remote command on this machine against a separate state root."""
import os
import sys
import time

import pytest

from terraform_provider_iterative_amd import backends
from terraform_provider_iterative_amd.backends.ssh import RemoteNodeError, RemoteNodeTask
from terraform_provider_iterative_amd.models.cloud import Cloud, Credentials, NodeCredentials
from terraform_provider_iterative_amd.models.values import (Environment, NotFoundError, Size,
                                                            Task, Variables)
from terraform_provider_iterative_amd.utils.identifier import new_deterministic_identifier

HERE = os.path.dirname(os.path.abspath(__file__))

# The task holds until the test opens GATE (after its second create): a fixed sleep raced the
# second create under `pytest -n 8`, which then found the task finished and re-ran it.
SCRIPT = """#!/bin/sh
i=0
while [ ! -e "%(gate)s" ] && [ $i -lt 1200 ]; do sleep 0.05; i=$((i+1)); done
echo "rank $RANK says $GREETING_FROM_CLIENT"
cat input.txt
test -e skip.log && echo "skip.log leaked"
test -e main.tf && echo "main.tf leaked"
mkdir -p results
echo "result of $(cat input.txt)" > results/out.txt
echo cache > cache.bin
"""


@pytest.fixture()
def remote(tmp_path, monkeypatch):
    node_root = tmp_path / "node-state"
    node_root.mkdir()
    monkeypatch.setenv("FAKE_SSH_STATE_ROOT", str(node_root))
    monkeypatch.setenv("TPI_SSH_COMMAND", "%s %s -o BatchMode=yes" % (
        sys.executable, os.path.join(HERE, "fake_ssh.py")))
    monkeypatch.setenv("TPI_REMOTE_PYTHON", sys.executable)
    monkeypatch.setenv("TPI_STATE_ROOT", str(tmp_path / "client-state"))  # must stay unused
    monkeypatch.setenv("GREETING_FROM_CLIENT", "hi")
    monkeypatch.delenv("TPI_REMOTE_FRAMEWORK", raising=False)
    return node_root


def _workdir(tmp_path):
    work = tmp_path / "project"
    work.mkdir()
    (work / "input.txt").write_text("payload-42\n")
    (work / "main.tf").write_text("# terraform config: default exclude\n")
    (work / "skip.log").write_text("excluded by the task\n")
    (work / "sub").mkdir()
    (work / "sub" / "big.bin").write_bytes(os.urandom(300001))
    return work


def _spec(work, gate):
    return Task(size=Size(machine="s"),
                environment=Environment(
                    script=SCRIPT % {"gate": gate}, directory=str(work), directory_out="results",
                    exclude_list=["skip.log"],
                    variables=Variables({"GREETING_*": None})),
                parallelism=1)


def _wait(task, timeout=60):
    deadline = time.time() + timeout
    while time.time() < deadline:
        task.read()
        status = task.status()
        if status.get("succeeded", 0) + status.get("failed", 0) >= 1 and \
                not status.get("running"):
            return status
        time.sleep(0.1)
    raise AssertionError("task did not finish: %s %s" % (task.status(), task.logs()))


def test_remote_node_create_read_delete(tmp_path, remote):
    work = _workdir(tmp_path)
    cloud = Cloud(provider="local", region="host=gpu-node-7")
    ident = new_deterministic_identifier("remote-smoke")
    gate = tmp_path / "gate"
    spec = _spec(work, gate)
    task = backends.new(cloud, ident, spec)
    assert isinstance(task, RemoteNodeTask)
    task.create()
    backends.new(cloud, ident, spec).create()  # idempotent, like the reference's smoke test
    gate.write_text("go")  # only now may the task finish
    status = _wait(task)
    assert status["succeeded"] == 1, task.logs()
    log = "".join(task.logs())
    assert "rank 0 says hi" in log and "payload-42" in log  # env enriched on the client
    assert "leaked" not in log
    # the node holds the task; the client's own state root was never used
    node_task = remote / "local" / ident.long()
    assert (node_task / "data" / "sub" / "big.bin").stat().st_size == 300001
    assert not (node_task / "data" / "skip.log").exists()
    assert not (tmp_path / "client-state").exists()
    assert any(e.code == "started" for e in task.events())
    assert ident.long() in [i.long() for i in backends.list_tasks(cloud)]
    # delete pulls the output only (LimitTransfer), then removes the task on the node
    task.delete()
    assert (work / "results" / "out.txt").read_text() == "result of payload-42\n"
    assert not (work / "cache.bin").exists()
    assert not node_task.exists()
    backends.new(cloud, ident, spec).delete()  # deleting twice is fine
    with pytest.raises(NotFoundError):
        backends.new(cloud, ident, spec).read()
    ops = (remote / "ssh.log").read_text().split()
    assert "push" in ops and "pull" in ops


def test_remote_node_state_root_and_placement_keys(tmp_path, remote):
    """``root=`` picks the node's state root; placement keys travel to the node."""
    custom = tmp_path / "custom-root"
    cloud = Cloud(provider="local", region="host=n1,root=%s,numa=0" % custom)
    ident = new_deterministic_identifier("remote-root")
    task = backends.new(cloud, ident, Task(environment=Environment(script="#!/bin/sh\necho ok\n")))
    assert task.transport.region == "numa=0" and task.transport.state_root == str(custom)
    task.create()
    assert _wait(task)["succeeded"] == 1
    assert (custom / "local" / ident.long() / "task.json").exists()
    assert not (remote / "local").exists()
    task.delete()


def test_remote_node_errors_are_reported(tmp_path, remote):
    cloud = Cloud(provider="local", region="host=n2")
    ident = new_deterministic_identifier("remote-gpu-on-cpu")
    task = backends.new(cloud, ident, Task(size=Size(machine="m+mi355x"),
                                           environment=Environment(script="#!/bin/sh\n")))
    with pytest.raises(RemoteNodeError, match="mi355x"):
        task.create()
    bad = Cloud(provider="local", region="host=n3")
    os.environ["TPI_REMOTE_FRAMEWORK"] = str(tmp_path / "no-such-checkout")
    try:
        with pytest.raises(RemoteNodeError, match="no answer"):
            backends.new(bad, ident, Task()).read()
    finally:
        del os.environ["TPI_REMOTE_FRAMEWORK"]


def test_local_cloud_without_host_stays_local(tmp_path):
    cloud = Cloud(provider="local", region="us-west",
                  credentials=Credentials(node=NodeCredentials(state_root=str(tmp_path))))
    assert not isinstance(backends.new(cloud, new_deterministic_identifier("x"), Task()),
                          RemoteNodeTask)


def test_leo_smoke_flow_on_a_remote_node(tmp_path, remote):
    """The reference smoke flow through ``leo --region host=...``."""
    import subprocess
    import uuid

    leo = [sys.executable, os.path.join(os.path.dirname(HERE), "bin", "leo"), "--cloud", "local",
           "--region", "host=node-b"]
    work = tmp_path / "w"
    (work / "cache").mkdir(parents=True)
    old, new = str(uuid.uuid4()), str(uuid.uuid4())
    (work / "cache" / "old").write_text(old)
    script = ("#!/bin/sh\ncat cache/old\necho $NEW_UUID\nmkdir -p output\n"
              "echo $NEW_UUID > output/new\necho changed > cache/old\n")

    def run(*args, check=True):
        r = subprocess.run(leo + list(args), cwd=str(tmp_path), capture_output=True, text=True,
                           timeout=120, env=dict(os.environ))
        if check and r.returncode:
            raise AssertionError("%s: %s\n%s" % (args, r.stdout, r.stderr))
        return r

    ident = run("create", "--name", "rsmoke", "--workdir", str(work), "--output", "output",
                "--environment", "NEW_UUID=%s" % new, "--script", script).stdout.split()[-1]
    follow = run("read", "--follow", ident)
    assert old in follow.stdout and new in follow.stdout
    assert ident in run("list").stdout
    run("delete", "--workdir", str(work), "--output", "output", ident)
    assert (work / "output" / "new").read_text().strip() == new
    assert (work / "cache" / "old").read_text() == old
    assert not (remote / "local" / ident).exists()


def test_remote_cloud_config_retargeted_to_a_remote_node(tmp_path, remote, monkeypatch):
    """An unchanged ``cloud = "aws"`` definition runs on a remote MI355X node's runtime with
    TPI_REMOTE_AS + TPI_REMOTE_HOST."""
    monkeypatch.setenv("TPI_REMOTE_AS", "local")
    monkeypatch.setenv("TPI_REMOTE_HOST", "node-c")
    cloud = Cloud(provider="aws", region="us-east")
    ident = new_deterministic_identifier("retarget-remote")
    task = backends.new(cloud, ident, Task(environment=Environment(script="#!/bin/sh\necho hi\n")))
    assert isinstance(task, RemoteNodeTask) and task.transport.host == "node-c"
    task.create()
    assert _wait(task)["succeeded"] == 1 and "hi" in "".join(task.logs())
    assert (remote / "local" / ident.long()).is_dir()
    task.delete()


@pytest.mark.parametrize("region", ["host=-oProxyCommand=touch_x", "host=user@-p",
                                    "host=n1,port=22;rm"])
def test_remote_host_cannot_inject_ssh_options(region):
    from terraform_provider_iterative_amd.backends.ssh import Transport

    with pytest.raises(ValueError):
        Transport(Cloud(provider="local", region=region))
