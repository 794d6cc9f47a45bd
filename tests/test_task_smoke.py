"""Port of the reference's smoke test (task/task_smoke_test.go:63-237) onto the node runtime.

Flow: sweep (Delete before anything exists), seed ``output/file`` with old data, Create twice
(idempotent), poll Read/Logs until one log shows both the uploaded old data and the injected
environment variable, wait for ``running == 0 && succeeded > 0``, Delete twice, then check
that only the output directory came back (``cache/file`` stays remote) and that it holds the
task's data.  ``local`` runs everywhere; ``mi355x`` runs with a fake GPU inventory on CPU and
for real (``rocm-smi``) under ``-m gpu``.
"""
import time
import uuid

import pytest

from terraform_provider_iterative_amd import backends
from terraform_provider_iterative_amd.models.cloud import Cloud, Credentials, NodeCredentials
from terraform_provider_iterative_amd.models.values import (STATUS_FAILED, STATUS_RUNNING,
                                                            STATUS_SUCCEEDED, Environment, Size,
                                                            Task, Variables)
from terraform_provider_iterative_amd.utils.identifier import new_deterministic_identifier

SCRIPT = """#!/bin/bash -e
test -v TEST_GPU && rocm-smi --showproductname
mkdir --parents cache output
touch cache/file
echo "$ENVIRONMENT_VARIABLE_DATA" | tee --append output/file
sleep 1
cat output/file
"""


def _smoke(tmp_path, provider, machine, env_extra=None):
    old, new = str(uuid.uuid4()), str(uuid.uuid4())
    base = tmp_path / "work"
    cache, output = base / "cache", base / "output"
    base.mkdir()
    cloud = Cloud(provider=provider, region="us-west",
                  credentials=Credentials(node=NodeCredentials(state_root=str(tmp_path / "st"))))
    variables = {"ENVIRONMENT_VARIABLE_DATA": new}
    variables.update(env_extra or {})
    spec = Task(size=Size(machine=machine), parallelism=1,
                environment=Environment(script=SCRIPT, variables=Variables(variables),
                                        directory=str(base), directory_out="output",
                                        timeout=600))
    task = backends.new(cloud, new_deterministic_identifier("smoke test"), spec)

    task.delete()  # sweep: nothing exists yet
    cache.mkdir()
    output.mkdir()
    (output / "file").write_text(old)

    task.create()
    task.create()  # idempotent

    deadline = time.time() + 120
    while time.time() < deadline:
        task.read()
        if any(old in log and new in log for log in task.logs()):
            break
        if task.status()[STATUS_FAILED] > 0:
            break
        time.sleep(0.1)
    else:
        pytest.fail("logs never showed both data markers: %s" % task.logs())
    while time.time() < deadline:
        task.read()
        status = task.status()
        if status[STATUS_RUNNING] == 0 and status[STATUS_SUCCEEDED] > 0:
            break
        time.sleep(0.1)
    assert status[STATUS_FAILED] == 0, (status, task.logs())

    task.delete()
    task.delete()  # idempotent

    assert not (cache / "file").exists()  # only the output directory is pulled back
    contents = (output / "file").read_text()
    assert old in contents and new in contents
    return task


def test_smoke_local(tmp_path):
    _smoke(tmp_path, "local", "m")


def test_smoke_mi355x_fake_inventory(tmp_path, monkeypatch):
    monkeypatch.setenv("TPI_MI355X_GPUS", "0,1")
    _smoke(tmp_path, "mi355x", "m+mi355x")


@pytest.mark.gpu
def test_smoke_mi355x_gpu(tmp_path):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    _smoke(tmp_path, "mi355x", "m+mi355x", {"TEST_GPU": "1"})
