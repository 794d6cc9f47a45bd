"""Runtime workdir staging on a real MI355X (``pytest -m gpu``): the native loader into HBM,
the task communicator (RCCL) at one rank, and an ``iterative_task`` whose workdir the
supervisor's stager puts in HBM before the rank starts; the rank maps it through HIP IPC.
The numerics reference is the host file content (byte equality)."""
import json
import os

import numpy as np
import pytest
import torch

from terraform_provider_iterative_amd import backends, ops
from terraform_provider_iterative_amd.models.cloud import Cloud, Credentials, NodeCredentials
from terraform_provider_iterative_amd.models.values import Environment, Size, Task, Variables
from terraform_provider_iterative_amd.runtime import stage
from terraform_provider_iterative_amd.utils.identifier import new_deterministic_identifier

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    ops.hip(required=True)


def _files(tmp_path):
    rng = np.random.default_rng(1)
    sizes = {"a.bin": (5 << 20) + 3, "sub/b.bin": 4097, "c.txt": 1, "d.bin": 64 << 20}
    for rel, n in sizes.items():
        p = tmp_path / "work" / rel
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_bytes(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
    return tmp_path / "work", sizes


def test_loader_fills_hbm_from_files(tmp_path):
    work, sizes = _files(tmp_path)
    files, nbytes = stage.layout(str(work))
    dev = torch.full((nbytes,), 7, dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    with stage.Loader(0, chunk_bytes=4 << 20, nbuf=3, threads=4) as loader:
        st = loader.load(str(work), files, 0, nbytes, dev.data_ptr())
    assert st["bytes"] == nbytes and st["chunks"] == (nbytes + (4 << 20) - 1) // (4 << 20)
    host = dev.cpu().numpy()
    for rel, off, size in files:
        assert host[off:off + size].tobytes() == (work / rel).read_bytes(), rel
        assert not host[off + size:(off + size + 4095) // 4096 * 4096].any()
    # write-back of one dirty range
    dev[files[0][1]:files[0][1] + 4] = torch.tensor([9, 8, 7, 6], dtype=torch.uint8)
    torch.cuda.synchronize()
    with stage.Loader(0, chunk_bytes=1 << 20) as loader:
        loader.store(str(work), files, [(0, 1 << 20)], dev.data_ptr())
    assert (work / files[0][0]).read_bytes()[:4] == bytes([9, 8, 7, 6])


def test_task_communicator_single_rank():
    from terraform_provider_iterative_amd.parallel.comm import TaskComm, unique_id

    buf = torch.arange(1 << 20, dtype=torch.int32, device="cuda:0").view(torch.uint8)
    ref = buf.clone()
    with TaskComm(unique_id(), 1, 0, 0) as comm:
        comm.allgather_inplace(buf, buf.numel())
        comm.broadcast(buf, buf.numel(), root=0)
    assert torch.equal(buf, ref)


ATTACH = """#!/bin/sh
exec python3 - <<'EOF'
import os, torch
from terraform_provider_iterative_amd.runtime.stage import attach
w = attach()
assert w.buffer.is_cuda, w.buffer.device
root = os.environ["TPI_DATA_DIRECTORY"]
for rel in w.paths():
    host = open(os.path.join(root, rel), "rb").read()
    assert bytes(w.tensor(rel).cpu().numpy()) == host, rel
w.tensor("a.bin")[:3] = torch.tensor(list(b"XYZ"), dtype=torch.uint8, device=w.buffer.device)
torch.cuda.synchronize()
print("attached", w.buffer.device, w.stats["verified"], w.stats["load_GBps"])
EOF
"""


def test_task_workdir_staged_in_hbm_and_written_back(tmp_path, monkeypatch):
    monkeypatch.delenv("TPI_MI355X_GPUS", raising=False)
    monkeypatch.setenv("PYTHONPATH", ROOT)
    work, sizes = _files(tmp_path)
    cloud = Cloud(provider="mi355x",
                  credentials=Credentials(node=NodeCredentials(state_root=str(tmp_path / "st"))))
    spec = Task(size=Size(machine="m+mi355x"), parallelism=1,
                environment=Environment(script=ATTACH, timeout=300, directory=str(work),
                                        variables=Variables({"TPI_STAGE": "hbm",
                                                             "TPI_SYNC_INTERVAL": "0.5"})))
    task = backends.new(cloud, new_deterministic_identifier("hbm-stage"), spec)
    task.create()
    status = task.wait(120)
    logs = "\n".join(task.logs())
    stager_log = open(os.path.join(task.sup_dir, "stager.log")).read()
    assert status["succeeded"] == 1, (logs, stager_log)
    assert "attached cuda" in logs and "True" in logs
    events = task.events()
    codes = [e.code for e in events]
    assert "workdir-staged" in codes  # the rank starts while staging runs; attach() waits
    manifest = json.load(open(os.path.join(task.sup_dir, "stage-manifest.json")))
    assert manifest["stats"]["verified"] is True and manifest["ranks"][0]["ipc"]
    data = open(os.path.join(task.data_dir, "a.bin"), "rb").read()
    assert data[:3] == b"XYZ" and data[3:] == (work / "a.bin").read_bytes()[3:]
    assert any(e.code == "workdir-sync" and "dirty_shards 1" in e.description for e in events)
    task.delete()
