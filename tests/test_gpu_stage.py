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



ATTACH_BIG = """#!/bin/sh
exec python3 - <<'EOF'
import os, time, torch
from terraform_provider_iterative_amd.runtime.stage import attach
t0 = time.monotonic()
w = attach()
took = time.monotonic() - t0
root = os.environ["TPI_DATA_DIRECTORY"]
rel = "big.bin"
view = w.tensor(rel)
size = os.path.getsize(os.path.join(root, rel))
assert view.numel() == size, (view.numel(), size)
with open(os.path.join(root, rel), "rb") as f:
    for k in range(17):  # 1 MiB windows across the whole image, the last one at its end
        off = min(k * (size // 16), size - (1 << 20))
        f.seek(off)
        host = f.read(1 << 20)
        assert bytes(view[off:off + (1 << 20)].cpu().numpy()) == host, off
print("attached big %.3f GB in %.4f s" % (size / 1e9, took), w.stats["verified"])
EOF
"""


def test_task_attaches_a_staged_workdir_beyond_2_gib(tmp_path, monkeypatch):
    """a workdir of 2.6 GB goes through the real stager (its image is one
    hipMalloc of the /opt/rocm runtime) and is mapped by the rank (PyTorch's HIP runtime)
    through HIP IPC -- the import that never returns for a PyTorch exporter's allocations of
    2 GiB or more (profiles/round5/ipc_cause.md).  The attach is bounded
    (TPI_IPC_OPEN_TIMEOUT): it either maps in time or fails the rank with an event."""
    monkeypatch.delenv("TPI_MI355X_GPUS", raising=False)
    monkeypatch.setenv("PYTHONPATH", ROOT)
    work = tmp_path / "work"
    work.mkdir()
    rng = np.random.default_rng(3)
    size = int(2.6e9) + 12345
    with open(work / "big.bin", "wb") as f:
        left = size
        while left:
            n = min(left, 256 << 20)
            f.write(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
            left -= n
    cloud = Cloud(provider="mi355x",
                  credentials=Credentials(node=NodeCredentials(state_root=str(tmp_path / "st"))))
    spec = Task(size=Size(machine="m+mi355x"), parallelism=1,
                environment=Environment(script=ATTACH_BIG, timeout=300, directory=str(work),
                                        variables=Variables({"TPI_STAGE": "hbm",
                                                             "TPI_IPC_OPEN_TIMEOUT": "20"})))
    task = backends.new(cloud, new_deterministic_identifier("hbm-stage-big"), spec)
    task.create()
    status = task.wait(240)
    logs = "\n".join(task.logs())
    events = task.events()
    stager_log = open(os.path.join(task.sup_dir, "stager.log")).read()
    try:
        assert status["succeeded"] == 1, (logs, stager_log, [(e.code, e.description)
                                                             for e in events])
        assert "attached big 2.600 GB" in logs and "True" in logs
        attached = [e for e in events if e.code == "workdir-attached"]
        assert attached and not any(e.code == "workdir-attach-failed" for e in events)
        print("big attach:", attached[0].description, logs.strip().splitlines()[-1])
    finally:
        task.delete()
