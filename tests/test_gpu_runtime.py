"""Runtime on a real MI355X (``pytest -m gpu``): HBM workdir staging, the mi355x provider
placing a rank on the GPU, and preempt/resume of a bf16 training job with device tensors."""
import os
import sys
import time

import numpy as np
import pytest
import torch

from terraform_provider_iterative_amd import backends, ops
from terraform_provider_iterative_amd.models.cloud import Cloud, Credentials, NodeCredentials
from terraform_provider_iterative_amd.models.values import Environment, Size, Task, Variables
from terraform_provider_iterative_amd.utils.identifier import new_deterministic_identifier

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    ops.hip(required=True)


@pytest.mark.parametrize("zero_copy_min", [1 << 40, 4096])  # bounce only / mixed
def test_stage_workdir_on_device(tmp_path, zero_copy_min, monkeypatch):
    monkeypatch.setenv("TPI_STAGE_ZERO_COPY", "1")
    from terraform_provider_iterative_amd.runtime.workdir import ALIGN, stage_workdir

    rng = np.random.default_rng(0)
    sizes = {"a.bin": 5000, "sub/b.bin": (3 << 20) + 17, "c.txt": 1}
    for rel, n in sizes.items():
        p = tmp_path / rel
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_bytes(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
    staged = stage_workdir(str(tmp_path), device=torch.device("cuda", 0), chunk_bytes=1 << 20,
                           zero_copy_min=zero_copy_min)
    assert staged.stats.get("zero_copy_files", 0) == (2 if zero_copy_min == 4096 else 0)
    assert staged.buffer.device.type == "cuda"
    for rel, n in sizes.items():
        got = staged.tensor(rel).cpu().numpy().tobytes()
        assert got == (tmp_path / rel).read_bytes(), rel
    # digest on device == host shard hash of the same layout (gaps zero)
    host = np.zeros(staged.buffer.numel(), dtype=np.uint8)
    for f in staged.files:
        host[f.offset:f.offset + f.size] = np.frombuffer((tmp_path / f.path).read_bytes(), np.uint8)
    assert all(f.offset % ALIGN == 0 for f in staged.files)
    assert staged.digest().cpu().numpy().view(np.uint64).tolist() == \
        ops.shard_hash(host).tolist()


@pytest.fixture()
def cloud(tmp_path, monkeypatch):
    monkeypatch.delenv("TPI_MI355X_GPUS", raising=False)
    return Cloud(provider="mi355x",
                 credentials=Credentials(node=NodeCredentials(state_root=str(tmp_path / "st"))))


def test_mi355x_task_sees_its_gpu(cloud):
    script = ("#!%s\nimport os, torch\nprint('visible', os.environ.get('HIP_VISIBLE_DEVICES'), "
              "torch.cuda.device_count(), torch.cuda.get_device_properties(0).gcnArchName, "
              "flush=True)\n" % sys.executable)
    spec = Task(size=Size(machine="m+mi355x"),
                environment=Environment(script=script, timeout=600,
                                        variables=Variables({"TPI_TASK": "true"})))
    task = backends.new(cloud, new_deterministic_identifier("gpu-visible"), spec)
    task.create()
    assert len(task.gpus()) == 1
    status = task.wait(300)
    logs = "".join(task.logs())
    assert status["succeeded"] == 1, logs
    assert "visible %d 1 gfx950" % task.gpus()[0] in logs
    task.delete()


@pytest.mark.parametrize("materialize", [False, True])
def test_preempt_resume_training_on_gpu(cloud, tmp_path, materialize):
    """examples/train/train.py preempted mid-run resumes from its checkpoint; with
    --materialize the successor builds its model on the meta device and resumes around the
    materialized tensors (TrainingState.from_materialized)."""
    env = {"TPI_FRAMEWORK_ROOT": ROOT, "TPI_TASK": "true"}
    script = ("#!/bin/sh\nexec %s %s/examples/train/train.py --steps 60 --hidden 256 --layers 2 "
              "--batch 4 --seq 64 --sleep 0.05%s\n" % (sys.executable, ROOT,
                                                       " --materialize" if materialize else ""))
    spec = Task(size=Size(machine="m+mi355x"),
                environment=Environment(script=script, timeout=600, variables=Variables(env)))
    task = backends.new(cloud, new_deterministic_identifier("gpu-preempt-%d" % materialize),
                        spec)
    task.create()
    deadline = time.time() + 300
    while time.time() < deadline and not any("step 11" in l for l in task.logs()):
        time.sleep(0.1)
    assert any("step 11" in l for l in task.logs()), task.logs()
    task.preempt()
    status = task.wait(300)
    logs = task.logs()
    assert status["succeeded"] == 1, logs
    assert len(logs) == 2 and "preemption checkpoint saved" in logs[0]
    resumed = [l for l in logs[1].splitlines() if "resumed from step" in l]
    assert resumed and int(resumed[0].rsplit(" ", 1)[1]) >= 11
    assert "done" in logs[1]
    task.delete()


def test_preempted_training_resumes_in_a_preloaded_successor_on_gpu(cloud, tmp_path):
    """A Python rank (examples/train/train.py behind a Python shebang) with TPI_PRELOAD=1:
    its successor is the parked interpreter that imported PyTorch before the preemption
    (runtime/preload.py); it resumes the training from the preemption checkpoint."""
    env = {"TPI_FRAMEWORK_ROOT": ROOT, "TPI_TASK": "true", "TPI_PRELOAD": "1"}
    train = os.path.join(ROOT, "examples", "train", "train.py")
    script = ("#!%s\nimport runpy, sys\nsys.argv = [%r, '--steps', '600', '--hidden', '256', "
              "'--layers', '2', '--batch', '4', '--seq', '64', '--sleep', '0.05']\n"
              "sys.path.insert(0, %r)\nprint('torch preloaded', 'torch' in sys.modules, "
              "flush=True)\nrunpy.run_path(%r, run_name='__main__')\n"
              % (sys.executable, train, os.path.dirname(train), train))
    spec = Task(size=Size(machine="m+mi355x"),
                environment=Environment(script=script, timeout=600, variables=Variables(env)))
    task = backends.new(cloud, new_deterministic_identifier("gpu-preload"), spec)
    task.create()
    deadline = time.time() + 300
    while time.time() < deadline and not any(
            e.code == "standby-start" and "preloaded" in e.description for e in task.events()):
        time.sleep(0.1)
    assert any(e.code == "standby-start" for e in task.events()), task.logs()
    # the default (TPI_PRELOAD=1 = auto): the rank's main process alone holds
    # /dev/kfd, so the supervisor has the parked successor create its GPU context (gpu-lite)
    while time.time() < deadline and not any(e.code == "preload-gpu-warm"
                                             for e in task.events()):
        time.sleep(0.1)
    assert any(e.code == "preload-gpu-warm" for e in task.events()), [
        (e.code, e.description) for e in task.events()]
    time.sleep(4.0)  # its imports and its GPU context; it then parks
    task.preempt()
    status = task.wait(300)
    logs = task.logs()
    assert status["succeeded"] == 1, logs
    assert len(logs) == 2 and "preemption checkpoint saved" in logs[0], logs
    assert "torch preloaded False" in logs[0] and "torch preloaded True" in logs[1], logs
    resumed = [l for l in logs[1].splitlines() if "resumed from step" in l]
    assert resumed and int(resumed[0].rsplit(" ", 1)[1]) >= 1, logs[1]
    assert "done" in logs[1]
    assert any(e.code == "rank-start" and "warm standby" in e.description and
               "GPU warmed" in e.description for e in task.events()), [
        (e.code, e.description) for e in task.events()]
    assert not any(e.code == "preload-plain" for e in task.events())
    task.delete()


def test_training_state_on_device_carries_cpu_step_counters(tmp_path):
    from terraform_provider_iterative_amd.checkpoint import TrainingState, collect

    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.GELU(),
                                torch.nn.Linear(128, 64)).cuda().to(torch.bfloat16)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3)

    def train(n):
        for _ in range(n):
            model(torch.randn(4, 64, device="cuda", dtype=torch.bfloat16)).float().pow(2) \
                .mean().backward()
            opt.step()
            opt.zero_grad()

    train(3)
    tensors, host = collect(model, opt)
    assert host and all(k.endswith(".step") for k in host)  # AdamW keeps step on the CPU
    want = {k: v.clone() for k, v in {**tensors, **host}.items()}
    with TrainingState(model, opt, path=str(tmp_path / "spill"), codec="tpz1") as state:
        state.save({"iteration": 3})
        train(2)
        assert state.resume()["iteration"] == 3
        torch.cuda.synchronize()
    tensors2, host2 = collect(model, opt)
    for k, v in {**tensors2, **host2}.items():
        assert torch.equal(v, want[k]), k


def test_prefetched_spill_region_is_adopted(tmp_path):
    from terraform_provider_iterative_amd.checkpoint import Checkpointer, host, prefetch

    spill = str(tmp_path / "spill")
    src = {"w": torch.randn(1 << 20, device="cuda"), "b": torch.randn(4096, device="cuda")}
    ref = {k: v.clone() for k, v in src.items()}
    with Checkpointer(src, path=spill) as ck:
        ck.save({"step": 3})
    assert prefetch(spill) and spill in host._prefetched
    dst = {k: torch.zeros_like(v) for k, v in ref.items()}
    with Checkpointer(dst, path=spill) as ck:
        assert spill not in host._prefetched  # adopted, not mapped a second time
        assert ck.region.registered and ck.header()["metadata"] == {"step": 3}
        assert ck.restore().bad_tiles == 0
        torch.cuda.synchronize()
    assert all(torch.equal(dst[k], ref[k]) for k in ref)
    assert not prefetch(str(tmp_path / "missing"))


def test_prefetch_holds_pinning_while_an_hbm_hand_off_is_offered(tmp_path):
    """A spill with an HBM hand-off next to it (``<spill>.hbm``): the prefetched region is
    mapped but not registered (GPU page-table updates would slow the successor's IPC
    imports), until a copy needs it -- here the restore -- which releases the hold."""
    from terraform_provider_iterative_amd.checkpoint import Checkpointer, host, prefetch

    spill = str(tmp_path / "spill")
    src = {"w": torch.randn(8 << 20, device="cuda")}
    ref = {k: v.clone() for k, v in src.items()}
    with Checkpointer(src, path=spill) as ck:
        ck.save({"step": 1})
    open(spill + ".hbm", "w").write("{}")  # an offer (its content is not read here)
    assert prefetch(spill, window=2 << 20)
    region = host._prefetched[spill][1]["region"]
    time.sleep(1.0)  # touching finished long ago; registration waits for the release
    assert ops.hip().tpi_host_pin_ready(region.pinner) == 0
    os.remove(spill + ".hbm")
    dst = {k: torch.zeros_like(v) for k, v in ref.items()}
    with Checkpointer(dst, path=spill) as ck2:
        assert ck2.restore().bad_tiles == 0  # its copies wait for their windows: released
        torch.cuda.synchronize()
        assert ops.hip().tpi_host_pin_ready(ck2.region.pinner) > 0
    assert torch.equal(dst["w"], ref["w"])


@pytest.mark.parametrize("codec", ["none", "tpz1"])
def test_progressively_pinned_region_restores_across_windows(tmp_path, codec):
    # 2 MiB registration windows: chunks (1 MiB tiles, 3 MiB chunks) and compressed blobs
    # straddle window boundaries, the restore runs while later windows are still pinning,
    # and later saves into the windowed region split their copies the same way
    from terraform_provider_iterative_amd.checkpoint import Checkpointer, host, prefetch

    spill = str(tmp_path / "spill")
    gen = torch.Generator(device="cuda").manual_seed(5)
    src = {"w": torch.randn(5 << 20, device="cuda", generator=gen).to(torch.bfloat16),
           "m": torch.randn(3 << 20, device="cuda", generator=gen) * 1e-3,
           "t": torch.randn(999, 777, device="cuda", generator=gen).t()}
    ref = {k: v.clone() for k, v in src.items()}
    kw = dict(tile_bytes=1 << 20, chunk_bytes=3 << 20, nbuf=2, codec=codec)
    with Checkpointer(src, path=spill, **kw) as ck:
        ck.save({"step": 9})
    assert prefetch(spill, window=2 << 20)
    dst = {k: torch.zeros_like(v) for k, v in ref.items()}
    with Checkpointer(dst, path=spill, **kw) as ck:
        assert ck.region.pinner and ck.region.window == 2 << 20
        assert ck.restore().bad_tiles == 0 and ck.header()["metadata"] == {"step": 9}
        torch.cuda.synchronize()
        assert all(torch.equal(dst[k], ref[k]) for k in ref)
        for v in dst.values():
            v.mul_(2)
        want = {k: v.clone() for k, v in dst.items()}
        ck.save({"step": 10})
        for v in dst.values():
            v.zero_()
        assert ck.restore().bad_tiles == 0
        torch.cuda.synchronize()
        assert all(torch.equal(dst[k], want[k]) for k in want)
    assert spill not in host._prefetched


def test_early_prefetched_region_is_adopted(tmp_path):
    from terraform_provider_iterative_amd.checkpoint import Checkpointer, early_prefetch, host

    spill = str(tmp_path / "spill")
    src = {"w": torch.randn(1 << 20, device="cuda")}
    ref = {k: v.clone() for k, v in src.items()}
    with Checkpointer(src, path=spill, codec="tpz1") as ck:
        ck.save({"step": 5})
    assert early_prefetch(spill)
    dst = {k: torch.zeros_like(v) for k, v in ref.items()}
    with Checkpointer(dst, path=spill) as ck:
        assert spill not in host._prefetched and ck.region._mmap is not None
        assert ck.restore().bad_tiles == 0 and ck.header()["metadata"] == {"step": 5}
        torch.cuda.synchronize()
    assert torch.equal(dst["w"], ref["w"])


def test_remote_node_mi355x_task_stages_and_runs_on_the_gpu(tmp_path, monkeypatch):
    """``region = "host=..."`` with ``cloud = "mi355x"``: the workdir travels to the node,
    its runtime stages it into HBM and the rank sees the placed GPU (fake ssh transport)."""
    node_root = tmp_path / "node-state"
    node_root.mkdir()
    monkeypatch.setenv("FAKE_SSH_STATE_ROOT", str(node_root))
    monkeypatch.setenv("TPI_SSH_COMMAND", "%s %s" % (sys.executable,
                                                     os.path.join(ROOT, "tests", "fake_ssh.py")))
    monkeypatch.setenv("TPI_REMOTE_PYTHON", sys.executable)
    monkeypatch.delenv("TPI_MI355X_GPUS", raising=False)
    work = tmp_path / "w"
    work.mkdir()
    payload = np.random.default_rng(1).integers(0, 256, 80 << 20, dtype=np.uint8)
    (work / "data.bin").write_bytes(payload.tobytes())
    (work / "run.py").write_text(
        "import os, sys\nsys.path.insert(0, %r)\nimport torch\n"
        "from terraform_provider_iterative_amd.runtime.stage import attach\n"
        "t = attach().tensor('data.bin')\n"
        "print('gpus', torch.cuda.device_count(), os.environ.get('HIP_VISIBLE_DEVICES'),\n"
        "      'staged', t.device.type, int(t[:4096].sum()))\n" % ROOT)
    script = "#!/bin/sh\nexec %s run.py\n" % sys.executable
    spec = Task(size=Size(machine="m+mi355x"),
                environment=Environment(script=script, directory=str(work), timeout=300,
                                        variables=Variables({"TPI_STAGE": "hbm"})))
    task = backends.new(Cloud(provider="mi355x", region="host=gpu-box"),
                        new_deterministic_identifier("remote-gpu"), spec)
    task.create()
    deadline = time.time() + 240
    while time.time() < deadline:
        task.read()
        if task.status().get("succeeded", 0) + task.status().get("failed", 0):
            break
        time.sleep(0.5)
    log = "".join(task.logs())
    assert task.status()["succeeded"] == 1, log
    assert "gpus 1" in log and "staged cuda %d" % int(payload[:4096].sum()) in log, log
    assert task.gpus() and (node_root / "mi355x").is_dir()
    task.delete()


SPOT_GPU = r'''#!%(python)s
import os, sys, time
sys.path.insert(0, %(root)r)
import torch
from terraform_provider_iterative_amd.checkpoint import Checkpointer, preemption
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(3)
state = {"w": torch.zeros(64 << 20, device=dev), "noise": torch.randn(1 << 20, device=dev, generator=g)}
ck = Checkpointer(state, path=os.path.join(os.environ["TPI_DATA_DIRECTORY"], ".spill"))
meta = preemption.resume(ck)
start = (meta or {}).get("step", 0)
print("start", start, "gpu", os.environ.get("HIP_VISIBLE_DEVICES"), flush=True)
preemption.register(ck)
preemption.install()
for step in range(start, 60):
    state["w"].add_(1)
    torch.cuda.synchronize()
    time.sleep(0.03)
    preemption.step(step + 1)
print("final", int(state["w"][0].item()), int(state["w"][-1].item()), flush=True)
'''


def test_on_demand_task_reclaims_a_spot_task_on_the_gpu(cloud):
    """Spot semantics on one MI355X: the spot task holds the GPU, an on-demand task arrives,
    queues, reclaims it (the spot task checkpoints 256 MB of HBM state at a step boundary and
    goes back to the queue), runs a bf16 matmul, and the spot task resumes afterwards."""
    spot_spec = Task(size=Size(machine="m+mi355x"), spot=0,
                     environment=Environment(script=SPOT_GPU % {"python": sys.executable,
                                                                "root": ROOT},
                                             timeout=600, variables=Variables({"TPI_TASK": "true"})))
    spot = backends.new(cloud, new_deterministic_identifier("gpu-spot"), spot_spec)
    spot.create()
    deadline = time.time() + 300
    while time.time() < deadline and "start 0" not in "".join(spot.logs()):
        time.sleep(0.1)
    assert "start 0" in "".join(spot.logs()), spot.logs()
    time.sleep(0.5)
    od_script = ("#!%s\nimport torch\nx = torch.randn(4096, 4096, device='cuda', "
                 "dtype=torch.bfloat16)\nprint('on-demand', float((x @ x).float().abs().mean()), "
                 "flush=True)\n" % sys.executable)
    od = backends.new(cloud, new_deterministic_identifier("gpu-ondemand"),
                      Task(size=Size(machine="m+mi355x"),
                           environment=Environment(script=od_script, timeout=600,
                                                   variables=Variables({"TPI_TASK": "true"}))))
    od.create()
    assert od.wait(300)["succeeded"] == 1, od.logs()
    assert spot.wait(300)["succeeded"] == 1, spot.logs()
    logs = spot.logs()
    assert len(logs) == 2, logs
    resumed = int(logs[1].split("start ")[1].split()[0])
    assert 0 < resumed < 60 and "final 60 60" in logs[1], logs
    codes = [e.code for e in spot.events()]
    for code in ("requeue-requested", "preempt-boundary", "checkpoint-saved", "requeued",
                 "dequeued", "checkpoint-restored"):
        assert code in codes, (code, codes)
    od_codes = [e.code for e in od.events()]
    assert od_codes.index("queued") < od_codes.index("reclaim") < od_codes.index("placed")
    od.delete()
    spot.delete()


FAILING_SPILL = r'''#!%(python)s
import os, sys, time
sys.path.insert(0, %(root)r)
import torch
from terraform_provider_iterative_amd.checkpoint import Checkpointer, CheckpointError, preemption
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(11)
state = {"w": torch.zeros(32 << 20, device=dev), "noise": torch.randn(1 << 20, device=dev, generator=g)}
ck = Checkpointer(state, path=os.path.join(os.environ["TPI_DATA_DIRECTORY"], ".spill"))
meta = preemption.resume(ck)
start = (meta or {}).get("step", 0)
print("start", start, "restart", os.environ["TPI_RESTART_COUNT"], flush=True)
if start == 0:
    _save = ck.save
    def failing_save(metadata=None, on_stream=None, **kw):
        on_stream()      # "released": the successor starts and finds the exported HBM
        time.sleep(0.5)
        raise CheckpointError("host spill failed (injected)")
    ck.save = failing_save
preemption.register(ck)
preemption.install()
for step in range(start, 40):
    state["w"].add_(1)
    torch.cuda.synchronize()
    time.sleep(0.03)
    preemption.step(step + 1)
print("final", int(state["w"][0].item()), int(state["w"][-1].item()), flush=True)
'''


def test_failed_spill_hands_off_from_hbm_and_waits_for_close(cloud):
    """The host spill of a preempted rank fails after it exported its HBM: the successor
    restores from the predecessor's HBM (the only good copy), and the predecessor exits
    (code 1) only after the successor closed its IPC mappings."""
    spec = Task(size=Size(machine="m+mi355x"),
                environment=Environment(script=FAILING_SPILL % {"python": sys.executable,
                                                                 "root": ROOT},
                                        timeout=600, variables=Variables({"TPI_TASK": "true"})))
    task = backends.new(cloud, new_deterministic_identifier("gpu-failed-spill"), spec)
    task.create()
    deadline = time.time() + 300
    while time.time() < deadline and "start 0" not in "".join(task.logs()):
        time.sleep(0.1)
    time.sleep(0.5)
    task.preempt()
    status = task.wait(300)
    logs = task.logs()
    assert status["succeeded"] == 1, logs
    resumed = int(logs[1].split("start ")[1].split()[0])
    assert resumed > 0 and "final 40 40" in logs[1], logs
    events = task.events()
    codes = [e.code for e in events]
    restored = [e for e in events if e.code == "checkpoint-restored"]
    assert restored and restored[0].description[1] == "HBM hand-off", restored
    t = {c: next(e.time for e in events if e.code == c)
         for c in ("checkpoint-failed", "hbm-handoff-closed", "predecessor-exit",
                   "rank-released-exit")}
    assert t["checkpoint-failed"] <= t["predecessor-exit"]
    assert t["hbm-handoff-closed"] <= t["predecessor-exit"] <= t["rank-released-exit"], codes
    exit_ev = next(e for e in events if e.code == "rank-released-exit")
    assert "code 1" in exit_ev.description, exit_ev
    assert "checkpoint-not-durable" in codes
    task.delete()


HOLDING_EXPORTER = r'''
import os, sys
sys.path.insert(0, %(root)r)
import torch
from terraform_provider_iterative_amd.checkpoint import TrainingState
torch.manual_seed(7)
model = torch.nn.Sequential(torch.nn.Linear(256, 512), torch.nn.Linear(512, 64)).cuda()
state = TrainingState(model, path=%(spill)r)
meta = {"step": 12, "reason": "preempted", "consistency": "boundary"}
assert state.checkpointer.export_hbm(meta)
state.checkpointer.save(meta, on_stream=lambda: None)
print("exported", flush=True)
sys.stdin.readline()  # hold the memory until the successor is done
'''


def test_resume_consistent_takes_the_hbm_hand_off(tmp_path):
    """resume_consistent passes the agreed generation; when that is the exported
    state's generation the device-to-device copy must be used (0 bytes over PCIe)."""
    import subprocess

    import torch.distributed as dist

    from terraform_provider_iterative_amd.checkpoint import TrainingState

    spill = str(tmp_path / "spill")
    proc = subprocess.Popen([sys.executable, "-c", HOLDING_EXPORTER % {"root": ROOT,
                                                                       "spill": spill}],
                            stdin=subprocess.PIPE, stdout=subprocess.PIPE)
    try:
        assert proc.stdout.readline().strip() == b"exported"
        torch.manual_seed(7)
        want = torch.nn.Sequential(torch.nn.Linear(256, 512), torch.nn.Linear(512, 64)).cuda()
        model = torch.nn.Sequential(torch.nn.Linear(256, 512), torch.nn.Linear(512, 64)).cuda()
        for p in model.parameters():
            p.data.zero_()
        dist.init_process_group("gloo", store=dist.FileStore(str(tmp_path / "store"), 1),
                                rank=0, world_size=1)
        try:
            state = TrainingState(model, path=spill)
            meta = state.resume_consistent()
            torch.cuda.synchronize()
            assert meta["step"] == 12
            assert state.checkpointer.last_restore.wire_bytes == 0  # device to device
            state.checkpointer.wait_hbm_close()
            assert state.checkpointer.hbm_claim_owner() is None
            for a, b in zip(model.parameters(), want.parameters()):
                assert torch.equal(a, b)
            state.close()
        finally:
            dist.destroy_process_group()
    finally:
        proc.stdin.write(b"\n")
        proc.stdin.flush()
        proc.wait(60)


RELEASE_BEHIND = r'''
import json, sys, torch
sys.path.insert(0, %(root)r)
from terraform_provider_iterative_amd.checkpoint import Checkpointer
g = torch.Generator(device="cuda").manual_seed(21)
src = {"w%%d" %% i: torch.randn(64 << 20, device="cuda", generator=g) for i in range(6)}
src["view_a"] = src["w5"][: 1 << 20]
ref = {k: v.clone() for k, v in src.items()}
torch.cuda.synchronize()
ck = Checkpointer(src, path=%(spill)r, chunk_bytes=64 << 20, codec="tpz1")
before = torch.cuda.memory_reserved()
res = ck.save({"step": 1}, release_behind=True)
out = {"released": res.released_bytes,
       "emptied": all(t.untyped_storage().nbytes() == 0 for t in src.values()),
       "reserved_drop": before - torch.cuda.memory_reserved()}
ck.close()
dst = {k: torch.zeros_like(v) for k, v in ref.items() if k != "view_a"}
dst["view_a"] = dst["w5"][: 1 << 20]
with Checkpointer(dst, path=%(spill)r, chunk_bytes=64 << 20, codec="tpz1") as ck2:
    out["bad_tiles"] = ck2.restore().bad_tiles
    out["meta"] = ck2.header()["metadata"]
    torch.cuda.synchronize()
out["equal"] = all(torch.equal(dst[k], ref[k]) for k in ref)
print(json.dumps(out))
'''


def test_save_releases_device_memory_behind_the_spill(tmp_path):
    """Big-state preemption: with release_behind the device storages are freed while the
    spill runs (each once its tiles are in host memory) and handed back to the driver; the
    host copy is complete and restores into fresh tensors.  Run in a fresh process: in this
    one, a tensor an earlier test still holds can pin a cached segment the state would be
    carved from, and such a segment never goes back to the driver."""
    import json
    import subprocess

    proc = subprocess.run([sys.executable, "-c", RELEASE_BEHIND % {
        "root": ROOT, "spill": str(tmp_path / "spill")}], capture_output=True, text=True,
        timeout=180)
    assert proc.returncode == 0, proc.stderr[-3000:]
    out = json.loads(proc.stdout.strip().splitlines()[-1])
    assert out["released"] == 6 * (64 << 20) * 4 and out["emptied"], out
    assert out["reserved_drop"] >= out["released"], out
    assert out["bad_tiles"] == 0 and out["meta"] == {"step": 1} and out["equal"], out
