"""Bit-identical resume of an *ordinary* training loop.

The loop draws from every global generator (dropout masks from torch's CPU generator, input
noise from Python's ``random`` and NumPy's), follows an LR schedule (OneCycleLR: the
optimizer's lr changes every step), scales its loss with an AMP ``GradScaler`` whose scale
grows during the run, and reads its samples in a shuffled order (:class:`DataCursor`).  It is
preempted at several points inside a step (the rank SIGTERMs itself there); the save happens at
the next step boundary, the successor resumes, and its final state -- parameters, optimizer
moments, lr, scheduler, scaler and data position -- must equal an uninterrupted run's bit for
bit.  The reference leaves all of this to the user script (README.md:88-101).
"""
import os
import subprocess
import sys

import pytest

from terraform_provider_iterative_amd import backends
from terraform_provider_iterative_amd.models.cloud import Cloud, Credentials, NodeCredentials
from terraform_provider_iterative_amd.models.values import Environment, Task, Variables
from terraform_provider_iterative_amd.utils.identifier import new_deterministic_identifier

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

LOOP = r'''#!%(python)s
import hashlib, os, random, signal, sys
sys.path.insert(0, %(root)r)
import numpy as np
import torch
from terraform_provider_iterative_amd.checkpoint import DataCursor, TrainingState

STEPS = %(steps)d
WHERE = os.environ.get("KILL_WHERE", "none")
AT = int(os.environ.get("KILL_AT", "-1"))
first = os.environ.get("TPI_RESTART_COUNT", "0") == "0"
DEV = os.environ.get("LOOP_DEVICE", "cpu")
torch.set_num_threads(1)
torch.manual_seed(0)
random.seed(1)
np.random.seed(2)
data = torch.randn(64, 16, generator=torch.Generator().manual_seed(5)).to(DEV)
target = torch.randn(64, 4, generator=torch.Generator().manual_seed(6)).to(DEV)
model = torch.nn.Sequential(torch.nn.Linear(16, 64), torch.nn.Dropout(0.3), torch.nn.GELU(),
                            torch.nn.Linear(64, 4)).to(DEV)
opt = torch.optim.AdamW(model.parameters(), lr=1e-2)
sched = torch.optim.lr_scheduler.OneCycleLR(opt, max_lr=3e-2, total_steps=STEPS + 1)
scaler = torch.amp.GradScaler(DEV, init_scale=2.0 ** 8, growth_interval=3)
cursor = DataCursor(len(data), seed=3)
aug = torch.Generator(device=DEV).manual_seed(9)  # its own generator, handed to TrainingState
model(torch.zeros(1, 16, device=DEV)).sum().backward()  # optimizer state exists from here on
opt.step()
opt.zero_grad()
state = TrainingState(model, opt, path=os.path.join(os.environ.get("TPI_DATA_DIRECTORY", "."),
                                                   ".spill"), tile_bytes=4096,
                      lr_scheduler=sched, scaler=scaler, generators={"aug": aug},
                      stateful={"cursor": cursor})
meta = state.resume()
start = state.step_value or 0
print("start", start, flush=True)
state.install()

def kill(where, step):
    if first and where == WHERE and step == AT:
        os.kill(os.getpid(), signal.SIGTERM)

for step in range(start, STEPS):
    idx = cursor.next(8)
    x = data[idx] + 0.01 * random.random() + torch.from_numpy(
        np.random.normal(0, 0.01, size=(8, 16)).astype(np.float32)).to(DEV)
    x = x + 0.01 * torch.randn(8, 16, generator=aug, device=DEV)
    loss = ((model(x) - target[idx]) ** 2).mean()  # dropout: the device's default generator
    kill("after-forward", step)
    opt.zero_grad()
    scaler.scale(loss).backward()
    kill("after-backward", step)
    scaler.step(opt)
    scaler.update()
    kill("after-opt-step", step)
    sched.step()
    kill("after-sched", step)
    state.step(step + 1)
    kill("after-boundary", step)
h = hashlib.sha256()
for t in model.state_dict().values():
    h.update(t.detach().cpu().contiguous().numpy().tobytes())
for s in opt.state.values():
    for k in sorted(s):
        h.update(s[k].detach().cpu().contiguous().numpy().tobytes())
h.update(repr([g["lr"] for g in opt.param_groups]).encode())
h.update(repr(sched.state_dict()).encode())
h.update(repr(scaler.state_dict()).encode())
h.update(repr(cursor.state_dict()).encode())
h.update(repr((torch.rand(3).tolist(), torch.rand(3, device=DEV).tolist(), random.random(),
               np.random.rand())).encode())
print("final", h.hexdigest(), "scale", scaler.get_scale(), flush=True)
state.close()
'''


def _script(steps=14):
    return LOOP % {"python": sys.executable, "root": ROOT, "steps": steps}


def _reference(d, device="cpu"):
    path = d / "loop.py"
    path.write_text(_script())
    env = dict(os.environ, TPI_DATA_DIRECTORY=str(d), LOOP_DEVICE=device)
    env.pop("TPI_EVENTS_FILE", None)
    out = subprocess.run([sys.executable, str(path)], env=env, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr
    final = [l for l in out.stdout.splitlines() if l.startswith("final")]
    assert final and "scale 256.0" not in final[0]  # the scaler's scale did grow
    return final[0]


@pytest.fixture(scope="module")
def reference(tmp_path_factory):
    return _reference(tmp_path_factory.mktemp("ref"))


def _preempted_run(cloud, name, where, device="cpu", machine=None):
    from terraform_provider_iterative_amd.models.values import Size

    spec = Task(size=Size(machine=machine) if machine else Size(),
                environment=Environment(script=_script(), timeout=300, variables=Variables(
                    {"TPI_TASK": "true", "KILL_WHERE": where, "KILL_AT": "6",
                     "LOOP_DEVICE": device})))
    task = backends.new(cloud, new_deterministic_identifier(name), spec)
    task.create()
    status = task.wait(240)
    logs = task.logs()
    task.delete()
    return status, logs


@pytest.mark.parametrize("where", ["after-forward", "after-backward", "after-opt-step",
                                   "after-sched", "after-boundary"])
def test_preempted_loop_resumes_bit_identically(tmp_path, reference, where):
    cloud = Cloud(provider="local",
                  credentials=Credentials(node=NodeCredentials(state_root=str(tmp_path / "st"))))
    status, logs = _preempted_run(cloud, "resume-" + where, where)
    assert status["succeeded"] == 1, (status, logs)
    assert len(logs) == 2, logs  # preempted once, resumed once
    resumed = int(logs[1].split("start ")[1].split()[0])
    # saved at the boundary that ends step 6 (the SIGTERM came during it), or the next one
    assert resumed == (8 if where == "after-boundary" else 7), logs
    final = [l for l in logs[1].splitlines() if " final " in l][0].split("Z ", 1)[1]
    assert final == reference


def test_header_round_trip_of_host_state():
    import numpy as np
    import torch

    from terraform_provider_iterative_amd.checkpoint.training import (from_jsonable,
                                                                      to_jsonable)

    value = {"a": (1, 2.5, None), 3: [b"\x00\xff", np.arange(3, dtype=np.uint32)],
             "t": torch.tensor([1.5, -2.0], dtype=torch.bfloat16), "__odd": True}
    back = from_jsonable(__import__("json").loads(__import__("json").dumps(to_jsonable(value))))
    assert back["a"] == (1, 2.5, None) and back[3][0] == b"\x00\xff"
    assert back[3][1].dtype == np.uint32 and back[3][1].tolist() == [0, 1, 2]
    assert back["t"].dtype == torch.bfloat16 and back["t"].tolist() == [1.5, -2.0]
    assert back["__odd"] is True
    with pytest.raises(TypeError):
        to_jsonable({"f": lambda: None})


@pytest.mark.gpu
@pytest.mark.parametrize("where", ["after-forward", "after-opt-step"])
def test_preempted_loop_resumes_bit_identically_on_the_gpu(tmp_path, monkeypatch, where):
    """The same loop on the MI355X (dropout from the GPU's Philox generator, a CUDA
    GradScaler, device tensors through the HIP checkpoint pipeline)."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    monkeypatch.delenv("TPI_MI355X_GPUS", raising=False)
    reference = _reference(tmp_path, "cuda")
    cloud = Cloud(provider="mi355x",
                  credentials=Credentials(node=NodeCredentials(state_root=str(tmp_path / "st"))))
    status, logs = _preempted_run(cloud, "gpu-resume-" + where, where, "cuda", "m+mi355x")
    assert status["succeeded"] == 1, (status, logs)
    assert len(logs) == 2 and "start 7" in logs[1], logs
    final = [l for l in logs[1].splitlines() if " final " in l][0].split("Z ", 1)[1]
    assert final == reference


def _materialize_round_trip(tmp_path, device):
    """Train, save, then rebuild model + optimizer + scheduler around the materialized tensors
    (model built on the meta device) and continue: bit-identical to the uninterrupted run."""
    import torch

    from terraform_provider_iterative_amd.checkpoint import TrainingState, preemption

    def make_model():
        return torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.GELU(),
                                   torch.nn.Linear(32, 4))

    def make_opt(m):
        return torch.optim.AdamW(m.parameters(), lr=1e-2)

    def make_sched(o):
        return torch.optim.lr_scheduler.StepLR(o, 2, 0.5)

    def train(model, opt, sched, steps, gen):
        for _ in range(steps):
            x = torch.randn(8, 16, generator=gen).to(device)
            model(x).pow(2).mean().backward()
            opt.step()
            sched.step()
            opt.zero_grad()

    torch.manual_seed(0)
    model = make_model().to(device)
    opt, gen = make_opt(model), torch.Generator().manual_seed(1)
    sched = make_sched(opt)
    train(model, opt, sched, 3, gen)
    path = str(tmp_path / "spill")
    state = TrainingState(model, opt, path=path, tile_bytes=4096, lr_scheduler=sched,
                          generators={"g": gen})
    state.save({"step": 3})
    train(model, opt, sched, 2, gen)  # the uninterrupted run
    state.close()

    with torch.device("meta"):
        fresh = make_model()
    got = preemption.materialize(path, device)
    assert got is not None
    gen2 = torch.Generator()
    resumed = TrainingState.from_materialized(got, fresh, make_opt, make_lr_scheduler=make_sched,
                                              generators={"g": gen2})
    assert resumed.step_value == 3 and all(p.device.type == torch.device(device).type
                                           for p in fresh.parameters())
    train(fresh, resumed.optimizer, resumed.lr_scheduler, 2, gen2)
    for (name, a), b in zip(model.state_dict().items(), fresh.state_dict().values()):
        assert torch.equal(a, b), name
    assert resumed.optimizer.param_groups[0]["lr"] == opt.param_groups[0]["lr"]
    for p, q in zip(model.parameters(), fresh.parameters()):
        for key in ("exp_avg", "exp_avg_sq", "step"):
            assert torch.equal(opt.state[p][key].cpu(), resumed.optimizer.state[q][key].cpu())
    resumed.save({"step": 5})  # the materialized checkpointer keeps saving into the region
    resumed.close()


def test_from_materialized_resumes_bit_identically(tmp_path):
    _materialize_round_trip(tmp_path, "cpu")


@pytest.mark.gpu
def test_from_materialized_resumes_bit_identically_on_the_gpu(tmp_path):
    _materialize_round_trip(tmp_path, "cuda")


def test_from_materialized_warns_about_non_persistent_buffers(tmp_path):
    import torch

    from terraform_provider_iterative_amd.checkpoint import TrainingState, preemption

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.lin = torch.nn.Linear(8, 8)
            self.register_buffer("cache", torch.arange(8.0), persistent=False)

    net = Net()
    path = str(tmp_path / "spill")
    state = TrainingState(net, path=path, tile_bytes=4096)
    state.save({"step": 1})
    state.close()
    with torch.device("meta"):
        fresh = Net()
    with pytest.warns(UserWarning, match="cache"):
        resumed = TrainingState.from_materialized(preemption.materialize(path, "cpu"), fresh)
    assert torch.equal(fresh.lin.weight, net.lin.weight) and fresh.cache.is_meta
    resumed.close()
