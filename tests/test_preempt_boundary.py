"""Step-consistent preemption checkpoints (checkpoint/preemption.py, checkpoint/agreement.py).

A SIGTERM may land anywhere in a training step.  The rank must save at the next step
boundary -- never between ``opt.step()`` and the step-counter update, never between two
moment updates of AdamW -- and all ranks of a gang must save the same step.  Every test
here runs a *non-idempotent* workload (AdamW on real data plus an accumulator ``acc += 1``)
and compares the final state of a preempted-and-resumed run with an uninterrupted run bit for
bit.  The reference leaves this to the user script (``README.md:88-101``: resume from
``results/epoch.txt``); here the runtime guarantees it.
"""
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

import pytest

from terraform_provider_iterative_amd import backends
from terraform_provider_iterative_amd.models.cloud import Cloud, Credentials, NodeCredentials
from terraform_provider_iterative_amd.models.values import Environment, Task, Variables
from terraform_provider_iterative_amd.utils.identifier import new_deterministic_identifier

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# One rank (or a gang with a manual gradient all-reduce) training a small MLP with AdamW on
# per-step deterministic data.  KILL_WHERE/KILL_AT choose where the first incarnation is
# preempted: the rank SIGTERMs itself there (or, with KILL_VIA=supervisor, asks the supervisor
# to preempt the whole gang) -- deterministic points inside the step.
WORKLOAD = r'''#!%(python)s
import hashlib, os, signal, sys, time
sys.path.insert(0, %(root)r)
import torch
from terraform_provider_iterative_amd.checkpoint import TrainingState, preemption

STEPS = %(steps)d
WHERE = os.environ.get("KILL_WHERE", "none")
AT = int(os.environ.get("KILL_AT", "-1"))
VIA = os.environ.get("KILL_VIA", "self")
first = os.environ.get("TPI_RESTART_COUNT", "0") == "0"
rank = int(os.environ.get("RANK", "0"))
world = int(os.environ.get("WORLD_SIZE", "1"))
if world > 1:
    import torch.distributed as dist
    dist.init_process_group("gloo")
torch.manual_seed(0)
torch.set_num_threads(1)
model = torch.nn.Sequential(torch.nn.Linear(16, 64), torch.nn.Tanh(), torch.nn.Linear(64, 4))
opt = torch.optim.AdamW(model.parameters(), lr=1e-2)
acc = torch.zeros(4, dtype=torch.float64)  # non-idempotent: += 1 per step
model(torch.zeros(1, 16)).sum().backward()
opt.step()  # optimizer state exists from here on (identical in every incarnation)
opt.zero_grad()
spill = os.path.join(os.environ.get("TPI_DATA_DIRECTORY", "."), ".spill-%%d" %% rank)
state = TrainingState(model, opt, extra={"acc": acc}, path=spill, tile_bytes=4096)
if world > 1:
    meta = state.resume_consistent()
else:
    meta = state.resume()
start = state.step_value or 0
print("start", start, (meta or {}).get("consistency"), flush=True)
state.install()

def kill(where, step):
    if first and where == WHERE and step == AT:
        if VIA == "supervisor":  # the supervisor preempts the whole gang
            os.kill(os.getppid(), signal.SIGUSR1)
            time.sleep(float(os.environ.get("KILL_SLEEP", "0")))
        else:
            os.kill(os.getpid(), signal.SIGTERM)

for step in range(start, STEPS):
    g = torch.Generator().manual_seed(1000 * (rank + 1) + step)
    x = torch.randn(32, 16, generator=g)
    y = torch.randn(32, 4, generator=g)
    loss = ((model(x) - y) ** 2).mean()
    opt.zero_grad()
    loss.backward()
    kill("after-backward", step)
    if world > 1:
        if rank == 1 and VIA == "supervisor":
            kill("before-allreduce", step)  # rank 0 is blocked in the all-reduce meanwhile
        for p in model.parameters():
            dist.all_reduce(p.grad)
            p.grad /= world
    opt.step()
    kill("after-opt-step", step)
    acc += 1
    kill("after-acc", step)
    state.step(step + 1)
    kill("after-boundary", step)
h = hashlib.sha256()
for t in list(model.state_dict().values()) + [acc]:
    h.update(t.detach().contiguous().numpy().tobytes())
for s in opt.state.values():
    for k in sorted(s):
        h.update(s[k].detach().contiguous().numpy().tobytes() if torch.is_tensor(s[k]) else repr(s[k]).encode())
print("final", rank, h.hexdigest(), flush=True)
state.close()
'''


@pytest.fixture()
def cloud(tmp_path):
    return Cloud(provider="local",
                 credentials=Credentials(node=NodeCredentials(state_root=str(tmp_path / "st"))))


def _script(steps=12):
    return WORKLOAD % {"python": sys.executable, "root": ROOT, "steps": steps}


def _reference(tmp_path, steps=12):
    """Final digest of an uninterrupted single-rank run (no supervisor)."""
    path = tmp_path / "ref.py"
    path.write_text(_script(steps))
    env = dict(os.environ, TPI_DATA_DIRECTORY=str(tmp_path), RANK="0", WORLD_SIZE="1")
    env.pop("TPI_EVENTS_FILE", None)
    out = subprocess.run([sys.executable, str(path)], env=env, capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stderr
    return _finals(out.stdout)


def _finals(text):
    return {int(l.split()[1]): l.split()[2] for l in text.splitlines()
            if l.split()[:1] == ["final"]}


def _run_task(cloud, name, env, parallelism=1, steps=12):
    spec = Task(parallelism=parallelism,
                environment=Environment(script=_script(steps), timeout=300,
                                        variables=Variables(dict(env, TPI_TASK="true"))))
    task = backends.new(cloud, new_deterministic_identifier(name), spec)
    task.create()
    status = task.wait(120)
    logs, events = task.logs(), task.events()
    task.delete()
    return status, logs, events


@pytest.mark.parametrize("where", ["after-backward", "after-opt-step", "after-acc",
                                   "after-boundary"])
def test_preempted_run_equals_uninterrupted_run(cloud, tmp_path, where):
    reference = _reference(tmp_path)
    status, logs, events = _run_task(cloud, "bnd-" + where,
                                     {"KILL_WHERE": where, "KILL_AT": "4"})
    assert status["succeeded"] == 1 and status["failed"] == 0, (status, logs)
    assert len(logs) == 2, logs
    finals = _finals("".join(l.split("Z ", 1)[-1] + "\n" for log in logs
                             for l in log.splitlines()))
    assert finals == reference, (where, finals, reference, logs)
    codes = [e.code for e in events]
    assert "preempt-boundary" in codes and "preempt-torn-risk" not in codes, codes
    boundary = [e for e in events if e.code == "preempt-boundary"][0]
    # a signal inside step 4 (0-based) is saved where step 5 ends; after the boundary, one later
    expect = 6 if where == "after-boundary" else 5
    assert boundary.description[1] == "boundary %d" % expect, boundary.description
    assert "step %d" % expect in boundary.description, boundary.description
    assert "start %d boundary" % expect in logs[1], logs[1]


def test_signal_time_save_is_torn(cloud, tmp_path):
    """Control experiment: the pre-boundary behaviour (TPI_PREEMPT_AT=signal) saves between
    opt.step() and the step counter, so the resumed run applies that update twice."""
    reference = _reference(tmp_path)
    status, logs, events = _run_task(cloud, "bnd-torn",
                                     {"KILL_WHERE": "after-opt-step", "KILL_AT": "4",
                                      "TPI_PREEMPT_AT": "signal"})
    assert status["succeeded"] == 1, (status, logs)
    finals = _finals("".join(l.split("Z ", 1)[-1] + "\n" for log in logs
                             for l in log.splitlines()))
    assert finals and finals != reference
    assert "start 4 signal" in logs[1], logs[1]


def test_no_boundary_falls_back_to_a_torn_risk_save(cloud, tmp_path):
    """A rank that never reaches the next boundary (stuck step) is saved by the watcher
    thread after TPI_PREEMPT_FALLBACK_SECONDS, marked torn-risk."""
    script = _script().replace("    kill(\"after-acc\", step)\n",
                               "    kill(\"after-acc\", step)\n"
                               "    if first and step == AT: time.sleep(30)\n")
    spec = Task(environment=Environment(script=script, timeout=300, variables=Variables({
        "TPI_TASK": "true", "KILL_WHERE": "after-acc", "KILL_AT": "4",
        "TPI_PREEMPT_FALLBACK_SECONDS": "0.5"})))
    task = backends.new(cloud, new_deterministic_identifier("bnd-fallback"), spec)
    task.create()
    status = task.wait(120)
    logs, events = task.logs(), task.events()
    task.delete()
    assert status["succeeded"] == 1, (status, logs)
    codes = [e.code for e in events]
    assert "preempt-torn-risk" in codes and "preempt-boundary" not in codes, codes
    assert "start 4 torn-risk" in logs[1], logs[1]
    t_sig = [e.time for e in events if e.code == "preempt-signal"][0]
    t_torn = [e.time for e in events if e.code == "preempt-torn-risk"][0]
    delta = (t_torn - t_sig).total_seconds()
    assert 0.4 <= delta < 5, delta


def _reference_gang(tmp_path, steps=12):
    """Final digests of an uninterrupted 2-rank gloo run (plain subprocesses)."""
    path = tmp_path / "ref2.py"
    path.write_text(_script(steps))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for rank in range(2):
        env = dict(os.environ, TPI_DATA_DIRECTORY=str(tmp_path), RANK=str(rank),
                   WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.pop("TPI_EVENTS_FILE", None)
        procs.append(subprocess.Popen([sys.executable, str(path)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    finals = {}
    for p in procs:
        out, err = p.communicate(timeout=120)
        assert p.returncode == 0, err
        finals.update(_finals(out))
    return finals


def test_gang_saves_the_same_step_while_a_rank_is_inside_a_collective(cloud, tmp_path):
    """Two gloo ranks; at step 4 rank 1 asks the supervisor to preempt the gang and then
    sleeps before its all-reduce, so the SIGTERM reaches rank 0 while it is blocked inside the
    collective (its Python handler cannot run).  Both ranks must save the same step, and the
    resumed gang must end bit-identical to an uninterrupted run."""
    reference = _reference_gang(tmp_path)
    status, logs, events = _run_task(
        cloud, "bnd-gang", {"KILL_WHERE": "before-allreduce", "KILL_AT": "4",
                            "KILL_VIA": "supervisor", "KILL_SLEEP": "1.5"}, parallelism=2)
    assert status["succeeded"] == 2 and status["failed"] == 0, (status, logs)
    finals = _finals("".join(l.split("Z ", 1)[-1] + "\n" for log in logs
                             for l in log.splitlines()))
    assert finals == reference, (finals, reference, logs)
    boundaries = [e for e in events if e.code == "preempt-boundary"]
    assert len(boundaries) == 2, [(e.code, e.description) for e in events]
    steps = {e.description[0]: e.description[2] for e in boundaries}
    assert set(steps) == {"rank 0", "rank 1"} and len(set(steps.values())) == 1, steps
    # the first rank at boundary 5 proposes it (or 6, if the other had already passed it)
    assert steps["rank 0"] in ("step 5", "step 6"), steps
    # rank 0 noticed the signal while blocked (watcher thread), before rank 1 woke up
    signals = {e.description[0]: e.time for e in events if e.code == "preempt-signal"}
    assert set(signals) == {"rank 0", "rank 1"}
    assert "preempt-torn-risk" not in [e.code for e in events]
    assert sum(("start %s boundary" % steps["rank 0"][5:]) in l for l in logs) == 2, logs


def _refuse_worker(rank, world, port, root, results, plan):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from terraform_provider_iterative_amd.checkpoint import TrainingState

        torch.manual_seed(rank)
        model = torch.nn.Linear(8, 8)
        opt = torch.optim.SGD(model.parameters(), lr=0.1)
        with TrainingState(model, opt, path=os.path.join(root, "r%d" % rank), tile_bytes=4096,
                           slots=2) as state:
            for meta in plan[rank]:  # oldest first
                with torch.no_grad():
                    model.weight.fill_(meta.get("step", 1))
                state.checkpointer.save(dict(meta, **state.host_metadata()))
            with torch.no_grad():
                model.weight.zero_()
            restored = state.resume_consistent()
            results[rank] = (None if restored is None else restored["step"],
                             float(model.weight[0, 0]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("plan,expect", [
    # the ranks' newest saves differ (rank 1 died mid-spill of step 6): the common step 5 wins
    ([[{"step": 5}, {"step": 6}], [{"step": 4}, {"step": 5}]], 5),
    # nothing in common: every rank starts fresh
    ([[{"step": 6}], [{"step": 5}]], None),
    # a torn-risk save is refused; the older boundary save in the other slot is used
    ([[{"step": 5}, {"step": 6, "consistency": "torn-risk"}],
      [{"step": 5}, {"step": 6, "consistency": "boundary"}]], 5),
    # a save without a step cannot be matched
    ([[{"reason": "x"}], [{"reason": "x"}]], None),
])
def test_resume_consistent_picks_the_newest_common_step(tmp_path, plan, expect):
    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    results = mp.Manager().dict()
    mp.spawn(_refuse_worker, args=(2, port, str(tmp_path), results, plan), nprocs=2)
    for rank in range(2):
        step, weight = results[rank]
        assert step == expect, (rank, step)
        assert weight == (expect or 0), (rank, weight)


def test_shm_agreement_protocol_under_skew(tmp_path):
    """ctl.cpp directly: 4 'ranks' (processes) at different boundary ordinals; one proposes a
    preemption; every rank must find the same target, ahead of all of them."""
    import multiprocessing as mp_

    from terraform_provider_iterative_amd.ops import native

    lib = native()
    world = 4
    path = str(tmp_path / "ctl")
    with open(path, "wb") as f:
        f.write(b"\0" * lib.ctl_bytes(world))
    ctx = mp_.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ctl_rank, args=(path, r, world, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=60) for _ in range(world)]
    for p in procs:
        p.join(30)
    targets = {t for _, t, _ in got}
    assert len(targets) == 1, got
    target = targets.pop()
    for rank, t, reached in got:
        assert reached == t, got  # every rank stopped exactly at the target


def _ctl_rank(path, rank, world, q):
    import mmap
    import random
    import ctypes

    from terraform_provider_iterative_amd.ops import native

    lib = native()
    fd = os.open(path, os.O_RDWR)
    m = mmap.mmap(fd, lib.ctl_bytes(world))
    addr = ctypes.addressof(ctypes.c_char.from_buffer(m))
    if rank == 0:
        lib.ctl_init(addr, world)
    while not lib.ctl_valid(addr, world):
        time.sleep(0.001)
    rng = random.Random(rank)
    ordinal, target = 0, 0
    while True:
        ordinal += 1
        pre, _ = lib.ctl_arrive(addr, rank, ordinal)
        if not pre and rank == 2 and ordinal == 50:
            pre = lib.ctl_propose_preempt(addr, world, rank)
        if pre and ordinal >= pre:
            target = pre
            break
        time.sleep(rng.random() * 0.002 * (rank + 1))  # skewed step times
    q.put((rank, target, ordinal))


BIG_STATE = r'''#!%(python)s
import os, sys, threading, time
sys.path.insert(0, %(root)r)
import torch
from terraform_provider_iterative_amd.checkpoint import Checkpointer, preemption
# A rank whose state is too big for two copies in HBM: until it has released its device
# memory there is no room for a successor (simulated: the hand-off check follows the flag).
released = threading.Event()
def fake_release():
    released.set()
    return 150 * 10**9
preemption._release_device_memory = fake_release
preemption._handoff_safe = released.is_set
state = {"w": torch.zeros(5000, dtype=torch.float64)}
ck = Checkpointer(state, path=os.path.join(os.environ["TPI_DATA_DIRECTORY"], ".spill"),
                  tile_bytes=4096)
meta = preemption.resume(ck)
start = (meta or {}).get("step", 0)
print("start", start, flush=True)
preemption.register(ck)
preemption.install()
for step in range(start, 40):
    state["w"] += 1
    time.sleep(0.05)
    preemption.step(step + 1)
print("final", int(state["w"][0]), flush=True)
'''


def test_big_state_rank_releases_hbm_before_the_hand_off(cloud):
    """State > half of HBM (no room for the successor's copy next to ours): the rank saves
    at the boundary, frees its device memory, then releases the successor while its host
    region stays pinned, and exits only after the successor restored -- instead of making
    the successor wait for its full exit."""
    spec = Task(environment=Environment(
        script=BIG_STATE % {"python": sys.executable, "root": ROOT}, timeout=300,
        # a loaded CI box can take longer than the default 20 s linger to start the successor
        variables=Variables({"TPI_TASK": "true", "TPI_LINGER_SECONDS": "120"})))
    task = backends.new(cloud, new_deterministic_identifier("big-state"), spec)
    task.create()
    deadline = time.time() + 60
    while time.time() < deadline and "start 0" not in "".join(task.logs()):
        time.sleep(0.05)
    time.sleep(0.3)
    task.preempt()
    status = task.wait(90)
    logs = task.logs()
    assert status["succeeded"] == 1, (status, logs)
    assert "final 40" in logs[1], logs
    events = task.events()
    codes = [e.code for e in events]
    # saved (not streamed: no room) -> HBM freed -> released -> successor restores -> exit
    assert "checkpoint-streaming" not in codes, codes
    order = ["checkpoint-saved", "device-memory-released", "checkpoint-released",
             "rank-released", "respawn", "checkpoint-restored", "predecessor-exit",
             "rank-released-exit"]
    idx = [codes.index(c) for c in order]
    assert idx == sorted(idx), list(zip(order, idx))
    exits = [e for e in events if e.code == "rank-released-exit"]
    assert "code 143" in exits[0].description
    task.delete()
