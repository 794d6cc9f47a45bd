#!/usr/bin/env python3
"""Config 5: 4 concurrent 2-GPU ``iterative_task`` resources on one node (placement +
auto-cleanup), driven through the node backend like ``tpi apply`` with Terraform's parallel
resource walk (4 creates in flight at once).

Reports, as one JSON line:

* ``create_s`` / ``first_log_s`` per task (from the moment all creates were issued);
* that the four GPU sets -- and the four tasks' reserved core sets -- are disjoint and cover
  the node, and that a fifth task is queued (``create`` returns, ``leo read`` says queued, like
  a scaling group without capacity) and starts as soon as GPUs are released
  (``queued_start_s``: last group exit -> the fifth task's first log);
* ``all_succeeded_s``: wall time until every supervisor exited with ``succeeded``;
* ``reuse_s``: time from the last supervisor exit until an 8-GPU task is placed on the
  released GPUs without any ``delete`` in between (lease auto-cleanup);
* ``delete_s``: destroying all five tasks.

In the reference, placement is a cloud API call per VM (ASG/MIG/VMSS resize, minutes); here
it is a lease-file allocator (parallel/placement.py).  On a node with fewer than 8 GPUs the
run uses 8 logical GPU slots (``TPI_MI355X_GPUS``) and says so in ``gpus``: the scripts only
echo, so oversubscribing the slots measures the orchestration path, not the device.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

SCRIPT = "#!/bin/sh\necho \"rank $RANK of $WORLD_SIZE on GPUs $HIP_VISIBLE_DEVICES\"\nsleep %s\n"
# --torch: every task also runs a bf16 matmul on each GPU it was given (real GPUs only)
TORCH = ("%s -c \"import torch; n = torch.cuda.device_count(); "
         "x = [torch.randn(4096, 4096, device=i, dtype=torch.bfloat16) for i in range(n)]; "
         "print('devices', n, 'sum', sum(float((a @ a).float().abs().sum()) for a in x))\"\n"
         % sys.executable)


def _first_log(task, t0: float, timeout: float) -> float:
    deadline = time.perf_counter() + timeout
    while time.perf_counter() < deadline:
        if any(chunk.strip() for chunk in task.logs()):
            return time.perf_counter() - t0
        time.sleep(0.0005)
    raise TimeoutError("no log from %s" % task.get_identifier().long())


def run(tasks: int = 4, gpus_per_task: int = 2, sleep: float = 1.0,
        torch_job: bool = False) -> dict:
    from terraform_provider_iterative_amd.parallel.placement import discover

    need = tasks * gpus_per_task
    physical = len(discover())
    keys = ("TPI_MI355X_GPUS", "TPI_NODE_CPUS", "TPI_NODE_MEMORY_MB")
    saved = {k: os.environ.get(k) for k in keys}
    if torch_job and physical < need:
        raise SystemExit("--torch needs %d GPUs, found %d" % (need, physical))
    logical = physical < need or saved["TPI_MI355X_GPUS"] is not None
    if physical < need:
        os.environ["TPI_MI355X_GPUS"] = ",".join(str(i) for i in range(need))
    if logical:  # logical slots stand for an 8-GPU node: its cores and DRAM too
        os.environ.setdefault("TPI_NODE_CPUS", "0-%d" % (16 * need - 1))
        os.environ.setdefault("TPI_NODE_MEMORY_MB", str(256000 * need))
    try:
        return _run(tasks, gpus_per_task, sleep, need, physical, torch_job, logical)
    finally:  # repeats must see the node again, not this run's logical slots
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _run(tasks: int, gpus_per_task: int, sleep: float, need: int, physical: int,
         torch_job: bool, logical: bool) -> dict:
    from terraform_provider_iterative_amd import backends
    from terraform_provider_iterative_amd.models.cloud import (Cloud, Credentials,
                                                               NodeCredentials)
    from terraform_provider_iterative_amd.models.values import (Environment, Size, Task,
                                                                Variables)
    from terraform_provider_iterative_amd.utils.identifier import new_deterministic_identifier

    state = tempfile.mkdtemp(prefix="tpi-concurrent-")
    cloud = Cloud(provider="mi355x",
                  credentials=Credentials(node=NodeCredentials(state_root=state)))

    def make(name: str, n: int, script: str):
        machine = "m+mi355x" if n == 1 else "16-64000+mi355x*%d" % n
        spec = Task(size=Size(machine=machine), parallelism=1,
                    environment=Environment(script=script, timeout=120,
                                            variables=Variables({"TPI_TASK": "true"})))
        return backends.new(cloud, new_deterministic_identifier(name), spec)

    body = SCRIPT % sleep + (TORCH if torch_job else "")
    group = [make("conc-%d-%d" % (os.getpid(), i), gpus_per_task, body)
             for i in range(tasks)]
    created = {}
    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(tasks) as pool:
        futures = {pool.submit(t.create): i for i, t in enumerate(group)}
        for fut in cf.as_completed(futures):
            fut.result()
            created[futures[fut]] = time.perf_counter() - t0
    first = [_first_log(t, t0, 30.0) for t in group]
    sets = [sorted(t.gpus()) for t in group]
    disjoint = len(set().union(*map(set, sets))) == need and all(len(s) == gpus_per_task
                                                                 for s in sets)
    cpu_sets = [sorted(c for cs in (t._definition().get("allocation") or {}).get("rank_cpus")
                       or [] for c in cs) for t in group]
    cpus_disjoint = sum(map(len, cpu_sets)) == len(set().union(*map(set, cpu_sets))) > 0
    extra = make("conc-extra-%d" % os.getpid(), 1, SCRIPT % 0)
    t1 = time.perf_counter()
    extra.create()
    queue_s = time.perf_counter() - t1
    queued = (extra.status() == {"running": 0, "succeeded": 0, "failed": 0}
              and not extra.gpus() and extra.supervisor_running())
    statuses = [t.wait(60.0) for t in group]
    t_done = time.perf_counter()
    all_ok = all(s.get("succeeded") == 1 for s in statuses)
    try:
        queued_start_s = _first_log(extra, t_done, 30.0)
    except TimeoutError:
        queued_start_s = None
    extra_ok = extra.wait(30.0).get("succeeded") == 1
    extra.delete()
    again = make("conc-after-%d" % os.getpid(), need, SCRIPT % 0)
    again.create()
    reuse_s = time.perf_counter() - t_done
    reused = sorted(again.gpus()) == list(range(need))
    again.wait(30.0)
    devices = [_devices(t.logs()) for t in group] if torch_job else None
    t2 = time.perf_counter()
    for t in group + [again]:
        t.delete()
    delete_s = time.perf_counter() - t2
    shutil.rmtree(state, ignore_errors=True)
    return {
        "config": "%d concurrent %d-GPU iterative_task resources on one node (placement + "
                  "auto-cleanup)" % (tasks, gpus_per_task),
        "gpus": {"physical": physical, "slots": need, "logical_slots": logical},
        "create_s": [round(created[i], 4) for i in range(tasks)],
        "first_log_s": [round(x, 4) for x in first],
        "gpu_sets": sets, "disjoint": disjoint,
        "cpu_sets": [_span(c) for c in cpu_sets], "cpus_disjoint": cpus_disjoint,
        "fifth_queued": queued, "queue_create_s": round(queue_s, 4),
        "queued_start_s": None if queued_start_s is None else round(queued_start_s, 4),
        "fifth_succeeded": extra_ok,
        "all_succeeded": all_ok, "all_succeeded_s": round(t_done - t0, 3),
        "task_sleep_s": sleep,
        "reuse_s": round(reuse_s, 4), "reused_all_gpus": reused,
        "delete_s": round(delete_s, 4),
        "torch_job": torch_job,
        "torch_devices": devices,
    }


def _span(cpus) -> str:
    return "%d-%d" % (cpus[0], cpus[-1]) if cpus else "-"


def _devices(logs) -> int:
    for chunk in logs:
        for line in chunk.splitlines():
            if " devices " in " " + line.split("Z ", 1)[-1] + " ":
                return int(line.split("devices", 1)[1].split()[0])
    return 0


def main() -> int:
    parser = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    parser.add_argument("--tasks", type=int, default=4)
    parser.add_argument("--gpus-per-task", type=int, default=2)
    parser.add_argument("--sleep", type=float, default=1.0)
    parser.add_argument("--repeats", type=int, default=3)
    parser.add_argument("--torch", action="store_true",
                        help="each task also runs a bf16 matmul on every GPU it was given")
    args = parser.parse_args()
    runs = [run(args.tasks, args.gpus_per_task, args.sleep, args.torch)
            for _ in range(args.repeats)]
    out = dict(runs[-1])
    out["repeats"] = len(runs)
    out["median_first_log_s"] = sorted(max(r["first_log_s"]) for r in runs)[len(runs) // 2]
    out["median_reuse_s"] = sorted(r["reuse_s"] for r in runs)[len(runs) // 2]
    out["ok"] = all(r["disjoint"] and r["cpus_disjoint"] and r["fifth_queued"]
                    and r["fifth_succeeded"] and r["all_succeeded"]
                    and r["reused_all_gpus"] and (not r["torch_job"] or
                                                  r["torch_devices"] == [args.gpus_per_task]
                                                  * args.tasks) for r in runs)
    print(json.dumps(out))
    return 0 if out["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
