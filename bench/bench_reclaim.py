#!/usr/bin/env python3
"""Spot reclaim on one MI355X: an on-demand task takes the GPU of a spot task that holds
``--gb`` of HBM state.

The spot task (``spot = 0``) runs a rank with ``--gb`` of synthetic AdamW state in HBM
(``bench.py``'s layout), registered with the preemption handler on a ``/dev/shm`` region.  Once
it is ready, an on-demand task is applied on the same node: it is queued (the GPU is taken),
reclaims the spot task -- which checkpoints at its next step boundary, frees its HBM, and
leaves without a hand-off (``TPI_REQUEUE_FILE``) -- and starts as soon as the spot task's
supervisor hands the GPU back (``resources-released``), while the victim process may still be
tearing down.  The on-demand script prints its first line, then allocates ``--od-gb`` of HBM
(proof that the victim's memory is really back) and exits; the spot task is then placed again
and resumes from its checkpoint, verifying the state digests.

Reported: on-demand apply -> first log / rank start / HBM allocated; spot reclaim request ->
checkpoint saved -> resources released (lease free) -> victim process reaped, with the
victim's ``exit-trace`` and ``predecessor-teardown`` journal lines; spot resume verified.

The reference replaces a reclaimed spot instance when capacity returns
(``resource_auto_scaling_group.go:51-106``) and scales its group to 0 right after the task
exits (``machine-script.sh.tpl:10-15``); it publishes no numbers.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SPOT_RANK = r'''#!%(python)s
import os, sys, time
sys.path.insert(0, %(root)r)
import torch
from bench import synthetic_checkpoint
from terraform_provider_iterative_amd import ops
from terraform_provider_iterative_amd.checkpoint import Checkpointer, preemption

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
spill = %(spill)r
resuming = os.path.exists(spill)
tensors = synthetic_checkpoint(int(%(gb)r * 1e9), 8192, dev, fill=not resuming)
torch.cuda.synchronize()
ck = Checkpointer(tensors, path=spill, codec="tpz1")
names = list(tensors)[:4]

def digests():
    return [ops.shard_hash(tensors[n].view(-1).view(torch.uint8)).cpu().tolist() for n in names]

if resuming:
    t0 = time.time()
    meta = preemption.resume(ck)
    torch.cuda.synchronize()
    ok = meta is not None and meta.get("digests") == digests()
    print("resumed step %%s in %%.3f s, verified %%s" %% ((meta or {}).get("step"),
                                                     time.time() - t0, ok), flush=True)
    ck.close()
    os.remove(spill)
    sys.exit(0 if ok else 3)
preemption.register(ck)
preemption.on_preempt(lambda: {"digests": digests()})
os.environ.setdefault("TPI_SYNC_INTERVAL", "0")
preemption.install()
print("ready %%d bytes in HBM" %% ck.plan.total, flush=True)
step = 0
while True:
    time.sleep(0.002)
    step += 1
    preemption.step(step)
'''

OD_RANK = r'''#!/bin/sh
echo "on-demand first log"
exec %(python)s -c '
import time
t0 = time.time()
import torch
x = torch.empty(int(%(gb)r * 1e9), dtype=torch.uint8, device="cuda")
x.fill_(1)
torch.cuda.synchronize()
print("on-demand allocated+wrote %%.1f GB in %%.3f s (import included)" %% (%(gb)r, time.time() - t0), flush=True)
'
'''


def main():
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--gb", type=float, default=100.0, help="HBM state of the spot task")
    p.add_argument("--od-gb", type=float, default=150.0,
                   help="HBM the on-demand task allocates once it runs")
    p.add_argument("--spill-dir", default="/dev/shm")
    p.add_argument("--timeout", type=float, default=600.0)
    args = p.parse_args()

    from terraform_provider_iterative_amd import backends
    from terraform_provider_iterative_amd.models.cloud import (Cloud, Credentials,
                                                               NodeCredentials)
    from terraform_provider_iterative_amd.models.values import (Environment, Size, Task,
                                                                Variables)
    from terraform_provider_iterative_amd.utils.identifier import new_random_identifier

    if shutil.disk_usage(args.spill_dir).free < args.gb * 1e9 * 1.02:
        raise SystemExit("not enough room in %s for the spill" % args.spill_dir)
    state = tempfile.mkdtemp(prefix="tpi-reclaim-")
    spill = os.path.join(args.spill_dir, "tpi-reclaim-%d.spill" % os.getpid())
    cloud = Cloud(provider="mi355x",
                  credentials=Credentials(node=NodeCredentials(state_root=state)))
    env = {"TPI_TASK": "true", "TPI_WARM_STANDBY": "0"}
    spot = backends.new(cloud, new_random_identifier("spot"), Task(
        size=Size(machine="m+mi355x"), spot=0,
        environment=Environment(script=SPOT_RANK % {"python": sys.executable, "root": ROOT,
                                                    "spill": spill, "gb": args.gb},
                                timeout=int(args.timeout) + 60, variables=Variables(env))))
    od = backends.new(cloud, new_random_identifier("ondemand"), Task(
        size=Size(machine="m+mi355x"),
        environment=Environment(script=OD_RANK % {"python": sys.executable, "gb": args.od_gb},
                                timeout=int(args.timeout) + 60, variables=Variables(env))))
    result = {"config": "Spot reclaim: on-demand task takes the GPU of a spot task holding "
                        "%.0f GB of HBM state (1 x MI355X)" % args.gb,
              "spot_gb": args.gb, "od_gb": args.od_gb}
    try:
        spot.create()
        deadline = time.time() + args.timeout
        while time.time() < deadline and not any("ready" in l for l in spot.logs()):
            if not spot.supervisor_running():
                raise SystemExit("spot task died: %s" % spot.logs())
            time.sleep(0.1)
        print("reclaim: spot ready, applying the on-demand task", file=sys.stderr, flush=True)
        t_apply = time.time()
        od.create()
        t_created = time.time()
        first_log = None
        while time.time() < deadline:
            if first_log is None and any("on-demand first log" in l for l in od.logs()):
                first_log = time.time()
            if first_log is not None and not od.supervisor_running():
                break
            time.sleep(0.005)
        print("reclaim: on-demand done, waiting for the spot task to resume",
              file=sys.stderr, flush=True)
        while time.time() < deadline and (spot.supervisor_running() or
                                          spot.status().get("succeeded", 0) < 1):
            if spot.status().get("failed", 0):
                break
            time.sleep(0.2)
        spot_events = [(e.code, e.time.timestamp(), e.description) for e in spot.events()]
        od_events = [(e.code, e.time.timestamp(), e.description) for e in od.events()]

        def first(events, code, after=0.0):
            return next((t for c, t, _ in events if c == code and t >= after), None)

        t_req = first(spot_events, "requeue-requested")
        marks = {
            "od_create_returned_s": t_created - t_apply,
            "od_apply_to_first_log_s": (first_log - t_apply) if first_log else None,
            "od_apply_to_rank_start_s": (first(od_events, "rank-start") or 0) - t_apply,
            "od_apply_to_reclaim_s": (first(od_events, "reclaim") or 0) - t_apply,
            "spot_request_to_boundary_s": first(spot_events, "preempt-boundary", t_req or 0),
            "spot_request_to_saved_s": first(spot_events, "checkpoint-saved", t_req or 0),
            "spot_request_to_hbm_released_s": first(spot_events, "device-memory-released",
                                                    t_req or 0),
            "spot_request_to_released_s": first(spot_events, "rank-released", t_req or 0),
            "spot_request_to_resources_released_s": first(spot_events, "resources-released",
                                                          t_req or 0),
            "spot_request_to_process_reaped_s": first(spot_events, "rank-released-exit",
                                                      t_req or 0),
        }
        for key, value in list(marks.items()):
            if key.startswith("spot_") and value is not None and t_req:
                marks[key] = value - t_req
            if isinstance(marks[key], float):
                marks[key] = round(marks[key], 4)
        result.update(marks)
        result["spot_timeline"] = [[c, round(t - (t_req or t_apply), 4), d]
                                   for c, t, d in spot_events if t >= (t_req or t_apply)]
        result["od_timeline"] = [[c, round(t - t_apply, 4), d] for c, t, d in od_events]
        result["od_logs"] = [l.strip() for l in od.logs()]
        result["spot_logs_tail"] = [l.strip().splitlines()[-1] for l in spot.logs() if l.strip()]
        result["spot_resumed_verified"] = any("verified True" in l for l in spot.logs())
        result["ok"] = bool(result["spot_resumed_verified"] and first_log is not None
                            and od.status().get("succeeded") == 1)
    finally:
        for task in (od, spot):
            try:
                task.delete()
            except Exception as error:  # report, keep cleaning
                print("reclaim: delete %s: %s" % (task.id, error), file=sys.stderr)
        shutil.rmtree(state, ignore_errors=True)
        if os.path.exists(spill):
            os.remove(spill)
    print(json.dumps(result))


if __name__ == "__main__":
    main()
