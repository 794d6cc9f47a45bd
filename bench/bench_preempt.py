#!/usr/bin/env python3
"""Config 4 end to end: SIGTERM mid-task -> checkpoint pack -> host DRAM -> respawn -> restore.

An ``iterative_task`` on ``cloud = "mi355x"`` runs a rank that holds ``--gb`` of synthetic
AdamW state in HBM (bf16 params + fp32 moments, as ``bench.py``), registered with the
preemption handler on a file-backed host region (``--spill-dir``, default ``/dev/shm``, so the
spill outlives the rank process).  Once the rank reports ready, ``leo preempt`` (SIGUSR1 to the
supervisor -> SIGTERM to the rank) fires; the rank spills and exits 143, the supervisor
respawns it with a new machine identity, and the successor restores the state and checks the
shard-hash digests recorded before the preemption.

Reported from the task's phase journal (``supervisor/events.jsonl``): save time and GB/s, the
respawn gap, process start -> restore done, restore GB/s, and signal -> state back in HBM.
The reference recovers a spot VM by re-provisioning it and ``rclone copy``-ing the bucket's
``data/`` prefix back (``machine-script.sh.tpl:89``); it publishes no numbers.
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

RANK = r'''#!%(python)s
import os, sys, time
t_start = time.time()
sys.path.insert(0, %(root)r)
from terraform_provider_iterative_amd.checkpoint import early_prefetch
if %(early)r and os.path.exists(%(spill)r):
    early_prefetch(%(spill)r)  # map + pin the spill while torch is being imported
import torch
t_import = time.time()
from bench import synthetic_checkpoint
from terraform_provider_iterative_amd import ops
from terraform_provider_iterative_amd.checkpoint import Checkpointer, prefetch, preemption

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
spill = %(spill)r
nbytes = int(%(gb)r * 1e9)
# warm standby: the successor waits here (imports done, spill being mapped) for its activation
materialize = %(materialize)r
activated = (preemption.standby(spill if %(prefetch)r else None, materialize=materialize)
             if %(standby)r else False)
t_active = time.time()
resuming = os.path.exists(spill)
if resuming and %(prefetch)r:
    prefetch(spill)  # map + pin the spill while the model state is being allocated
t_prefetch = time.time()
free_before = torch.cuda.mem_get_info(0)[0]
probe = torch.empty(1 << 20, dtype=torch.uint8, device=dev)  # context + allocator warm
torch.cuda.synchronize()
t_probe = time.time()

def digests():
    return [ops.shard_hash(tensors[n].view(-1).view(torch.uint8)).cpu().tolist() for n in names]

if resuming and materialize:
    # the state is allocated group by group as the predecessor frees its HBM, each group
    # restored behind the predecessor's spill: no up-front allocation of the whole state
    t0 = time.time()
    ck, tensors, meta = preemption.materialize(spill, dev)
    torch.cuda.synchronize()
    t1 = time.time()
    names = list(tensors)[:4]
    ok = meta is not None and meta.get("digests") == digests()
    print("restored %%d bytes in %%.3f s, verified %%s, warm standby %%s, materialized %%s, "
          "activation -> restored %%.3f s (prefetch %%.3f, %%.1f GB free before); "
          "process start -> import done %%.3f s; Checkpointer %%s" %% (
              ck.plan.total, t1 - t0, ok, activated, ck.materialize_stats, t1 - t_active,
              t_prefetch - t_active, free_before / 1e9, t_import - t_start, ck.init_times),
          flush=True)
    ck.wait_stream(timeout=600)
    ck.close()
    os.remove(spill)
    sys.exit(0 if ok else 3)
extra = %(extra)r  # GiB each: single tensors of 2 GiB or more (a large vocabulary's fp32
                   # embedding / Adam moments), beyond what HIP IPC can hand off
tensors = synthetic_checkpoint(nbytes - int(sum(extra) * 2 ** 30), 8192, dev, fill=not resuming)
gen = torch.Generator(device=dev).manual_seed(77)
for i, gib in enumerate(extra):
    big = torch.empty(int(gib * 2 ** 30) // 4, dtype=torch.float32, device=dev)
    if not resuming:
        big.normal_(0, 1e-3, generator=gen)
    tensors["embedding.%%d" %% i] = big
torch.cuda.synchronize()
t_alloc = time.time()
ck = Checkpointer(tensors, path=spill, codec=%(codec)r)
t_map = time.time()
names = list(tensors)[:4]

if resuming:
    # no zero-fill needed to prove the restore: a fresh process's allocations never hold the
    # saved bytes, so the digest check below fails unless the restore wrote every tensor
    t0 = time.time()
    meta = preemption.resume(ck)
    torch.cuda.synchronize()
    t1 = time.time()
    ok = meta is not None and meta.get("digests") == digests()
    print("restored %%d bytes in %%.3f s, verified %%s, warm standby %%s, activation -> restored "
          "%%.3f s (prefetch %%.3f, HBM state %%.3f [first 1 MiB %%.3f, %%.1f GB free before], "
          "host region map+register %%.3f after it); "
          "process start -> import done %%.3f s; Checkpointer %%s" %% (
              ck.plan.total, t1 - t0, ok, activated, t1 - t_active, t_prefetch - t_active,
              t_alloc - t_prefetch, t_probe - t_prefetch, free_before / 1e9, t_map - t_alloc,
                                  t_import - t_start, ck.init_times),
          flush=True)
    # the predecessor is still spilling behind the HBM hand-off: wait for the host copy, so
    # the journal shows when this resumed state became durable (checkpoint-durable)
    ck.wait_stream(timeout=600)
    ck.close()
    os.remove(spill)
    sys.exit(0 if ok else 3)
preemption.register(ck)
# the verification oracle: the loop below never changes the state, so its digests are taken
# once here rather than inside the preemption save (where hashing 100 GB and syncing per
# tensor added ~7 ms to signal -> restored that a real script's metadata would not)
state_digests = digests()
preemption.on_preempt(lambda: {"digests": state_digests})
os.environ.setdefault("TPI_SYNC_INTERVAL", "0")  # preemption saves only
preemption.install()
print("ready %%d bytes in HBM" %% ck.plan.total, flush=True)
step = 0
while True:  # a "training loop" whose steps leave the state consistent at every boundary
    time.sleep(%(step_s)r)
    step += 1
    if %(boundary)r:
        preemption.step(step)  # a SIGTERM is saved here, at most one step after it arrived
'''


def main():
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--gb", type=float, default=100.0)
    p.add_argument("--codec", choices=("none", "tpz1"), default="tpz1")
    p.add_argument("--spill-dir", default="/dev/shm")
    p.add_argument("--timeout", type=float, default=900.0)
    p.add_argument("--standby", action="store_true",
                   help="the rank script calls preemption.standby(): its successor is started "
                        "warm at the preemption (the supervisor's default for such scripts)")
    p.add_argument("--hot", action="store_true",
                   help="hot standby (TPI_WARM_STANDBY=hot): the successor is started with the "
                        "rank, so it is ready to restore behind the streamed spill")
    p.add_argument("--preload", action="store_true",
                   help="TPI_PRELOAD=1 (the default): the successor is a preloaded interpreter "
                        "(PyTorch imported before the preemption, runtime/preload.py)")
    p.add_argument("--preload-gpu", action="store_true",
                   help="TPI_PRELOAD=gpu: the preloaded successor has also initialised the GPU "
                        "and prewarmed a checkpoint engine")
    p.add_argument("--preload-gpu-lite", action="store_true",
                   help="TPI_PRELOAD=gpu-lite: the preloaded successor has initialised the GPU "
                        "(context, first queue) but made no engine")
    p.add_argument("--no-preload", action="store_true",
                   help="TPI_PRELOAD=0: the successor is a fresh process")
    p.add_argument("--no-stream", action="store_true",
                   help="TPI_STREAM_HANDOFF=0: release the successor only after the spill")
    p.add_argument("--no-prefetch", action="store_true",
                   help="successor maps its host region only when the Checkpointer is built")
    p.add_argument("--early-prefetch", action="store_true",
                   help="successor maps + pins the spill before importing torch (measured "
                        "slower on MI355X: the pinning stalls the import)")
    p.add_argument("--materialize", action="store_true",
                   help="the successor restores with preemption.materialize(): its state is "
                        "allocated group by group while the predecessor frees its HBM")
    p.add_argument("--step-seconds", type=float, default=0.002,
                   help="duration of the rank's (idle) training step")
    p.add_argument("--extra-gib", default="",
                   help="comma list: also hold single fp32 tensors of these sizes (GiB) inside "
                        "the --gb total, e.g. 4.2,2.5")
    p.add_argument("--signal-mode", action="store_true",
                   help="the rank never calls preemption.step(): save in the signal handler")
    args = p.parse_args()
    if args.hot:
        args.standby = True

    from terraform_provider_iterative_amd import backends
    from terraform_provider_iterative_amd.models.cloud import (Cloud, Credentials,
                                                               NodeCredentials)
    from terraform_provider_iterative_amd.models.values import (Environment, Size, Task,
                                                                Variables)
    from terraform_provider_iterative_amd.utils.identifier import new_random_identifier

    need = args.gb * 1e9 * 1.02
    free = shutil.disk_usage(args.spill_dir).free
    if free < need:  # a tmpfs that cannot hold the spill would SIGBUS the rank mid-save
        raise SystemExit("need %.0f GB free in %s for the spill, have %.0f"
                         % (need / 1e9, args.spill_dir, free / 1e9))
    state = tempfile.mkdtemp(prefix="tpi-preempt-")
    spill = os.path.join(args.spill_dir, "tpi-preempt-%d.spill" % os.getpid())
    cloud = Cloud(provider="mi355x",
                  credentials=Credentials(node=NodeCredentials(state_root=state)))
    script = RANK % {"python": sys.executable, "root": ROOT, "spill": spill, "gb": args.gb,
                     "codec": args.codec, "prefetch": not args.no_prefetch,
                     "early": args.early_prefetch, "standby": args.standby,
                     "step_s": args.step_seconds, "boundary": not args.signal_mode,
                     "materialize": args.materialize,
                     "extra": [float(x) for x in args.extra_gib.split(",") if x.strip()]}
    # the ranks' runtime knobs travel as task variables (the rank environment is the task's)
    rank_env = {"TPI_TASK": "true", "TPI_STREAM_HANDOFF": "0" if args.no_stream else "1"}
    if args.preload or args.no_preload or args.preload_gpu or args.preload_gpu_lite:
        rank_env["TPI_PRELOAD"] = "0" if args.no_preload else (
            "gpu" if args.preload_gpu else ("gpu-lite" if args.preload_gpu_lite else "1"))
    preload = (not args.no_preload and not args.hot and
               (args.preload or args.preload_gpu or args.preload_gpu_lite or
                os.environ.get("TPI_PRELOAD", "1") not in ("0", "false", "no")))
    for knob in ("TPI_D2H_ENGINE", "TPI_STREAM_TIMEOUT", "TPI_LINGER_SECONDS",
                 "TPI_HBM_HANDOFF", "TPI_RELEASE_HBM", "TPI_EXPLICIT_TEARDOWN",
                 "HSA_ENABLE_SDMA", "GPU_MAX_HW_QUEUES", "TPI_DIRECT_META",
                 "TPI_ALLOC_LOOKAHEAD", "TPI_MATERIALIZE_H2D", "TPI_HBM_ROUTE",
                 "TPI_HANDOFF_VERIFY", "TPI_HANDOFF_UNROLL", "TPI_HANDOFF_SPAN_MB"):
        if os.environ.get(knob):
            rank_env[knob] = os.environ[knob]
    spec = Task(size=Size(machine="m+mi355x"),
                environment=Environment(script=script, timeout=int(args.timeout) + 60,
                                        variables=Variables(rank_env)))
    task = backends.new(cloud, new_random_identifier("preempt"), spec)
    result = {"config": "Preempt-recover: SIGTERM mid-task, %.0f GB checkpoint pack->host "
                        "DRAM->restore (1 x MI355X, iterative_task)" % args.gb,
              "codec": args.codec, "spill": spill, "prefetch": not args.no_prefetch,
              "early_prefetch": args.early_prefetch, "standby": args.standby,
              "hot_standby": args.hot, "preload": preload,
              "stream_handoff": not args.no_stream,
              "save_at": "signal" if args.signal_mode else "step boundary",
              "release_hbm": os.environ.get("TPI_RELEASE_HBM", "1") != "0",
              "step_seconds": args.step_seconds, "materialize": args.materialize,
              "extra_tensors_gib": [float(x) for x in args.extra_gib.split(",") if x.strip()]}
    os.environ["TPI_WARM_STANDBY"] = "hot" if args.hot else ("1" if args.standby else "0")
    # No drain of our own here: memory that earlier runs (or bench.py itself) gave back is
    # waited for by the product -- the task's start (placement.settle_gpus, "gpu-drain") and
    # the successor's allocation gate (preemption.wait_for_device_memory, "successor-hbm-wait")
    try:
        task.create()
        deadline = time.time() + args.timeout
        while time.time() < deadline and not any("ready" in l for l in task.logs()):
            if not task.supervisor_running():
                break
            time.sleep(0.2)
        if not any("ready" in l for l in task.logs()):
            raise SystemExit("rank never became ready: %s" % task.logs())
        if args.hot:
            # a hot standby maps and pins the whole spill once the rank has created it; a
            # preemption hours into training finds it pinned, so wait for that here too
            # (recorded as standby_pinned_s) instead of racing the pinning
            t_wait = time.time()
            while time.time() - t_wait < 300 and not any(
                    e.code == "standby-pinned" for e in task.events()):
                time.sleep(0.1)
            result["standby_pinned_wait_s"] = round(time.time() - t_wait, 3)
            result["standby_pinned"] = next((e.description for e in task.events()
                                             if e.code == "standby-pinned"), None)
        if preload:
            # the preloaded successor is spawned 2 s after the rank and then imports PyTorch;
            # a preemption hours into training finds it parked, so wait for that here too
            t_wait = time.time()
            while time.time() - t_wait < 120 and not any(
                    e.code == "standby-start" and "preloaded" in e.description
                    for e in task.events()):
                time.sleep(0.1)
            # its imports (it parks on its activation pipe after them) and -- by default, once
            # the supervisor has seen the rank use the GPU from one process -- its GPU context
            t_park = time.time()
            while time.time() - t_park < 20 and not any(
                    e.code == "preload-gpu-warmed" for e in task.events()):
                if any(e.code == "preload-plain" for e in task.events()):
                    break
                time.sleep(0.1)
            if not any(e.code == "preload-gpu-warmed" for e in task.events()):
                time.sleep(max(0.0, 3.0 - (time.time() - t_park)))
            result["preloaded_wait_s"] = round(time.time() - t_wait, 3)
            result["preload_gpu"] = next((e.description for e in task.events() if e.code in (
                "preload-gpu-warmed", "preload-plain")), None)
        t_preempt = time.time()
        task.preempt()
        status = task.wait(args.timeout)
        logs = task.logs()
        events = [(e.code, e.time.timestamp() if hasattr(e.time, "timestamp") else e.time,
                   e.description) for e in task.events()]
        result["status"] = status
        result["logs_tail"] = [l.strip().splitlines()[-1] for l in logs if l.strip()]

        def first(code, after=0.0):
            for c, t, d in events:
                if c == code and t >= after:
                    return t, d
            return None, None

        t_sig, _ = first("preempt-signal")
        t_saved, saved = first("checkpoint-saved")
        # with a streamed hand-off the successor starts before the spill has finished
        t_respawn, _ = first("respawn", t_sig or 0.0)
        result["streamed"] = first("checkpoint-streaming")[0] is not None
        result["early_handoff"] = first("rank-released")[0] is not None
        t_start2, _ = first("rank-start", t_respawn or 0.0)
        result["warm_standby_activated"] = first("standby-activated")[0] is not None
        t_restored, restored = first("checkpoint-restored", t_respawn or 0.0)
        if t_sig and t_saved:
            result["save_s"] = round(t_saved - t_sig, 3)
            result["save_journal"] = saved
        if t_saved and t_respawn:  # negative: respawned while the spill was still running
            result["saved_to_respawn_s"] = round(t_respawn - t_saved, 3)
        if t_start2 and t_restored:  # (with a warm standby: activation -> restored)
            result["rank_start_to_restored_s"] = round(t_restored - t_start2, 3)
            result["restore_journal"] = restored
        if t_restored:
            result["signal_to_restored_s"] = round(t_restored - (t_sig or t_preempt), 3)
            if t_saved:
                result["saved_to_restored_s"] = round(t_restored - t_saved, 3)
        if t_sig:  # every journal phase after the signal, seconds from it
            result["timeline"] = [[c, round(t - t_sig, 4), d] for c, t, d in events if t >= t_sig]
        t_durable, _ = first("checkpoint-durable", t_restored or 0.0)
        if t_durable and t_sig:  # host copy of the resumed state complete (HBM hand-off)
            result["signal_to_durable_s"] = round(t_durable - t_sig, 3)
        result["durability"] = next((c for c, _, _ in events if c in (
            "checkpoint-durable", "checkpoint-not-durable", "checkpoint-durability-unknown")), None)
        result["verified"] = any("verified True" in l for l in logs)
        # the host-memory guard the supervisor runs for the ranks (cgroup, or the 20 ms poll)
        result["memory_guard"] = next((d for c, _, d in events
                                       if c in ("memory-cgroup", "memory-guard")), None)
        t_settled, _ = first("supervisor-settled")
        t_exit, _ = first("rank-exit", t_respawn or 0.0)
        if t_settled and t_exit:  # the successor's exit -> final sync + final state
            result["rank_exit_to_settled_s"] = round(t_settled - t_exit, 3)
        result["released_exit_pending_at_settle"] = first("rank-released-exit")[0] is None
        # the product's own memory gates (no bench-side drain): the task's start on a GPU
        # whose memory was still coming back, and each successor's allocation gate
        result["gpu_drain"] = [d for c, _, d in events if c == "gpu-drain"]
        result["successor_hbm_wait"] = [d for c, _, d in events if c == "successor-hbm-wait"]
        result["hbm_failed"] = [d for c, _, d in events
                                if c in ("checkpoint-hbm-failed", "checkpoint-hbm-fatal")]
        # a failed hand-off copy leaves its descriptors next to the spill (handoff.py
        # _dump_copy_plan): keep them with the result, the spill directory is removed below
        import glob

        dumps = []
        for path in glob.glob(spill + ".hbm.fault.*.json"):
            try:
                with open(path) as f:
                    dumps.append(json.load(f))
            except (OSError, ValueError):
                pass
        if dumps:
            result["hbm_fault_dumps"] = dumps
        result["hbm_skipped"] = [d for c, _, d in events if c == "checkpoint-hbm-skipped"]
        result["ok"] = bool(status.get("succeeded") == 1 and result["verified"])
        if result["hbm_failed"] or not result["ok"]:  # the whole journal, for the record
            result["timeline_on_failure"] = result.get("timeline")
    finally:
        try:
            # the task is over for its users once the supervisor settled; a released
            # predecessor may still be tearing down its pinned region:
            # delete must not wait for it
            t_del = time.time()
            task.delete()
            result["delete_s"] = round(time.time() - t_del, 3)
        finally:
            shutil.rmtree(state, ignore_errors=True)
            if os.path.exists(spill):
                os.remove(spill)
    print(json.dumps(result))


if __name__ == "__main__":
    main()
