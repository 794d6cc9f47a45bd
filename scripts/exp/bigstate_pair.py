#!/usr/bin/env python3
"""A big-state hand-off without the supervisor, so a profiler sees both processes (round 4).

A predecessor holds ``--gb`` of synthetic AdamW state (more than half of HBM) and saves it
into a /dev/shm region with a streamed save that frees each tensor's HBM behind the spill
(``save(release_behind=True)``).  Its successor -- already running, engine prewarmed and the
region prefetched, as a hot standby is -- is told to go when the stream starts and either
materializes the state group by group (``--mode materialize``) or waits for room, allocates
the whole state and restores behind the spill (``--mode upfront``).  Both print timestamped
phases on stderr; the parent prints one JSON line.

Meant to run under ``rocprofv3 --kernel-trace --memory-copy-trace`` to see what the
successor's copies and kernels wait for in the ~2 s stall of profiles/round4/materialize_170g.md.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PRED = r'''
import json, os, sys, time
sys.path.insert(0, %(root)r)
import torch
from bench import synthetic_checkpoint
from terraform_provider_iterative_amd.checkpoint import Checkpointer
T0 = float(sys.argv[2])
def say(msg):
    print("[%%.3f] predecessor: %%s" %% (time.time() - T0, msg), file=sys.stderr, flush=True)
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
tensors = synthetic_checkpoint(int(float(sys.argv[1]) * 1e9), 8192, dev)
torch.cuda.synchronize()
ck = Checkpointer(tensors, path=%(spill)r, codec="tpz1")
say("ready, %%.1f GB free" %% (torch.cuda.mem_get_info(0)[0] / 1e9))
print("ready", flush=True)
sys.stdin.readline()
t = time.time()
def started():
    say("stream started")
    print("stream", flush=True)
res = ck.save({"step": 1}, on_stream=started, release_behind=True)
say("saved in %%.3f s, released %%.1f GB" %% (time.time() - t, res.released_bytes / 1e9))
print(json.dumps({"save_s": round(time.time() - t, 3), "released_GB": res.released_bytes / 1e9}),
      flush=True)
sys.stdin.readline()
'''

SUCC = r'''
import json, os, sys, time
sys.path.insert(0, %(root)r)
import torch
from terraform_provider_iterative_amd.checkpoint import Checkpointer, prewarm_engine
from terraform_provider_iterative_amd.checkpoint.host import prefetch
T0 = float(sys.argv[2])
mode = sys.argv[3]
def say(msg):
    print("[%%.3f] successor: %%s" %% (time.time() - T0, msg), file=sys.stderr, flush=True)
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
torch.empty(1, device=dev)
prewarm_engine(0)
prefetch(%(spill)r)
if "--racing" not in sys.argv:  # a hot standby has long pinned the spill when a preemption comes
    from terraform_provider_iterative_amd.checkpoint.host import wait_pinned
    say("pinned in %%.3f s" %% wait_pinned(%(spill)r))
say("standing by")
print("ready", flush=True)
sys.stdin.readline()
t = time.time()
say("go")
out = {}
if mode == "materialize":
    ck, tensors, res = Checkpointer.materialize(%(spill)r, dev)
    out["stats"] = {k: v for k, v in ck.materialize_stats.items() if k != "trace"}
    out["trace"] = ck.materialize_stats["trace"]
else:
    from bench import synthetic_checkpoint
    need = int(float(sys.argv[1]) * 1e9 * 1.05) + (2 << 30)
    while torch.cuda.mem_get_info(0)[0] < need:
        time.sleep(0.005)
    out["wait_s"] = round(time.time() - t, 3)
    say("room")
    tensors = synthetic_checkpoint(int(float(sys.argv[1]) * 1e9), 8192, dev, fill=False)
    torch.cuda.synchronize()
    out["alloc_s"] = round(time.time() - t - out["wait_s"], 3)
    say("allocated")
    ck = Checkpointer(tensors, path=%(spill)r, codec="tpz1")
    res = ck.restore(stream_timeout=60)
torch.cuda.synchronize()
out["restored_s"] = round(time.time() - t, 3)
out["bad_tiles"] = res.bad_tiles
say("restored in %%.3f s" %% out["restored_s"])
print(json.dumps(out), flush=True)
ck.close()
'''


def main():
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--gb", type=float, default=170.0)
    p.add_argument("--mode", choices=("materialize", "upfront"), default="materialize")
    p.add_argument("--spill", default="/dev/shm/tpi-bigstate-pair-%d.spill" % os.getpid())
    p.add_argument("--successor-env", action="append", default=[], metavar="KEY=VALUE",
                   help="environment of the successor only (e.g. HSA_ENABLE_SDMA=0)")
    p.add_argument("--racing", action="store_true",
                   help="the successor starts restoring while it is still pinning the spill")
    args = p.parse_args()
    t0 = time.time()
    sub = {"root": ROOT, "spill": args.spill}
    env = dict(os.environ)
    pred = subprocess.Popen([sys.executable, "-c", PRED % sub, str(args.gb), str(t0)],
                            stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, env=env)
    succ = None
    try:
        assert pred.stdout.readline().strip() == "ready"
        succ_env = dict(env, **dict(kv.split("=", 1) for kv in args.successor_env))
        succ = subprocess.Popen([sys.executable, "-c", SUCC % sub, str(args.gb), str(t0),
                                 args.mode] + (["--racing"] if args.racing else []),
                                stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True,
                                env=succ_env)
        assert succ.stdout.readline().strip() == "ready"
        t_sig = time.time()
        pred.stdin.write("\n")
        pred.stdin.flush()
        assert pred.stdout.readline().strip() == "stream"
        succ.stdin.write("\n")
        succ.stdin.flush()
        saved = json.loads(pred.stdout.readline())
        restored = json.loads(succ.stdout.readline())
        t_end = time.time()
        succ.wait(120)
        pred.stdin.write("\n")
        pred.stdin.flush()
        pred.wait(120)
        print(json.dumps({"gb": args.gb, "mode": args.mode, "signal_to_restored_s":
                          round(t_end - t_sig, 3), "predecessor": saved, "successor": restored}))
    finally:
        for proc in (pred, succ):
            if proc is not None and proc.poll() is None:
                proc.kill()
                proc.wait(60)
        if os.path.exists(args.spill):
            os.remove(args.spill)


if __name__ == "__main__":
    main()
