#!/usr/bin/env python3
"""Where does the teardown of a pinned host region go?  (round 4)

In the hot-standby preemption flow a predecessor's explicit close of its 100 GB region took
~11 s (``predecessor-teardown``, profiles/round4/preempt_hot_100g_r4c_*.json); a reclaimed
victim's took 1.37 s (profiles/round4/reclaim_100g_r4a.json).  The difference between the two:
in the hot flow other processes (the successor, its new hot standby) map and pin the same
/dev/shm pages.  This isolates that on one box, each scenario on a fresh shm file:

  alone         the owner (mapped + populated + hipHostRegister'ed, as a Checkpointer region)
                closes it: unregister, unmap
  pinned-twice  a second process maps and pins the same file window by window (prefetch());
                the owner closes, then the second process closes
  mapped-twice  the second process only maps (populated, not pinned); the owner closes
  exit-pinned   as pinned-twice, but the owner just exits (the kernel's teardown, timed to
                the parent's waitpid)

Prints one JSON line.  ``--gb`` (default 64) per region.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CHILD = r'''
import json, os, sys, time
sys.path.insert(0, %(root)r)
import torch
torch.cuda.init()
torch.empty(1, device="cuda")
from terraform_provider_iterative_amd.checkpoint.host import HostRegion
from terraform_provider_iterative_amd.ops import hip
role, path, size = sys.argv[1], sys.argv[2], int(sys.argv[3])
t0 = time.perf_counter()
if role == "owner":
    region = HostRegion(size, path, device=True, numa_node=-1, populate=True)
elif role == "pinner":
    region = HostRegion(size, path, device=True, numa_node=-1, progressive=True)
    hip().check(hip().tpi_host_pin_wait(region.pinner), "pin wait")
else:  # mapper: populated, never registered
    import mmap
    fd = os.open(path, os.O_RDWR)
    region = mmap.mmap(fd, size, mmap.MAP_SHARED | getattr(mmap, "MAP_POPULATE", 0))
    os.close(fd)
setup = time.perf_counter() - t0
print(json.dumps({"ready": True, "setup_s": round(setup, 3)}), flush=True)
cmd = sys.stdin.readline().strip()
if cmd == "exit":
    os._exit(0)
t0 = time.perf_counter()
timings = {}
if role == "mapper":
    region.close()
else:
    region.close(timings)
print(json.dumps({"close_s": round(time.perf_counter() - t0, 3),
                  **{k: round(v, 3) for k, v in timings.items()}}), flush=True)
'''


def start(role, path, size):
    proc = subprocess.Popen([sys.executable, "-c", CHILD % {"root": ROOT}, role, path, str(size)],
                            stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    ready = json.loads(proc.stdout.readline())
    return proc, ready


def finish(proc, cmd="close"):
    t0 = time.perf_counter()
    proc.stdin.write(cmd + "\n")
    proc.stdin.flush()
    out = {}
    if cmd == "close":
        out = json.loads(proc.stdout.readline())
    proc.wait(600)
    out["reaped_s"] = round(time.perf_counter() - t0, 3)
    return out


def main():
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--gb", type=float, default=64.0)
    p.add_argument("--dir", default="/dev/shm")
    p.add_argument("--only", nargs="*", default=None)
    args = p.parse_args()
    size = int(args.gb * 1e9) // 4096 * 4096
    result = {"gb": args.gb}
    for scenario in ("alone", "pinned-twice", "mapped-twice", "exit-pinned"):
        if args.only and scenario not in args.only:
            continue
        path = os.path.join(args.dir, "tpi-teardown-%d-%s" % (os.getpid(), scenario))
        with open(path, "wb") as f:
            f.truncate(size)
        try:
            owner, ready = start("owner", path, size)
            entry = {"owner_setup_s": ready["setup_s"]}
            other = None
            if scenario in ("pinned-twice", "exit-pinned"):
                other, ready2 = start("pinner", path, size)
                entry["pinner_setup_s"] = ready2["setup_s"]
            elif scenario == "mapped-twice":
                other, ready2 = start("mapper", path, size)
                entry["mapper_setup_s"] = ready2["setup_s"]
            entry["owner"] = finish(owner, "exit" if scenario == "exit-pinned" else "close")
            if other is not None:
                entry["other"] = finish(other)
            result[scenario] = entry
            print("teardown %s: %s" % (scenario, json.dumps(entry)), file=sys.stderr, flush=True)
        finally:
            os.remove(path)
    print(json.dumps(result))


if __name__ == "__main__":
    main()
