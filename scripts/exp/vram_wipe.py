"""Experiment: is HBM freed by one process cleared in the background (allocation fast once the
wipe is done) or when the next process allocates it?

A child allocates and touches GB of HBM and exits; after `delay` seconds a second child times
its own allocation of the same size.  The big-state preemption path (a rank over half of
HBM frees its memory after the boundary save, profiles/preempt_e2e_170g_round3.md) spends
~5 s of its 10 s signal -> restored in the successor's allocation.

    python scripts/exp/vram_wipe.py [GB] [delay ...]
    python scripts/exp/vram_wipe.py [GB] alive      # the first process frees but stays alive
    python scripts/exp/vram_wipe.py [GB] many       # the state as ~400 tensors, cold vs one
                                                    # block reserved first
"""
import json
import subprocess
import sys
import time

CHILD = r'''
import sys, time, torch
gb, mode = float(sys.argv[1]), sys.argv[2]
torch.cuda.init()
torch.empty(1, device="cuda")  # HIP context up before the clock starts
torch.cuda.synchronize()
t = time.perf_counter()
x = torch.empty(int(gb * 1e9), dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
alloc = time.perf_counter() - t
if mode == "fill":
    x.fill_(1)
    torch.cuda.synchronize()
print(alloc, flush=True)
'''


def child(gb, mode):
    out = subprocess.run([sys.executable, "-c", CHILD, str(gb), mode], capture_output=True,
                         text=True, timeout=300)
    if out.returncode != 0:
        raise RuntimeError(out.stderr[-2000:])
    return float(out.stdout.strip().splitlines()[-1])


HOLDER = r'''
import sys, time, torch
gb = float(sys.argv[1])
x = torch.empty(int(gb * 1e9), dtype=torch.uint8, device="cuda")
x.fill_(1)
torch.cuda.synchronize()
del x
torch.cuda.empty_cache()  # hipFree: given back while this process lives on
torch.cuda.synchronize()
print("freed", flush=True)
sys.stdin.readline()
'''


def alive(gb):
    """The predecessor-release path: free with the process still alive, then allocate."""
    holder = subprocess.Popen([sys.executable, "-c", HOLDER, str(gb)], stdin=subprocess.PIPE,
                              stdout=subprocess.PIPE, text=True)
    assert holder.stdout.readline().strip() == "freed"
    out = {"alloc_while_releaser_alive_s": child(gb, "none")}
    t = time.perf_counter()
    out["alloc_and_touch_while_releaser_alive_s"] = child(gb, "fill")
    holder.stdin.write("\n")
    holder.stdin.flush()
    holder.wait(120)
    return out


MANY = r'''
import sys, time, torch
sys.path.insert(0, ".")
from bench import synthetic_checkpoint
gb, warm = float(sys.argv[1]), sys.argv[2] == "warm"
torch.empty(1, device="cuda")
torch.cuda.synchronize()
t = time.perf_counter()
if warm:  # one block of the state's size into the caching allocator, given back at once
    block = torch.empty(int(gb * 1e9) + (1 << 30), dtype=torch.uint8, device="cuda")
    del block
t1 = time.perf_counter()
state = synthetic_checkpoint(int(gb * 1e9), 8192, torch.device("cuda"), fill=False)
torch.cuda.synchronize()
print(t1 - t, time.perf_counter() - t1, len(state), flush=True)
'''


def many(gb):
    """The successor's state as the training script allocates it (hundreds of tensors) right
    after a releaser freed the memory: cold caching allocator vs one block reserved first."""
    out = {}
    for mode in ("cold", "warm"):
        holder = subprocess.Popen([sys.executable, "-c", HOLDER, str(gb)], stdin=subprocess.PIPE,
                                  stdout=subprocess.PIPE, text=True)
        assert holder.stdout.readline().strip() == "freed"
        r = subprocess.run([sys.executable, "-c", MANY, str(gb), mode], capture_output=True,
                           text=True, timeout=300)
        holder.stdin.write("\n")
        holder.stdin.flush()
        holder.wait(120)
        if r.returncode != 0:
            raise RuntimeError(r.stderr[-2000:])
        reserve, alloc, n = r.stdout.split()
        out[mode] = {"reserve_s": float(reserve), "tensors_s": float(alloc), "tensors": int(n)}
    return out


def main():
    gb = float(sys.argv[1]) if len(sys.argv) > 1 else 100.0
    if sys.argv[2:3] == ["many"]:
        print(json.dumps(dict(many(gb), GB=gb)), flush=True)
        return
    if sys.argv[2:3] == ["alive"]:
        print(json.dumps(dict(alive(gb), GB=gb)), flush=True)
        return
    delays = [float(d) for d in sys.argv[2:]] or [0.0, 5.0]
    res = {"GB": gb, "fresh_alloc_s": child(gb, "fill")}
    for d in delays:
        t = time.perf_counter()
        child(gb, "fill")  # allocate + touch, then exit (frees)
        exit_s = time.perf_counter() - t
        time.sleep(d)
        res["after_free_delay_%gs_alloc_s" % d] = child(gb, "none")
        res["first_child_s_%g" % d] = round(exit_s, 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
