#!/usr/bin/env python3
"""Do the driver's clears of freshly allocated HBM stall another process's host-to-device
copies?  (round 4, profiles/round4/materialize_170g.md)

A "copier" process streams pinned host memory to the device (hipMemcpyAsync H2D, 256 MB
pieces) and, in a second phase, device to host, printing the GB/s of every 100 ms window.
Meanwhile a "filler" process holds ``--gb`` of HBM it has written; it frees it, and at that
moment an "allocator" process allocates the same amount in ``--piece-gb`` tensors, timing each
allocation (a preempted rank and its successor on one GPU).  If the H2D rate
collapses while the allocator runs and D2H does not, the clears and HIP's H2D copies share an
engine.  Prints one JSON line.
"""
import argparse
import json
import subprocess
import sys
import time

COPIER = r'''
import json, sys, time, torch
direction, seconds = sys.argv[1], float(sys.argv[2])
dev = torch.device("cuda", 0)
piece = 256 << 20
host = torch.empty(8 * piece, dtype=torch.uint8).pin_memory()
devbuf = torch.empty(8 * piece, dtype=torch.uint8, device=dev)
s = torch.cuda.Stream()
print(json.dumps({"ready": True}), flush=True)
t0 = time.perf_counter()
windows, moved, wstart = [], 0, t0
i = 0
with torch.cuda.stream(s):
    while time.perf_counter() - t0 < seconds:
        k = i % 8
        if direction == "h2d":
            devbuf[k * piece:(k + 1) * piece].copy_(host[k * piece:(k + 1) * piece], non_blocking=True)
        else:
            host[k * piece:(k + 1) * piece].copy_(devbuf[k * piece:(k + 1) * piece], non_blocking=True)
        i += 1
        if i % 4 == 0:
            s.synchronize()
            moved += 4 * piece
            now = time.perf_counter()
            if now - wstart >= 0.1:
                windows.append([round(wstart - t0, 3), round(moved / (now - wstart) / 1e9, 1)])
                moved, wstart = 0, now
print(json.dumps({"windows": windows, "t0": t0}), flush=True)
'''

FILLER = r'''
import json, sys, time, torch
gb = float(sys.argv[1])
dev = torch.device("cuda", 0)
held = torch.empty(int(gb * 1e9), dtype=torch.uint8, device=dev)
held.fill_(7)
torch.cuda.synchronize()
print(json.dumps({"filled": True}), flush=True)
sys.stdin.readline()
t = time.perf_counter()
del held
torch.cuda.empty_cache()
torch.cuda.synchronize()
print(json.dumps({"freed_s": round(time.perf_counter() - t, 4), "t_free": t}), flush=True)
sys.stdin.readline()
'''

ALLOCATOR = r'''
import json, sys, time, torch
gb, piece_gb = float(sys.argv[1]), float(sys.argv[2])
dev = torch.device("cuda", 0)
torch.empty(1, device=dev)
print(json.dumps({"ready": True}), flush=True)
sys.stdin.readline()
out = []
held = []
for j in range(int(gb / piece_gb)):
    t = time.perf_counter()
    held.append(torch.empty(int(piece_gb * 1e9), dtype=torch.uint8, device=dev))
    torch.cuda.synchronize()
    out.append([j, t, round(time.perf_counter() - t, 4)])
print(json.dumps({"allocs": out}), flush=True)
'''



def run(direction, args):
    """Copier running; a filler process holds ``--gb`` of written HBM and frees it; at that
    moment a second process allocates the same amount (a preempted rank and its successor)."""
    py = sys.executable
    copier = subprocess.Popen([py, "-c", COPIER, direction, str(args.seconds)],
                              stdout=subprocess.PIPE, text=True)
    assert json.loads(copier.stdout.readline())["ready"]
    filler = subprocess.Popen([py, "-c", FILLER, str(args.gb)], stdin=subprocess.PIPE,
                              stdout=subprocess.PIPE, text=True)
    assert json.loads(filler.stdout.readline())["filled"]
    alloc = subprocess.Popen([py, "-c", ALLOCATOR, str(args.gb), str(args.piece_gb)],
                             stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    assert json.loads(alloc.stdout.readline())["ready"]
    time.sleep(1.0)
    filler.stdin.write("\n")
    filler.stdin.flush()
    freed = json.loads(filler.stdout.readline())
    alloc.stdin.write("\n")
    alloc.stdin.flush()
    a_out = json.loads(alloc.stdout.readline())
    alloc.wait(60)
    filler.stdin.write("\n")
    filler.stdin.flush()
    filler.wait(60)
    c_out = json.loads(copier.stdout.readline())
    copier.wait(120)
    base = c_out["t0"]  # perf_counter is CLOCK_MONOTONIC: one clock for all processes
    allocs = [[j, round(t - base, 3), d] for j, t, d in a_out["allocs"]]
    busy = (allocs[0][1], allocs[-1][1] + allocs[-1][2])
    inside = [g for t, g in c_out["windows"] if busy[0] <= t <= busy[1]]
    outside = [g for t, g in c_out["windows"] if t < freed["t_free"] - base - 0.2]
    return {"direction": direction, "free_at_s": round(freed["t_free"] - base, 3),
            "free_s": freed["freed_s"], "alloc_window_s": [round(busy[0], 3), round(busy[1], 3)],
            "gbps_before": round(sum(outside) / max(len(outside), 1), 1),
            "gbps_during_allocs": round(sum(inside) / max(len(inside), 1), 1),
            "alloc_s_total": round(sum(d for _, _, d in allocs), 3),
            "allocs": allocs, "windows": c_out["windows"]}


def main():
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--gb", type=float, default=100.0)
    p.add_argument("--piece-gb", type=float, default=4.0)
    p.add_argument("--seconds", type=float, default=20.0)
    args = p.parse_args()
    result = {"gb": args.gb, "piece_gb": args.piece_gb}
    for direction in ("h2d", "d2h"):
        result[direction] = run(direction, args)
        print("%s: %.1f GB/s before, %.1f GB/s during %.2f s of allocations"
              % (direction, result[direction]["gbps_before"],
                 result[direction]["gbps_during_allocs"], result[direction]["alloc_s_total"]),
              file=sys.stderr, flush=True)
    print(json.dumps(result))


if __name__ == "__main__":
    main()
