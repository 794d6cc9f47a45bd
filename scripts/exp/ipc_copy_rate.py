#!/usr/bin/env python3
"""Is the hand-off copy slower when its source is another process's HBM (HIP IPC mapping)?

The hot hand-off's copy + read-back of 100 GB takes 57-58 ms of kernel time
(profiles/round5/r5k, r5m) where the same kernels take 49.7 ms between two tensor sets of
one process (handoff_kernels.md).  A first-copy cost per process was ruled out (r5l / r5m:
the prewarm absorbs it).  Here a sibling exports ``GB`` of state (``export_hbm``); this
process restores it with ``restore_hbm`` but runs the copy four times on the IPC-mapped
source, then copies four times between two local tensor sets of the same layout.  One JSON
line per copy.

    python scripts/exp/ipc_copy_rate.py [GB]
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

EXPORTER = r'''
import sys, torch
sys.path.insert(0, %(root)r)
from bench import synthetic_checkpoint
from terraform_provider_iterative_amd.checkpoint import Checkpointer
t = synthetic_checkpoint(%(nbytes)d, 8192, torch.device("cuda", 0))
torch.cuda.synchronize()
ck = Checkpointer(t, path=%(path)r, codec="tpz1")
print("exported", ck.export_hbm(), flush=True)
if sys.stdin.readline().strip() == "save":  # spill to host while the successor copies
    import time
    t0 = time.perf_counter()
    res = ck.save({"step": 1})
    print("saved %%.3f s" %% (time.perf_counter() - t0), flush=True)
    sys.stdin.readline()
'''


def main():
    gb = float(sys.argv[1]) if len(sys.argv) > 1 else 50.0
    nbytes = int(gb * 1e9)
    path = "/dev/shm/tpi-ipc-rate-%d.spill" % os.getpid()
    child = subprocess.Popen([sys.executable, "-c", EXPORTER % {"root": ROOT, "nbytes": nbytes,
                                                                "path": path}],
                             stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    import torch

    from bench import synthetic_checkpoint
    from terraform_provider_iterative_amd.checkpoint import Checkpointer
    from terraform_provider_iterative_amd.ops.packing import PackPlan

    try:
        line = child.stdout.readline()
        assert line.startswith("exported"), line
        dev = torch.device("cuda", 0)
        dst = synthetic_checkpoint(nbytes, 8192, dev, fill=False)
        torch.cuda.synchronize()
        ck = Checkpointer(dst, path=path, populate=False)
        stream = torch.cuda.current_stream().cuda_stream
        ck.engine.copy_segments(ck.plan.segs.copy(), ck.plan, stream)  # first copy of the process
        orig = ck.engine.copy_segments

        saving = bool(os.environ.get("IPC_RATE_SAVE"))

        def repeated(src, plan, sig, dst_segs=None):
            res = None
            for i in range(4):
                t = time.perf_counter()
                res = orig(src, plan, sig, dst_segs)
                print(json.dumps({"case": "ipc source %d" % i, "gb": gb, "concurrent_save": saving,
                                  "wall_s": round(time.perf_counter() - t, 4),
                                  "kernels_s": round(res.device_seconds, 4),
                                  "bad_tiles": res.bad_tiles}), flush=True)
            return res

        ck.engine.copy_segments = repeated
        assert ck.hbm_ready(), "no hand-off"
        saving = bool(os.environ.get("IPC_RATE_SAVE"))
        if saving:  # the predecessor's save shares the GPU, as in a hot hand-off
            child.stdin.write("save\n")
            child.stdin.flush()
            time.sleep(0.05)
        ck.restore_hbm()
        print(json.dumps({"case": "ipc open", "threads": os.environ.get("TPI_IPC_OPEN_THREADS", "8"),
                          "allocations": len(getattr(ck, "_last_bases", []) or []),
                          "open_s": round(ck.hbm_open_s, 4),
                          "steps": {k: round(v, 4) for k, v in ck.hbm_phases.items()}}),
              flush=True)
        ck.engine.copy_segments = orig
        ck.wait_hbm_close()
        if saving:
            print(json.dumps({"case": "predecessor", "save": child.stdout.readline().strip()}),
                  flush=True)
        child.stdin.write("\n")
        child.stdin.flush()
        child.wait(60)
        src = synthetic_checkpoint(nbytes, 8192, dev)
        torch.cuda.synchronize()
        src_segs = PackPlan.from_tensors(src, ck.plan.tile_bytes).segs.copy()
        for i in range(4):
            t = time.perf_counter()
            res = ck.engine.copy_segments(src_segs, ck.plan, stream)
            print(json.dumps({"case": "local source %d" % i, "gb": gb,
                              "wall_s": round(time.perf_counter() - t, 4),
                              "kernels_s": round(res.device_seconds, 4),
                              "bad_tiles": res.bad_tiles}), flush=True)
        ck.close()
    finally:
        if child.poll() is None:
            child.kill()
            child.wait()
        for suffix in ("", ".hbm", ".hbm.claim"):
            try:
                os.remove(path + suffix)
            except OSError:
                pass


if __name__ == "__main__":
    main()
