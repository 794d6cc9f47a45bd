#!/usr/bin/env python3
"""HBM-to-HBM preemption hand-off alone (config 4's same-GPU path), per copy route.

A child process (the "preempted rank") holds ``--gb`` of AdamW-like state (bf16 params, fp32
moments; contiguous tensors) and exports HIP IPC handles of it (``Checkpointer.export_hbm``);
this process (the "successor") binds tensors of the same shapes and restores them device to
device (``Checkpointer.restore_hbm``), once per route and ``--repeats`` times:

  fused   MODE_COPY tensor -> tensor + tile CRCs, then MODE_VERIFY read-back (default route)
  staged  pack into the engine's staging buffer, unpack + verify (TPI_HANDOFF_COPY=staged)

Prints one JSON line: seconds and GB/s per route (median), every restore verified bit-exact.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CHILD = r'''
import sys, torch
sys.path.insert(0, %(root)r)
from terraform_provider_iterative_amd.checkpoint import Checkpointer
sys.path.insert(0, %(bench)r)
from bench_handoff import make_state
t = make_state(%(gb)r, seed=5)
ck = Checkpointer(t, path=%(path)r)
for line in sys.stdin:
    if line.strip() != "export":
        break
    print("exported", ck.export_hbm(), flush=True)
'''


def make_state(gb: float, seed: int, fill: bool = True):
    """Three tensor kinds per layer, ~1 GB per tensor, like bench.py's synthetic state."""
    import torch

    g = torch.Generator(device="cuda").manual_seed(seed)
    total, out, layer = int(gb * 1e9), {}, 0
    per = 1 << 28  # elements per fp32 tensor (1 GiB)
    while total > 0:
        for kind, dtype in (("param", torch.bfloat16), ("exp_avg", torch.float32),
                            ("exp_avg_sq", torch.float32)):
            n = min(per, max(total // (2 if dtype == torch.bfloat16 else 4), 1))
            if fill:
                t = torch.randn(n, device="cuda", generator=g).to(dtype)
            else:
                t = torch.zeros(n, device="cuda", dtype=dtype)
            out["l%d.%s" % (layer, kind)] = t
            total -= t.numel() * t.element_size()
            if total <= 0:
                break
        layer += 1
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--gb", type=float, default=16.0)
    p.add_argument("--repeats", type=int, default=3)
    p.add_argument("--routes", default="fused,staged")
    args = p.parse_args()
    import torch

    from terraform_provider_iterative_amd.checkpoint import Checkpointer

    tmp = tempfile.mkdtemp(prefix="tpi-handoff-")
    path = os.path.join(tmp, "spill")
    child = subprocess.Popen(
        [sys.executable, "-c", CHILD % {"root": ROOT, "bench": os.path.dirname(__file__),
                                         "gb": args.gb, "path": path}],
        stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    out = {"bytes": 0, "routes": {}}
    try:
        want = make_state(args.gb, seed=5)
        dst = make_state(args.gb, seed=0, fill=False)
        out["bytes"] = sum(t.numel() * t.element_size() for t in dst.values())
        ck = Checkpointer(dst, path=path)
        for route in args.routes.split(","):
            if route == "staged":
                os.environ["TPI_HANDOFF_COPY"] = "staged"
            else:
                os.environ.pop("TPI_HANDOFF_COPY", None)
            times = []
            for _ in range(args.repeats):
                for t in dst.values():
                    t.zero_()
                child.stdin.write("export\n")
                child.stdin.flush()
                line = child.stdout.readline()
                assert line.startswith("exported"), line
                torch.cuda.synchronize()
                res = ck.restore_hbm()
                torch.cuda.synchronize()
                assert res.bad_tiles == 0
                assert all(torch.equal(dst[k], want[k]) for k in want), "restore differs"
                times.append(res.seconds)
                print("handoff %s %.4f s" % (route, res.seconds), file=sys.stderr, flush=True)
            med = sorted(times)[len(times) // 2]
            out["routes"][route] = {"s": round(med, 4), "GBps": round(out["bytes"] / med / 1e9, 1),
                                    "all_s": [round(x, 4) for x in times], "verified": True}
        ck.close()
    finally:
        try:
            child.stdin.write("quit\n")
            child.stdin.flush()
        except OSError:
            pass
        child.wait(60)
        import shutil

        shutil.rmtree(tmp, ignore_errors=True)  # the spill region file is state-sized
    print(json.dumps(out))


if __name__ == "__main__":
    main()
