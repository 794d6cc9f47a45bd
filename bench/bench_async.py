#!/usr/bin/env python3
"""Asynchronous checkpoint: training-stream stall vs. blocking save (1 GPU).

``save_async`` packs the state into an HBM snapshot on the current stream (the only part
the training stream waits for) and spills it to host DRAM in the background.  Reports the
stall (device time until the current stream is free again), the background spill time, and
a blocking ``save`` of the same state for comparison, and ``rollback`` (restore from the
HBM snapshot, device to device, CRC-verified).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--gb", type=float, default=32.0)
    p.add_argument("--codec", default="tpz1")
    args = p.parse_args()
    import torch

    from bench import synthetic_checkpoint
    from terraform_provider_iterative_amd.checkpoint import Checkpointer

    dev = torch.device("cuda", 0)
    tensors = synthetic_checkpoint(int(args.gb * 1e9), 8192, dev)
    torch.cuda.synchronize()
    out = {"GB": args.gb, "codec": args.codec}
    with Checkpointer(tensors, codec=args.codec) as ck:
        ck.save_async().result()  # warm-up (allocates the snapshot)
        stream = torch.cuda.current_stream(dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pending = ck.save_async({"bench": True})
        stream.synchronize()  # the training stream is free from here on
        t1 = time.perf_counter()
        res = pending.result()
        t2 = time.perf_counter()
        out["stall_ms"] = round((t1 - t0) * 1e3, 2)
        out["snapshot_GBps"] = round(ck.plan.total / (t1 - t0) / 1e9, 1)
        out["spill_s"] = round(t2 - t0, 3)
        out["spill_GBps"] = round(ck.plan.total / (t2 - t0) / 1e9, 2)
        out["wire_bytes"] = res.wire_bytes
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        rb = ck.rollback()
        out["rollback_ms"] = round((time.perf_counter() - t3) * 1e3, 2)
        out["rollback_GBps"] = round(ck.plan.total / (time.perf_counter() - t3) / 1e9, 1)
        out["rollback_verified"] = rb.bad_tiles == 0
        t3 = time.perf_counter()
        ck.save()
        out["blocking_save_s"] = round(time.perf_counter() - t3, 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
