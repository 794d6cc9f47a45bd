#!/usr/bin/env python3
"""Pack/unpack throughput of non-contiguous tensor views (GB/s of payload):
transposed 2-D (fp32 / bf16), row-sliced 2-D, channels-last 4-D activations and conv weights
(small C = kh*kw), every-other-element.  Each view is >= 150 MB so the pack kernel has a
full grid (one workgroup per 1 MiB tile), as inside a checkpoint chunk."""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from terraform_provider_iterative_amd.ops.packing import PackPlan, pack, unpack

    dev = torch.device("cuda", 0)
    cases = {
        "transpose_fp32": torch.randn(8192, 8192, device=dev).t(),
        "transpose_bf16": torch.randn(16384, 8192, device=dev).to(torch.bfloat16).t(),
        "row_slice_fp32": torch.randn(8192, 8192, device=dev)[:, 100:8000],
        "channels_last_bf16": torch.randn(256, 256, 32, 32, device=dev).to(torch.bfloat16)
        .contiguous(memory_format=torch.channels_last),
        "conv_weight_cl_bf16": torch.randn(16384, 512, 3, 3, device=dev).to(torch.bfloat16)
        .contiguous(memory_format=torch.channels_last),
        "stride2_fp32": torch.randn(1 << 27, device=dev)[::2],
    }
    out = {}
    for name, t in list(cases.items()):
        plan = PackPlan.from_tensors({name: t})
        stream, crcs = pack(plan)
        torch.cuda.synchronize()
        iters = 3
        t0 = time.perf_counter()
        for _ in range(iters):
            pack(plan, stream)
        torch.cuda.synchronize()
        tp = (time.perf_counter() - t0) / iters
        t0 = time.perf_counter()
        for _ in range(iters):
            bad, _ = unpack(plan, stream, crcs)
        torch.cuda.synchronize()
        tu = (time.perf_counter() - t0) / iters
        nbytes = t.numel() * t.element_size()
        out[name] = {"pack_GBps": round(nbytes / tp / 1e9, 1),
                     "unpack_GBps": round(nbytes / tu / 1e9, 1), "bad": int(bad),
                     "MB": round(nbytes / 1e6)}
        del cases[name], plan, stream, crcs, t
        torch.cuda.empty_cache()
    out["many_small"] = many_small()
    print(json.dumps(out))



def many_small(n=20000):
    """Checkpoint of many small tensors (norm weights / biases): descriptor walking cost."""
    import torch

    from terraform_provider_iterative_amd.checkpoint import Checkpointer

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    tensors = {"p%d" % i: torch.randn(1000 + (i % 7) * 13, device=dev, generator=g)
               for i in range(n)}
    nbytes = sum(t.numel() * 4 for t in tensors.values())
    out = {}
    with Checkpointer(tensors, codec="none") as ck:
        ck.save()
        ck.restore()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            ck.save()
        t1 = time.perf_counter()
        for _ in range(3):
            ck.restore()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
    out["tensors"] = n
    out["MB"] = round(nbytes / 1e6)
    out["save_GBps"] = round(3 * nbytes / (t1 - t0) / 1e9, 1)
    out["restore_GBps"] = round(3 * nbytes / (t2 - t1) / 1e9, 1)
    return out


if __name__ == "__main__":
    main()
