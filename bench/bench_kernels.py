#!/usr/bin/env python3
"""Device-side throughput of the data-plane kernels (HBM-bound reference: a torch copy).

Reports GB/s of payload processed per kernel (pack/unpack move 2x that over HBM):
  crc32c_tiles   read-only CRC32C per 1 MiB tile
  shard_hash     read-only striped XXH64 per 1 MiB shard
  pack_device    gather tensors -> packed buffer + CRC (read + write)
  unpack_device  packed buffer -> tensors + CRC verify (read + write)
  torch_copy     dst.copy_(src) (read + write), the roofline reference
  sync_unchanged incremental-checkpoint digest pass when nothing changed
  tpz_encode / tpz_decode  TPZ1 byte-plane codec on an AdamW-like state (GB/s of raw bytes)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters):
    import torch

    for _ in range(iters):  # steady state: the first launches of a kernel run ~12 % slower
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--gb", type=float, default=8.0)
    p.add_argument("--iters", type=int, default=5)
    args = p.parse_args()
    import torch

    from terraform_provider_iterative_amd import ops
    from terraform_provider_iterative_amd.ops.packing import PackPlan, pack, unpack

    n = int(args.gb * 1e9) // 4096 * 4096
    dev = torch.device("cuda", 0)
    buf = torch.randint(0, 256, (n,), dtype=torch.uint8, device=dev)
    out = {}
    t = timeit(lambda: ops.crc32c_tiles(buf), args.iters)
    out["crc32c_tiles_GBps"] = n / t / 1e9
    t = timeit(lambda: ops.shard_hash(buf), args.iters)
    out["shard_hash_GBps"] = n / t / 1e9
    # 16 tensors of mixed size (like a model shard) -> one stream
    sizes = [n // 32] * 8 + [n // 64] * 16
    views, off = {}, 0
    for i, s in enumerate(sizes):
        s = s // 256 * 256
        views["t%d" % i] = buf[off:off + s]
        off += s
    plan = PackPlan.from_tensors(views)
    stream = torch.empty(plan.total, dtype=torch.uint8, device=dev)
    crcs = [None]

    def do_pack():
        crcs[0] = pack(plan, stream)[1]

    t = timeit(do_pack, args.iters)
    out["pack_GBps"] = plan.total / t / 1e9
    t = timeit(lambda: unpack(plan, stream, crcs[0]), args.iters)
    out["unpack_GBps"] = plan.total / t / 1e9
    dst = torch.empty_like(buf)
    t = timeit(lambda: dst.copy_(buf), args.iters)
    out["torch_copy_GBps"] = n / t / 1e9
    # incremental checkpoint: digest pass over unchanged tensors (nothing to move)
    from terraform_provider_iterative_amd.checkpoint import Checkpointer

    ck = Checkpointer(views, chunk_bytes=256 << 20)
    ck.sync()
    t = timeit(lambda: ck.sync(), args.iters)
    out["sync_unchanged_GBps"] = plan.total / t / 1e9
    ck.close()
    # TPZ1 codec on AdamW-like state (bf16 N(0,.02) + fp32 N(0,1e-3) + fp32 N(0,1e-3)^2)
    from terraform_provider_iterative_amd.ops import codec

    q = n // 10 // 16 * 16
    state = torch.empty(10 * q, dtype=torch.uint8, device=dev)
    state[:2 * q].view(torch.bfloat16).normal_(0, 0.02)
    state[2 * q:6 * q].view(torch.float32).normal_(0, 1e-3)
    sq = state[6 * q:].view(torch.float32)
    sq.normal_(0, 1e-3)
    sq.mul_(sq)
    enc = [None]

    def do_encode():
        enc[0] = codec.encode(state)

    t = timeit(do_encode, args.iters)
    out["tpz_encode_GBps"] = state.numel() / t / 1e9
    blobs, sizes = enc[0]
    out["tpz_ratio"] = blobs.numel() / state.numel()
    t = timeit(lambda: codec.decode(blobs, sizes, state.numel()), args.iters)
    out["tpz_decode_GBps"] = state.numel() / t / 1e9
    back, _ = codec.decode(blobs, sizes, state.numel())
    out["tpz_roundtrip_ok"] = bool(torch.equal(back, state))
    del state, back, blobs
    out["bytes"] = n
    print(json.dumps({k: round(v, 4 if k == "tpz_ratio" else 1) if isinstance(v, float) else v
                      for k, v in out.items()}))


if __name__ == "__main__":
    main()
