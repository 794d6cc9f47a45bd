"""Experiment: the HBM hand-off's copy + read-back verify in one process (no IPC), so a
kernel trace splits its time between the fused copy and the verify: k_stream_hash<1> / <2>
(default tile digest) or, with TPI_HANDOFF_HASH=crc32c, k_stream_crc<3> / <4>.

    python scripts/exp/handoff_kernels.py [GB]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import synthetic_checkpoint  # noqa: E402
from terraform_provider_iterative_amd.checkpoint import Checkpointer  # noqa: E402
from terraform_provider_iterative_amd.ops.packing import PackPlan  # noqa: E402


def main():
    gb = float(sys.argv[1]) if len(sys.argv) > 1 else 32.0
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    src = synthetic_checkpoint(int(gb * 1e9), 8192, dev)
    dst = synthetic_checkpoint(int(gb * 1e9), 8192, dev, fill=False)
    torch.cuda.synchronize()
    tile = int(float(os.environ.get("HK_TILE_MB", "1")) * (1 << 20))
    ck = Checkpointer(dst, populate=False, tile_bytes=tile)  # the host region is not used here
    src_segs = PackPlan.from_tensors(src, ck.plan.tile_bytes).segs.copy()
    stream = torch.cuda.current_stream().cuda_stream
    for i in range(4):
        t = time.perf_counter()
        res = ck.engine.copy_segments(src_segs, ck.plan, stream)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        print("copy+verify %.1f GB: %.4f s, %.2f TB/s of state, %.2f TB/s of HBM traffic, "
              "bad tiles %d" % (ck.plan.total / 1e9, dt, ck.plan.total / dt / 1e12,
                                3 * ck.plan.total / dt / 1e12, res.bad_tiles), flush=True)
    names = list(src)[:3]
    assert all(torch.equal(src[n], dst[n]) for n in names)
    ck.close()


if __name__ == "__main__":
    main()
