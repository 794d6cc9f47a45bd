"""The HBM copy ceiling on this GPU, for the hand-off kernels' numbers: HIP's own
device-to-device copy (``Tensor.copy_`` -> ``hipMemcpyAsync`` D2D, a blit kernel) against the
hand-off's copy kernel alone (``TPI_HANDOFF_VERIFY=none``) and with its read-back verify, on
one flat ``GB`` tensor.  One JSON line per case (median of 5 after one warm-up).

    python scripts/exp/d2d_ceiling.py [GB]
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from terraform_provider_iterative_amd.checkpoint import Checkpointer  # noqa: E402
from terraform_provider_iterative_amd.ops.packing import PackPlan  # noqa: E402


def timed(fn, n=5):
    fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        out.append(a.elapsed_time(b) / 1e3)
    return statistics.median(out)


def main():
    gb = float(sys.argv[1]) if len(sys.argv) > 1 else 50.0
    n = int(gb * 1e9) // 8 * 8
    src = torch.arange(n // 8, dtype=torch.int64, device="cuda").view(torch.uint8)
    dst = torch.empty_like(src)
    torch.cuda.synchronize()
    rows = []

    def emit(case, seconds, traffic):
        row = {"case": case, "gb": gb, "seconds": round(seconds, 5),
               "state_TBps": round(n / seconds / 1e12, 3),
               "hbm_traffic_TBps": round(traffic * n / seconds / 1e12, 3)}
        rows.append(row)
        print(json.dumps(row), flush=True)

    emit("hipMemcpy D2D (Tensor.copy_)", timed(lambda: dst.copy_(src)), 2)
    ck = Checkpointer({"dst": dst}, populate=False)
    segs = PackPlan.from_tensors({"dst": src}, ck.plan.tile_bytes).segs.copy()
    stream = torch.cuda.current_stream().cuda_stream
    for verify, traffic in (("none", 2), ("readback", 3)):
        os.environ["TPI_HANDOFF_VERIFY"] = verify
        emit("hand-off copy, verify=%s" % verify,
             timed(lambda: ck.engine.copy_segments(segs, ck.plan, stream)), traffic)
    os.environ.pop("TPI_HANDOFF_VERIFY", None)
    emit("read only (Tensor.sum over int64)",
         timed(lambda: src.view(torch.int64).sum()), 1)
    assert torch.equal(src[-4096:], dst[-4096:])
    ck.close()


if __name__ == "__main__":
    main()
