"""Experiment: why the hand-off's first copy runs ~12 % slower than later ones (57 vs 50 ms per
100 GB, profiles/round5/handoff_kernels.md). One process, ``GB`` of state per tensor set:

  A  copy src -> dst three times (first vs steady);
  B  copy src -> a freshly allocated dst2 (never touched);
  C  a fresh dst3, written once by a fill kernel, then copied into;
  D  2 s of an idle GPU, then src -> dst again (clock ramp).

Prints the kernels' device time of each copy (``TransferResult.device_seconds``).

    python scripts/exp/first_touch.py [GB]
"""
import json
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
    gb = float(sys.argv[1]) if len(sys.argv) > 1 else 50.0
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream().cuda_stream
    src = synthetic_checkpoint(int(gb * 1e9), 8192, dev)
    src_segs = None
    out = []

    def copy(ck, label):
        t = time.perf_counter()
        res = ck.engine.copy_segments(src_segs, ck.plan, stream)
        torch.cuda.synchronize()
        row = {"case": label, "wall_s": round(time.perf_counter() - t, 4),
               "kernels_s": round(res.device_seconds, 4), "bad_tiles": res.bad_tiles}
        out.append(row)
        print(json.dumps(row), flush=True)

    dst = synthetic_checkpoint(int(gb * 1e9), 8192, dev, fill=False)
    torch.cuda.synchronize()
    ck = Checkpointer(dst, populate=False)
    src_segs = PackPlan.from_tensors(src, ck.plan.tile_bytes).segs.copy()
    if os.environ.get("FT_RESERVE"):  # what a hot standby does before the signal
        ck.engine.reserve(len(src_segs), ck.plan.ntiles, False)
    if os.environ.get("FT_SMALL_FIRST"):  # one small copy first: is the cost per launch size?
        n = max(1, int(float(os.environ["FT_SMALL_FIRST"]) * (1 << 20)) // 4)  # MiB -> floats
        small = {"a": torch.ones(n, device=dev)}
        small_dst = {"a": torch.zeros(n, device=dev)}
        cks = Checkpointer(small_dst, populate=False)
        r = cks.engine.copy_segments(PackPlan.from_tensors(small, cks.plan.tile_bytes).segs.copy(),
                                     cks.plan, stream)
        print(json.dumps({"case": "small %s MiB first" % os.environ["FT_SMALL_FIRST"],
                          "kernels_s": round(r.device_seconds, 4)}),
              flush=True)
        cks.close()
    for i in range(3):
        copy(ck, "A%d src->dst" % i)
    ck2 = Checkpointer(synthetic_checkpoint(int(gb * 1e9), 8192, dev, fill=False), populate=False)
    torch.cuda.synchronize()
    copy(ck2, "B fresh dst2")
    copy(ck2, "B fresh dst2 again")
    ck2.close()
    del ck2
    torch.cuda.empty_cache()
    dst3 = synthetic_checkpoint(int(gb * 1e9), 8192, dev, fill=False)
    for t in dst3.values():
        t.zero_()
    torch.cuda.synchronize()
    ck3 = Checkpointer(dst3, populate=False)
    copy(ck3, "C zeroed dst3")
    ck3.close()
    time.sleep(2.0)
    copy(ck, "D after 2 s idle")
    copy(ck, "D again")
    ck.close()


if __name__ == "__main__":
    main()
