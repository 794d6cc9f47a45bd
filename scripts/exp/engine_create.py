"""Where a device engine's creation time goes (TPI_ENGINE_TRACE=1 prints each step): the
successor of a cold preemption creates one before its first restore (~0.24-0.32 s,
profiles/round5/r5v)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.environ["TPI_ENGINE_TRACE"] = "1"

import torch  # noqa: E402

from terraform_provider_iterative_amd.checkpoint.engine import DeviceEngine  # noqa: E402

t = time.perf_counter()
torch.empty(1 << 20, device="cuda")
torch.cuda.synchronize()
print("torch cuda init %.3f s" % (time.perf_counter() - t), flush=True)
for i in range(2):
    t = time.perf_counter()
    e = DeviceEngine(0, 256 << 20, 3, 1 << 20)
    print("engine %d: %.3f s" % (i, time.perf_counter() - t), flush=True)
    e.close()
