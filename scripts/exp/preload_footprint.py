"""HBM held by a parked TPI_PRELOAD=gpu successor: the device's used VRAM (sysfs, read without
touching the GPU) before and after runtime/preload.py's GPU warm-up in this process."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from terraform_provider_iterative_amd.parallel.placement import (discover, vram_usage,  # noqa: E402
                                                                 wait_vram_drained)

PCI = discover()[0].pci  # KFD sysfs: no HIP call


def used():
    u = vram_usage(PCI)
    return None if u is None else round(u[0] / 1e9, 3)


drained = wait_vram_drained(PCI, fraction=0.002)  # earlier runs may still hold VRAM
before = used()
import torch  # noqa: E402,F401

from terraform_provider_iterative_amd.runtime.preload import _warm_gpu  # noqa: E402

t = time.perf_counter()
_warm_gpu(engine=os.environ.get("FOOTPRINT_LITE") is None)
took = time.perf_counter() - t
time.sleep(0.5)
after = used()
print(json.dumps({"drained": drained, "vram_before_gb": before, "vram_after_gb": after,
                  "parked_gb": round(after - before, 3), "warm_s": round(took, 3)}))
