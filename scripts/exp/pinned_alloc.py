"""Experiment: cost of pinned bounce buffers (torch pin_memory vs mmap + parallel touch +
hipHostRegister through HostRegion)."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from terraform_provider_iterative_amd.checkpoint.host import HostRegion
torch.cuda.init(); torch.empty(1, device="cuda")
out = {}
for mb in (64, 256):
    t = time.perf_counter(); a = [torch.empty(mb << 20, dtype=torch.uint8, pin_memory=True) for _ in range(2)]; out["torch_pin_2x%dMB_s" % mb] = round(time.perf_counter() - t, 4)
    t = time.perf_counter(); r = HostRegion(2 * (mb << 20), None, device=True, numa_node=-1, populate=True); out["hostregion_2x%dMB_s" % mb] = round(time.perf_counter() - t, 4)
    t = time.perf_counter(); r.close(); out["hostregion_close_%dMB_s" % mb] = round(time.perf_counter() - t, 4)
    del a
print(json.dumps(out))
