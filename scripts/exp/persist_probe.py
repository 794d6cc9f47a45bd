"""Time Checkpointer.persist/load of a 16 GB device checkpoint on this box's disk (and the
raw sequential rate of that filesystem), to size a native persist/load path."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from terraform_provider_iterative_amd.checkpoint import Checkpointer

target = sys.argv[1] if len(sys.argv) > 1 else "/tmp"
gb = float(sys.argv[2]) if len(sys.argv) > 2 else 16
n = int(gb * 1e9) // 4
t = {"w": torch.randn(n, device="cuda")}
ck = Checkpointer(t, codec="tpz1")
ck.save()
path = os.path.join(target, "tpi-persist-probe.ckpt")
t0 = time.perf_counter()
ck.persist(path)
tp = time.perf_counter() - t0
size = os.path.getsize(path)
os.sync()  # the file may still be in the page cache: load is an upper bound
t0 = time.perf_counter()
ck.load(path)
torch.cuda.synchronize()
tl = time.perf_counter() - t0
print("persist %.2f GB in %.2f s (%.1f GB/s); load+restore %.2f s (%.1f GB/s of file)" % (
    size / 1e9, tp, size / tp / 1e9, tl, size / tl / 1e9), flush=True)
os.remove(path)
