"""Workdir staging: zero-copy vs bounce on the same 10 x 1 GB page-cached files."""
import json, os, shutil, sys, tempfile, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from terraform_provider_iterative_amd.runtime.workdir import stage_workdir
d = tempfile.mkdtemp(dir=os.environ.get("DIR", "/tmp"))
blk = os.urandom(64 << 20)
for i in range(10):
    with open(os.path.join(d, "f%d.bin" % i), "wb") as f:
        for _ in range(16):
            f.write(blk)
out = []
for zc in (1 << 40, 64 << 20, 1 << 40, 64 << 20):
    torch.cuda.synchronize()
    t = time.perf_counter()
    s = stage_workdir(d, device=torch.device("cuda", 0), zero_copy_min=zc)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    out.append({"zero_copy_min": zc, "GBps": round(s.stats["bytes"] / dt / 1e9, 2),
                "stats": {k: (round(v, 4) if isinstance(v, float) else v) for k, v in s.stats.items()}})
    del s
shutil.rmtree(d)
print(json.dumps(out, indent=1))
