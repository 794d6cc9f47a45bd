#!/usr/bin/env python3
"""How PyTorch's caching allocator holds a block of --mib MiB (round 4, IPC size probe):
the allocator settings and the snapshot's segment record for that block."""
import json
import os
import sys

import torch

mib = float(sys.argv[sys.argv.index("--mib") + 1]) if "--mib" in sys.argv else 2100
t = torch.empty(int(mib * (1 << 20)), dtype=torch.uint8, device="cuda")
segs = [{k: v for k, v in s.items() if k != "blocks"} | {"blocks": len(s["blocks"])}
        for s in torch.cuda.memory_snapshot()]
print(json.dumps({"env": {k: v for k, v in os.environ.items() if "ALLOC" in k},
                  "backend": torch.cuda.get_allocator_backend(),
                  "ptr": t.data_ptr(), "segments": segs}, default=str))
