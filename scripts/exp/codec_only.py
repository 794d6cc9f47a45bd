"""Run only the TPZ1 device encode + decode of a 2 GB AdamW-like state (for PMC passes)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from terraform_provider_iterative_amd.ops import codec
q = int(2e9) // 10 // 16 * 16
state = torch.empty(10 * q, dtype=torch.uint8, device="cuda")
state[:2 * q].view(torch.bfloat16).normal_(0, 0.02)
state[2 * q:6 * q].view(torch.float32).normal_(0, 1e-3)
sq = state[6 * q:].view(torch.float32); sq.normal_(0, 1e-3); sq.mul_(sq)
blobs, sizes = codec.encode(state)
for _ in range(2):
    out, _ = codec.decode(blobs, sizes, state.numel())
torch.cuda.synchronize()
print("ok", torch.equal(out, state))
