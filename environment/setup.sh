#!/bin/bash
# Prepare an MI355X node for the tpi runtime (the node-local analogue of the reference's
# environment/setup.sh CML image setup): verify ROCm + PyTorch-ROCm, build the native
# components in-tree, and report the GPUs the placement layer will see.
set -euo pipefail
ROOT="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
command -v hipcc > /dev/null || { echo "hipcc not found: install ROCm >= 7.0" >&2; exit 1; }
python3 -c "import torch; print('torch', torch.__version__, 'hip', torch.version.hip)"
PYTORCH_ROCM_ARCH="${PYTORCH_ROCM_ARCH:-gfx950}" python3 -m terraform_provider_iterative_amd._build
python3 - << 'PY'
from terraform_provider_iterative_amd.parallel.placement import discover
gpus = discover()
print("GPUs visible to tpi placement:", len(gpus))
for g in gpus:
    print("  ", g.to_json())
PY
echo "state root: ${TPI_STATE_ROOT:-$HOME/.local/state/tpi}"
echo "add $ROOT/bin to PATH for leo, tpi and terraform-provider-iterative"
