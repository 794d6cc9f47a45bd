set -o pipefail; mkdir -p gpurun_out; timeout -k 10 200 python scripts/exp/pinned_alloc.py 2>/dev/null | tail -1
