#!/bin/bash
# Which engine runs our D2H/H2D copies?  Each case under rocprofv3 --kernel-trace: a line
# "blit kernels: N" counts __amd_rocclr_copyBuffer dispatches (0 = SDMA / copy engine).
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/copyeng
mkdir -p "$OUT"
i=0
for env in "X=0" "GPU_BLIT_ENGINE_TYPE=1" "GPU_BLIT_ENGINE_TYPE=2"; do
  for kind in register hostmalloc; do
    for dir in d2h h2d; do
      i=$((i+1))
      d="$OUT/c$i"
      echo "== $env $kind $dir" >> "$OUT/summary.txt"
      env $env timeout -k 5 120 rocprofv3 --kernel-trace --stats -d "$d" -o run -- \
        python3 scripts/exp/copy_engines.py $kind $dir 1 >> "$OUT/summary.txt" 2>> "$OUT/err.txt" || exit 1
      n=$(cat $(find "$d" -name '*kernel_stats.csv') 2>/dev/null | grep -c copyBuffer || true)
      echo "blit kernels: $n" >> "$OUT/summary.txt"
      grep copyBuffer $(find "$d" -name '*kernel_stats.csv') >> "$OUT/summary.txt" 2>/dev/null || true
    done
  done
done
