#!/bin/bash
# Round 5: hand-off copy / verify kernel sweep (rows in flight per lane x bytes per launch),
# 32 GB state, with and without the read-back verify.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5b
mkdir -p $O
cd $R
for u in 8 16 4; do
  for span in 4096 16384 0; do
    for v in readback none; do
      echo "== unroll $u span_mb $span verify $v" >> $O/sweep.txt
      TPI_HANDOFF_UNROLL=$u TPI_HANDOFF_SPAN_MB=$span TPI_HANDOFF_VERIFY=$v \
        timeout -k 10 200 python -u scripts/exp/handoff_kernels.py 32 >> $O/sweep.txt 2>&1 || exit $?
    done
  done
done
grep -v amdgpu.ids $O/sweep.txt
