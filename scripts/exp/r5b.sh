#!/bin/bash
# Round 5: hand-off copy / verify kernel sweep (rows in flight per lane x bytes per launch x
# verify mode), 32 GB state; then the hand-off GPU tests under the inline check.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5b
mkdir -p $O
cd $R
run() {  # unroll span_mb verify
  echo "== unroll $1 span_mb $2 verify $3" >> $O/sweep.txt
  TPI_HANDOFF_UNROLL=$1 TPI_HANDOFF_SPAN_MB=$2 TPI_HANDOFF_VERIFY=$3 \
    timeout -k 10 200 python -u scripts/exp/handoff_kernels.py 32 2>&1 | grep -v amdgpu.ids >> $O/sweep.txt
}
for u in 8 16 4; do
  for span in 4096 0; do
    for v in readback inline none; do
      run $u $span $v || exit $?
    done
  done
done
cat $O/sweep.txt
TPI_HANDOFF_VERIFY=inline timeout -k 10 300 python -u -m pytest -x -v --timeout 120 \
  --timeout-method thread tests/test_gpu_kernels.py -k "handoff" > $O/pytest_inline.txt 2>&1
rc=$?
tail -12 $O/pytest_inline.txt
exit $rc
