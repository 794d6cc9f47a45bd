#!/bin/bash
# Round 5: hand-off kernels at 100 GB (the hand-off's size): tile size x rows in flight, and
# the read-back's share; the GPU tests touched by this round's engine changes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5j
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_runtime.py -k "hbm or handoff or releases or prewarm" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
run() {  # tile_mb unroll verify
  echo "== tile_mb $1 unroll $2 verify $3" >> $O/sweep.txt
  HK_TILE_MB=$1 TPI_HANDOFF_UNROLL=$2 TPI_HANDOFF_VERIFY=$3 \
    timeout -k 10 300 python -u scripts/exp/handoff_kernels.py 100 2>&1 | grep -v amdgpu.ids >> $O/sweep.txt
}
for t in 1 2 4; do
  for u in 4 2; do
    run $t $u readback || exit $?
  done
done
run 1 4 none || exit $?
cat $O/sweep.txt
