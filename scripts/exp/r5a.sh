#!/bin/bash
# Round 5, first GPU call: the dma-buf hand-off route (probe + GPU tests), then the hand-off
# copy / verify kernels: timing, kernel trace, and one counter pass per block limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5a
mkdir -p $O
cd $R
step() { echo "[$(date +%T)] $*"; }
step dmabuf probe
for a in "--mib 64" "--mib 2100" "--mib 4300" "--mib 4300 --raw"; do
  timeout -k 10 150 python -u scripts/exp/dmabuf_handoff.py $a >> $O/dmabuf.jsonl || exit $?
done
cat $O/dmabuf.jsonl
step hbm tests
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_kernels.py -k "hbm" > $O/pytest_hbm.txt 2>&1 || { tail -30 $O/pytest_hbm.txt; exit 1; }
tail -8 $O/pytest_hbm.txt
step kernel timing
timeout -k 10 300 python -u scripts/exp/handoff_kernels.py 32 > $O/timing.txt 2>&1 || exit $?
TPI_HANDOFF_VERIFY=none timeout -k 10 300 python -u scripts/exp/handoff_kernels.py 32 > $O/timing_noverify.txt 2>&1 || exit $?
cat $O/timing.txt $O/timing_noverify.txt
export TMPDIR=/tmp
step kernel trace
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- \
  python3 $R/scripts/exp/handoff_kernels.py 16) > $O/trace.log 2>&1 || exit $?
step pmc FETCH_SIZE
(cd /tmp && timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run -- \
  python3 $R/scripts/exp/handoff_kernels.py 8) > $O/pmc_fetch.log 2>&1 || exit $?
step pmc WRITE_SIZE
(cd /tmp && timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run -- \
  python3 $R/scripts/exp/handoff_kernels.py 8) > $O/pmc_write.log 2>&1 || exit $?
step pmc occupancy
(cd /tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -d $O/pmc_occ -o run -- python3 $R/scripts/exp/handoff_kernels.py 8) > $O/pmc_occ.log 2>&1 || exit $?
step done
