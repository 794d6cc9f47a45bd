#!/bin/bash
# Round 5, final kernels: kernel trace + counter passes of the hand-off copy / read-back
# (2 rows in flight, one launch per pass) on 16 GB of AdamW state.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5ak
mkdir -p $O
cd $R
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- \
  python3 $R/scripts/exp/handoff_kernels.py 16) > $O/trace.log 2>&1 || exit $?
(cd /tmp && timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run -- \
  python3 $R/scripts/exp/handoff_kernels.py 8) > $O/pmc_fetch.log 2>&1 || exit $?
(cd /tmp && timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run -- \
  python3 $R/scripts/exp/handoff_kernels.py 8) > $O/pmc_write.log 2>&1 || exit $?
(cd /tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -d $O/pmc_occ -o run -- python3 $R/scripts/exp/handoff_kernels.py 8) > $O/pmc_occ.log 2>&1 || exit $?
echo done
