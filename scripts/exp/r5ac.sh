#!/bin/bash
# Round 5: HIP IPC import time of a 50 GB state against the number of opening threads.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5ac
mkdir -p $O
cd $R
for t in 1 8 32; do
  TPI_IPC_OPEN_THREADS=$t timeout -k 10 240 python -u scripts/exp/ipc_copy_rate.py 50 > $O/threads_$t.jsonl 2> $O/threads_$t.log || exit $?
  grep '"ipc open"' $O/threads_$t.jsonl
done
