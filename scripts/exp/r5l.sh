#!/bin/bash
# Round 5: where the first hand-off copy's extra ~7 ms goes (scripts/exp/first_touch.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5l
mkdir -p $O
cd $R
FT_RESERVE=1 timeout -k 10 200 python -u scripts/exp/first_touch.py 50 > $O/reserve.jsonl 2> $O/reserve.log || exit $?
FT_RESERVE=1 FT_SMALL_FIRST=1 timeout -k 10 200 python -u scripts/exp/first_touch.py 50 > $O/small_first.jsonl 2> $O/small_first.log || exit $?
export TMPDIR=/tmp
(cd /tmp && FT_RESERVE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- \
  python3 $R/scripts/exp/first_touch.py 20) > $O/trace.log 2>&1 || exit $?
cat $O/reserve.jsonl $O/small_first.jsonl
