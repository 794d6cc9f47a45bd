#!/bin/bash
# Round 5: the hand-off copy with the predecessor's save running on the same GPU (as in a hot
# hand-off), copy stream at normal vs highest priority; then the 100 GB hot hand-off.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5o
mkdir -p $O
cd $R
IPC_RATE_SAVE=1 TPI_HANDOFF_PRIORITY=normal timeout -k 10 300 python -u scripts/exp/ipc_copy_rate.py 50 > $O/save_normal.jsonl 2> $O/save_normal.log || exit $?
IPC_RATE_SAVE=1 timeout -k 10 300 python -u scripts/exp/ipc_copy_rate.py 50 > $O/save_high.jsonl 2> $O/save_high.log || exit $?
cat $O/save_normal.jsonl $O/save_high.jsonl
timeout -k 10 400 python -u bench/bench_preempt.py --gb 100 --hot --extra-gib 4.2,2.5 > $O/hot_100g_big.json 2> $O/hot_100g_big.log || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/r5o/hot_100g_big.json"))
print("hot_100g_big", d.get("signal_to_restored_s"), d.get("restore_journal"), "ok", d.get("ok"))
PY
