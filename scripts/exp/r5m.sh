#!/bin/bash
# Round 5: which first copy absorbs the process's first-copy cost (16 KiB / 64 MiB / 256 MiB),
# then the 100 GB hot hand-off with the span fix.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5m
mkdir -p $O
cd $R
for mb in 0.016 64 256; do
  FT_RESERVE=1 FT_SMALL_FIRST=$mb timeout -k 10 200 python -u scripts/exp/first_touch.py 50 > $O/small_$mb.jsonl 2> $O/small_$mb.log || exit $?
  head -3 $O/small_$mb.jsonl
done
timeout -k 10 400 python -u bench/bench_preempt.py --gb 100 --hot --extra-gib 4.2,2.5 > $O/hot_100g_big.json 2> $O/hot_100g_big.log || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/r5m/hot_100g_big.json"))
print("hot_100g_big", d.get("signal_to_restored_s"), d.get("restore_journal"), "ok", d.get("ok"))
PY
