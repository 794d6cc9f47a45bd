#!/bin/bash
# Round 5: where do the hot hand-off's 2.3 s go?  Hot standby, 100 GB, with and without the
# 4.2/2.5 GiB tensors; full phase timelines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5e
mkdir -p $O
cd $R
timeout -k 10 400 python -u bench/bench_preempt.py --gb 100 --hot > $O/hot_100g.json 2> $O/hot_100g.log || exit $?
timeout -k 10 400 python -u bench/bench_preempt.py --gb 100 --hot --extra-gib 4.2,2.5 > $O/hot_100g_big.json 2> $O/hot_100g_big.log || exit $?
python - <<'PY'
import json
for f in ("hot_100g", "hot_100g_big"):
    d = json.load(open("gpurun_out/r5e/%s.json" % f))
    print(f, d.get("signal_to_restored_s"), d.get("restore_journal"))
    for row in d.get("timeline", []):
        print("   ", row)
PY
