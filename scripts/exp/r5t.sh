#!/bin/bash
# Round 5: the hot hand-off's steps (claim / open / plan / meminfo / copy) in the journal.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5t
mkdir -p $O
cd $R
timeout -k 10 400 python -u bench/bench_preempt.py --gb 100 --hot --extra-gib 4.2,2.5 > $O/hot_100g_big.json 2> $O/hot_100g_big.log || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/r5t/hot_100g_big.json"))
print("hot_100g_big", d.get("signal_to_restored_s"), "ok", d.get("ok"))
for name, t, desc in d["timeline"][:12]:
    print("%8.4f %-28s %s" % (t, name, " | ".join(desc)[:240]))
PY
