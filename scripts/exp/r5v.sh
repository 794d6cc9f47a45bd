#!/bin/bash
# Round 5: the cold preempt-recover path with a preloaded successor (TPI_PRELOAD=1) vs plain.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5v
mkdir -p $O
cd $R
timeout -k 10 400 python -u bench/bench_preempt.py --gb 100 --preload > $O/cold_preload_100g.json 2> $O/cold_preload_100g.log || exit $?
timeout -k 10 400 python -u bench/bench_preempt.py --gb 100 > $O/cold_100g.json 2> $O/cold_100g.log || exit $?
python - <<'PY'
import json
for f in ("cold_preload_100g", "cold_100g"):
    d = json.load(open("gpurun_out/r5v/%s.json" % f))
    print(f, d.get("signal_to_restored_s"), "rank_start_to_restored", d.get("rank_start_to_restored_s"), "ok", d.get("ok"))
    print("   ", d.get("restore_journal"))
    for name, t, desc in d["timeline"][:14]:
        print("   %8.4f %-26s %s" % (t, name, " | ".join(desc)[:200]))
PY
