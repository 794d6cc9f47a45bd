#!/bin/bash
# Round 5: cold preempt-recover with a preloaded successor that also initialised the GPU.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5x
mkdir -p $O
cd $R
timeout -k 10 400 python -u bench/bench_preempt.py --gb 100 --preload-gpu > $O/cold_preload_gpu_100g.json 2> $O/cold_preload_gpu_100g.log || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/r5x/cold_preload_gpu_100g.json"))
print("cold_preload_gpu", d.get("signal_to_restored_s"), "ok", d.get("ok"))
print("   ", d.get("restore_journal"))
for name, t, desc in d["timeline"][:12]:
    print("   %8.4f %-26s %s" % (t, name, " | ".join(desc)[:200]))
print([l for l in d.get("logs_tail", [])][-3:])
PY
