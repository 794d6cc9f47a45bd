#!/bin/bash
# Round 5: TPI_PRELOAD=gpu-lite (context + first queue, no engine): cold 100 GB preempt-recover
# and the parked process's HBM.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5ai
mkdir -p $O
cd $R
FOOTPRINT_LITE=1 timeout -k 10 300 python -u scripts/exp/preload_footprint.py > $O/footprint_lite.json 2> $O/footprint_lite.log || exit $?
cat $O/footprint_lite.json
timeout -k 10 400 python -u bench/bench_preempt.py --gb 100 --preload-gpu-lite > $O/cold_preload_gpu_lite.json 2> $O/cold_preload_gpu_lite.log || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/r5ai/cold_preload_gpu_lite.json"))
print("cold_preload_gpu_lite", d.get("signal_to_restored_s"), "ok", d.get("ok"))
print([l for l in d.get("logs_tail", [])][-1][:600])
PY
