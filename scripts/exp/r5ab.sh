#!/bin/bash
# Round 5: HBM hand-off GPU tests + the 100 GB hot hand-off after the vectorized plan.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5ab
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_runtime.py -k "hbm or handoff or hand_off" > $O/pytest_hbm.txt 2>&1 || { tail -30 $O/pytest_hbm.txt; exit 1; }
tail -2 $O/pytest_hbm.txt
timeout -k 10 400 python -u bench/bench_preempt.py --gb 100 --hot --extra-gib 4.2,2.5 > $O/hot_100g_big.json 2> $O/hot_100g_big.log || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/r5ab/hot_100g_big.json"))
print("hot_100g_big", d.get("signal_to_restored_s"), "ok", d.get("ok"))
print(d.get("restore_journal"))
PY
