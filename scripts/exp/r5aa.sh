#!/bin/bash
# Round 5: engine creation with the host pipelines' streams made on a thread of their own;
# the kernel/runtime GPU tests on it; then the cold (preloaded) 100 GB preempt-recover.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5aa
mkdir -p $O
cd $R
timeout -k 10 200 python -u scripts/exp/engine_create.py > $O/engine_create.txt 2>&1 || { cat $O/engine_create.txt; exit 1; }
cat $O/engine_create.txt
timeout -k 10 700 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_stage.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
timeout -k 10 400 python -u bench/bench_preempt.py --gb 100 > $O/cold_100g.json 2> $O/cold_100g.log || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/r5aa/cold_100g.json"))
print("cold (preloaded)", d.get("signal_to_restored_s"), "ok", d.get("ok"))
print([l for l in d.get("logs_tail", [])][-2:])
PY
