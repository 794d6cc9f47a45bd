#!/bin/bash
# Round 5: the successor's region pinning held during the HBM hand-off; preloaded (gpu and
# default) and hot 100 GB preempt-recover; the prefetch / hand-off GPU tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5ad
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_runtime.py tests/test_gpu_kernels.py -k "prefetch or hbm or hand_off or handoff or pinned" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for run in "cold_preload_gpu --preload-gpu" "cold_preload --preload" "hot_big --hot --extra-gib 4.2,2.5"; do
  set -- $run; name=$1; shift
  timeout -k 10 400 python -u bench/bench_preempt.py --gb 100 "$@" > $O/$name.json 2> $O/$name.log || exit $?
  python - "$name" <<'PY'
import json, sys
d = json.load(open("gpurun_out/r5ad/%s.json" % sys.argv[1]))
j = d.get("restore_journal") or []
print(sys.argv[1], d.get("signal_to_restored_s"), "ok", d.get("ok"), [x for x in j if "ipc open" in x or "steps" in x])
PY
done
