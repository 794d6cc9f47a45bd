#!/bin/bash
# Round 5: the relocation route for allocations >= 2 GiB: GPU tests, then 100 GB hot hand-offs
# with and without 4.2 / 2.5 GiB tensors.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5g
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_kernels.py -k "hbm or handoff" > $O/pytest_hbm.txt 2>&1 || { tail -30 $O/pytest_hbm.txt; exit 1; }
tail -3 $O/pytest_hbm.txt
timeout -k 10 400 python -u bench/bench_preempt.py --gb 100 --hot > $O/hot_100g.json 2> $O/hot_100g.log || exit $?
timeout -k 10 400 python -u bench/bench_preempt.py --gb 100 --hot --extra-gib 4.2,2.5 > $O/hot_100g_big.json 2> $O/hot_100g_big.log || exit $?
python - <<'PY'
import json
for f in ("hot_100g", "hot_100g_big"):
    d = json.load(open("gpurun_out/r5g/%s.json" % f))
    print(f, d.get("signal_to_restored_s"), d.get("restore_journal"), "ok", d.get("ok"))
    for row in d.get("timeline", [])[:12]:
        print("   ", row)
PY
