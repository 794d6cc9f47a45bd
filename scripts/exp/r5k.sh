#!/bin/bash
# Round 5: hot hand-off e2e with the prewarmed hand-off kernels and 2 rows in flight (100 GB,
# with and without the 4.2 / 2.5 GiB tensors); each run waits for the GPU to drain first.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5k
mkdir -p $O
cd $R
timeout -k 10 400 python -u bench/bench_preempt.py --gb 100 --hot --extra-gib 4.2,2.5 > $O/hot_100g_big.json 2> $O/hot_100g_big.log || exit $?
timeout -k 10 400 python -u bench/bench_preempt.py --gb 100 --hot > $O/hot_100g.json 2> $O/hot_100g.log || exit $?
python - <<'PY'
import json
for f in ("hot_100g_big", "hot_100g"):
    d = json.load(open("gpurun_out/r5k/%s.json" % f))
    print(f, d.get("signal_to_restored_s"), d.get("restore_journal"), "ok", d.get("ok"),
          "vram", d.get("vram_before_start"))
PY
