#!/bin/bash
# Round 5: the relocation route on a fresh box, the big-tensor state FIRST (r5f / r5g ran it
# second, right after another 100 GB run whose processes may still have held HBM); every run
# now waits for the GPU's memory to drain first and journals the free HBM at the copy.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5h
mkdir -p $O
cd $R
cat /sys/bus/pci/devices/*/mem_info_vram_total 2>/dev/null | head -3 > $O/vram_total.txt
timeout -k 10 400 python -u bench/bench_preempt.py --gb 100 --hot --extra-gib 4.2,2.5 > $O/hot_100g_big.json 2> $O/hot_100g_big.log || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/r5h/hot_100g_big.json"))
print("big", d.get("signal_to_restored_s"), d.get("restore_journal"), "ok", d.get("ok"),
      "vram", d.get("vram_before_start"))
for row in d.get("timeline", [])[:14]:
    print("   ", row)
PY
