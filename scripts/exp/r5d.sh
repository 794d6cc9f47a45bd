#!/bin/bash
# Round 5: the one GPU test that failed in r5c, then the headline bench with preempt_e2e.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5d
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_runtime.py -m gpu -v --timeout 240 \
  --timeout-method thread -k "releases_device_memory" > $O/gpu_test.txt 2>&1
rc=$?
tail -3 $O/gpu_test.txt
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 1000 python -u bench.py --steps 5 --warmup 1 > $O/bench.json 2> $O/bench.log
brc=$?
grep -v amdgpu.ids $O/bench.log | tail -6
cat $O/bench.json
exit $(( rc > brc ? rc : brc ))
