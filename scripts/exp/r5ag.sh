#!/bin/bash
# Round 5: GPU tests + smoke + headline bench on the last tree of the round.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5ag
mkdir -p $O
cd $R
echo "[$(date +%T)] gpu tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread \
  > $O/gpu_tests.txt 2>&1
rc=$?
tail -25 $O/gpu_tests.txt
case $rc in 0|1) ;; *) echo "tests ended with $rc: stopping"; exit $rc;; esac
echo "[$(date +%T)] smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
echo "[$(date +%T)] bench"
timeout -k 10 900 python -u bench.py --steps 5 --warmup 1 > $O/bench.json 2> $O/bench.log
brc=$?
tail -5 $O/bench.log
cat $O/bench.json
exit $(( rc > brc ? rc : brc ))
