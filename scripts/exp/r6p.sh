#!/bin/bash
# round 6, call P: the 150 GB hot hand-off with the parked-standby measure (the standby's
# context counted once), then 100 GB hot (regression), 160 GB hot (still the big-state path)
# and the GPU tests of the preemption paths.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6p
mkdir -p $O
cd $R
export TMPDIR=/tmp
S="import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1].split('/')[-1], {k:d.get(k) for k in ('ok','verified','signal_to_restored_s','gpu_drain','successor_hbm_wait','hbm_failed','hbm_skipped','restore_journal')})"
for spec in "150 --hot" "100 --hot --extra-gib 4.2,2.5" "160 --hot" "150 --hot"; do
  set -- $spec
  name=hot_${1}g_$(date +%s)
  timeout -k 10 400 python -u bench/bench_preempt.py --gb $spec > $O/$name.json 2> $O/$name.err
  rc=$?; python -c "$S" $O/$name.json; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider -k "preempt or standby or handoff or hbm or resume" > $O/pytest.txt 2>&1
rc=$?
tail -3 $O/pytest.txt
exit $rc
