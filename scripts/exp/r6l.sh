#!/bin/bash
# round 6, call L: distributions on the final tree -- the bench's cold (default preloaded
# successor) and hot e2e runs, four each, back to back through the product's gates (each
# start waits for the previous run's memory), plus two spot reclaims.
set -o pipefail
O=gpurun_out/r6l
mkdir -p $O
export TMPDIR=/tmp
S="import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1].split('/')[-1], {k:d.get(k) for k in ('ok','verified','signal_to_restored_s','gpu_drain','preload_gpu')})"
for i in 1 2 3 4; do
  timeout -k 10 300 python -u bench/bench_preempt.py --gb 100 > $O/cold_$i.json 2> $O/cold_$i.err
  rc=$?; python -c "$S" $O/cold_$i.json; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u bench/bench_preempt.py --gb 100 --hot --extra-gib 4.2,2.5 > $O/hot_$i.json 2> $O/hot_$i.err
  rc=$?; python -c "$S" $O/hot_$i.json; [ $rc -eq 0 ] || exit $rc
done
for i in 1 2; do
  timeout -k 10 400 python -u bench/bench_reclaim.py --gb 100 > $O/reclaim_$i.json 2> $O/reclaim_$i.err
  rc=$?; python -c "import json;d=json.load(open('$O/reclaim_$i.json'));print({k:d.get(k) for k in ('ok','od_apply_to_first_log_s','spot_resumed_verified')})"
  [ $rc -eq 0 ] || exit $rc
done
