#!/bin/bash
# round 6, call G: the 150 GB hot hand-off after aligning the predecessor's offer with the
# successor's need (r6f: both waited out the 20 s linger), and a 160 GB hot run, which no
# longer fits twice: the spill frees behind itself and the successor streams behind it.
set -o pipefail
O=gpurun_out/r6g
mkdir -p $O
export TMPDIR=/tmp
S="import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print({k:d.get(k) for k in ('ok','signal_to_restored_s','gpu_drain','successor_hbm_wait','hbm_failed','hbm_skipped','restore_journal')})"
for gb in 150 160; do
  timeout -k 10 400 python -u bench/bench_preempt.py --gb $gb --hot > $O/hot_${gb}g.json 2> $O/hot_${gb}g.err
  rc=$?; python -c "$S" $O/hot_${gb}g.json; [ $rc -eq 0 ] || exit $rc
done
