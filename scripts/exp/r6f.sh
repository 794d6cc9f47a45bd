#!/bin/bash
# round 6, call F: the other recovery paths through the product's memory gates -- a spot
# reclaim (100 GB victim, the on-demand task then allocates 150 GB), a 150 GB hot hand-off,
# and a 170 GB state restored with materialize() behind its predecessor's spill.
set -o pipefail
O=gpurun_out/r6f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u bench/bench_reclaim.py --gb 100 > $O/reclaim_100g.json 2> $O/reclaim.err
rc=$?; tail -c 1500 $O/reclaim_100g.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench/bench_preempt.py --gb 150 --hot > $O/hot_150g.json 2> $O/hot_150g.err
rc=$?; python -c "import json;d=json.loads(open('$O/hot_150g.json').read().strip().splitlines()[-1]);print({k:d.get(k) for k in ('ok','signal_to_restored_s','gpu_drain','successor_hbm_wait','hbm_failed','hbm_skipped','restore_journal')})"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench/bench_preempt.py --gb 170 --materialize > $O/materialize_170g.json 2> $O/materialize_170g.err
rc=$?; python -c "import json;d=json.loads(open('$O/materialize_170g.json').read().strip().splitlines()[-1]);print({k:d.get(k) for k in ('ok','signal_to_restored_s','gpu_drain','successor_hbm_wait','hbm_failed','restore_journal')})"
exit $rc
