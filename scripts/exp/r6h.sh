#!/bin/bash
# round 6, call H: the 150 GB hot hand-off with the offer measured against the registered
# state (r6g: the hot standby's context counted as state sent it to the host path), and the
# spot reclaim again (r6f: the requeued spot task's start took 150 GB being wiped for an idle
# level; the flat window now scales with the count).
set -o pipefail
O=gpurun_out/r6h
mkdir -p $O
export TMPDIR=/tmp
S="import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print({k:d.get(k) for k in ('ok','signal_to_restored_s','gpu_drain','successor_hbm_wait','hbm_failed','hbm_skipped','restore_journal')})"
timeout -k 10 400 python -u bench/bench_preempt.py --gb 150 --hot > $O/hot_150g.json 2> $O/hot_150g.err
rc=$?; python -c "$S" $O/hot_150g.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench/bench_reclaim.py --gb 100 > $O/reclaim_100g.json 2> $O/reclaim.err
rc=$?; python -c "import json;d=json.load(open('$O/reclaim_100g.json'));print({k:d.get(k) for k in ('ok','od_apply_to_first_log_s','spot_resumed_verified')});[print(e) for e in d.get('spot_timeline',[]) if e[0] in ('gpu-drain','placed','rank-start','checkpoint-restored')]"
exit $rc
