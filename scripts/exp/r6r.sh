#!/bin/bash
# round 6, call R: the final tree on the remaining recovery paths -- a spot reclaim and a
# 170 GB state restored with materialize() -- after the supervisor took over the port probe.
set -o pipefail
O=gpurun_out/r6r
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u bench/bench_reclaim.py --gb 100 > $O/reclaim_100g.json 2> $O/reclaim.err
rc=$?; python -c "import json;d=json.load(open('$O/reclaim_100g.json'));print({k:d.get(k) for k in ('ok','od_apply_to_first_log_s','spot_resumed_verified')})"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench/bench_preempt.py --gb 170 --materialize > $O/materialize_170g.json 2> $O/materialize_170g.err
rc=$?; python -c "import json;d=json.loads(open('$O/materialize_170g.json').read().strip().splitlines()[-1]);print({k:d.get(k) for k in ('ok','verified','signal_to_restored_s','gpu_drain','restore_journal')})"
exit $rc
