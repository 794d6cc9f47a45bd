#!/bin/bash
# round 6, call U: (1) the workdir push's copy methods on the box's /tmp (CPU only);
# (2) the 170 GB materialize recovery twice more: r6r's first group took 2.75 s (r6f: 0.14 s).
set -o pipefail
O=gpurun_out/r6u
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 bash scripts/exp/r6t.sh > $O/push.txt 2>&1 || exit $?
cp gpurun_out/r6t/* $O/ 2>/dev/null
for i in 1 2; do
  timeout -k 10 500 python -u bench/bench_preempt.py --gb 170 --materialize > $O/materialize_170g_$i.json 2> $O/materialize_170g_$i.err
  rc=$?
  python -c "
import json
d=json.loads(open('$O/materialize_170g_$i.json').read().strip().splitlines()[-1])
t=d['logs_tail'][1]; i=t.find(\"'trace'\")
print({k:d.get(k) for k in ('ok','verified','signal_to_restored_s','rank_start_to_restored_s')}, t[i:i+120])"
  [ $rc -eq 0 ] || exit $rc
done
