#!/bin/bash
# round 6, call D: the whole GPU suite on the final tree (split engine + supervisor, gates),
# kernel traces of the save/restore pipelines and of the hand-off kernels, then the driver's
# bench command.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6d
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $O/pytest.txt 2>&1
rc=$?
tail -3 $O/pytest.txt
echo "pytest rc $rc"
[ $rc -eq 0 ] || exit $rc
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_bench -o run -- \
  python3 $R/bench.py --steps 2 --warmup 1 --preempt-e2e none --config2 none --no-latency \
  --no-async --broadcast-gb 0) > $O/trace_bench.log 2>&1 || exit $?
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_handoff -o run -- \
  python3 $R/scripts/exp/handoff_kernels.py 16) > $O/trace_handoff.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?
tail -12 $O/bench.err
exit $rc
