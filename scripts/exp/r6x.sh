#!/bin/bash
# round 6, call X: kernel traces of the final tree -- the headline's save/restore pipeline
# (2 timed steps of bench.py, side measurements off) and the HBM hand-off kernels (16 GB).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6x
mkdir -p $O
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_bench -o run -- \
  python3 $R/bench.py --steps 2 --warmup 1 --preempt-e2e none --config2 none --no-latency \
  --no-async --broadcast-gb 0) > $O/trace_bench.log 2>&1 || exit $?
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_handoff -o run -- \
  python3 $R/scripts/exp/handoff_kernels.py 16) > $O/trace_handoff.log 2>&1 || exit $?
find $O -name '*.db' | head
