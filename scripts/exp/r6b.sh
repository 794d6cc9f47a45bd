#!/bin/bash
# round 6, call B: the GPU suite on the split engine, the HIP IPC runtime matrix
# (VERDICT r5 #3), then the driver's bench command (preempt_e2e without a bench-side drain).
set -o pipefail
O=gpurun_out/r6b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $O/pytest.txt 2>&1
rc=$?
tail -3 $O/pytest.txt
echo "pytest rc $rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u scripts/exp/ipc_runtime.py --out $O/ipc_runtime > $O/ipc_runtime.txt 2>&1
rc=$?
cut -c1-400 $O/ipc_runtime.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?
tail -c 3000 $O/bench.json
exit $rc
