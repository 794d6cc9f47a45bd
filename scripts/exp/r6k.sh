#!/bin/bash
# round 6, call K: the final tree -- GPU suite, smoke(), the driver's bench command, and the
# N=4 rehearsal (gloo, one GPU) with rank 0's first-log probe now run before the other
# ranks' setup.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6k
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $O/pytest.txt 2>&1
rc=$?
tail -3 $O/pytest.txt
echo "pytest rc $rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
tail -1 $O/smoke.txt
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?
tail -12 $O/bench.err
[ $rc -eq 0 ] || exit $rc
TPI_BENCH_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29604 bench.py --gpus 4 \
    --steps 2 --warmup 1 > $O/rehearse_n4.json 2> $O/rehearse_n4.err
rc=$?
grep "apply -> first log" $O/rehearse_n4.err
exit $rc
