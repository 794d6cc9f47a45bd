#!/bin/bash
# round 6, call W: the final tree (64 MiB push pieces) -- GPU
# suite, smoke(), apply -> first log with 9 samples, then the driver's bench command.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6w
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
for i in 1 2; do
  timeout -k 10 300 python -u -c "import json; from terraform_provider_iterative_amd.bench_latency import measure_first_log_latency as m; print(json.dumps(m(repeats=9)))" >> $O/latency.txt 2>> $O/latency.err || exit $?
done
cat $O/latency.txt
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?
tail -12 $O/bench.err
exit $rc
