#!/bin/bash
# round 6, call E: stage tests after the stage/stage_native split, and the apply -> first-log
# latency (mi355x, 9 samples) after the CLI import trims.
set -o pipefail
O=gpurun_out/r6e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_stage.py -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $O/pytest.txt 2>&1
rc=$?
tail -3 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "
import json, sys; sys.path.insert(0, '.')
from terraform_provider_iterative_amd.bench_latency import measure_first_log_latency
for i in range(2):
    print(json.dumps(measure_first_log_latency(repeats=9)), flush=True)
" > $O/latency.txt 2>&1
rc=$?
cat $O/latency.txt
exit $rc
