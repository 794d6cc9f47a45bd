set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for mode in 1 0 1 0; do timeout -k 10 900 python bench/bench_workdir.py --gb 10 --steps 5 --zero-copy $mode > gpurun_out/wd_zc_$mode.json 2>/dev/null && python3 -c "import json; d=json.load(open('gpurun_out/wd_zc_$mode.json')); print('zc=$mode', round(d['stage_GBps'],2), d['stage_stats'])" || exit 1; done
