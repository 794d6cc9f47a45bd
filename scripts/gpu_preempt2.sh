set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python bench/bench_preempt.py --gb 100 > gpurun_out/preempt_100g_b.json 2> gpurun_out/preempt_100g_b.err && echo P100_OK && cat gpurun_out/preempt_100g_b.json
