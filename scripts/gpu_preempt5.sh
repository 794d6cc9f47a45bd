set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_runtime.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "prefetch" > gpurun_out/pytest_early.log 2>&1 && echo EARLY_TESTS_OK &&
timeout -k 10 600 python bench/bench_preempt.py --gb 100 > gpurun_out/preempt_100g_g.json 2> gpurun_out/preempt_100g_g.err && echo P100_OK && cat gpurun_out/preempt_100g_g.json
