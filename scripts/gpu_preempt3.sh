set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_runtime.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_runtime_c.log 2>&1 && echo RT_OK &&
timeout -k 10 600 python bench/bench_preempt.py --gb 100 > gpurun_out/preempt_100g_c.json 2> gpurun_out/preempt_100g_c.err && echo P100_OK && cat gpurun_out/preempt_100g_c.json &&
timeout -k 10 600 python bench/bench_preempt.py --gb 100 --no-prefetch > gpurun_out/preempt_100g_d.json 2> gpurun_out/preempt_100g_d.err && echo P100N_OK && cat gpurun_out/preempt_100g_d.json
