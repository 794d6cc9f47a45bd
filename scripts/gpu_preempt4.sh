set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_runtime.py tests/test_examples.py tests/test_task_smoke.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_runtime_e.log 2>&1 && echo RT_OK &&
timeout -k 10 600 python bench/bench_preempt.py --gb 100 > gpurun_out/preempt_100g_e.json 2> gpurun_out/preempt_100g_e.err && echo P100_OK && cat gpurun_out/preempt_100g_e.json &&
timeout -k 10 600 python bench/bench_preempt.py --gb 100 --no-standby > gpurun_out/preempt_100g_f.json 2> gpurun_out/preempt_100g_f.err && echo P100C_OK && cat gpurun_out/preempt_100g_f.json
