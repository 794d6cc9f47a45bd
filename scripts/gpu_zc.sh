set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_runtime.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "stage or prefetch" > gpurun_out/pytest_zc.log 2>&1 && echo ZC_TESTS_OK &&
timeout -k 10 900 python bench/bench_workdir.py --gb 10 --steps 20 > gpurun_out/workdir_10g_zc.json 2>gpurun_out/workdir_10g_zc.err && echo WD_OK && cat gpurun_out/workdir_10g_zc.json
