set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_runtime.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "stage" > gpurun_out/pytest_zc2.log 2>&1 && echo ZC_TESTS_OK &&
timeout -k 10 300 python scripts/exp/stage_modes.py > gpurun_out/stage_modes2.json 2>gpurun_out/stage_modes2.err && echo SM_OK && grep GBps gpurun_out/stage_modes2.json &&
timeout -k 10 900 python bench/bench_workdir.py --gb 10 --steps 20 > gpurun_out/workdir_10g_zc2.json 2>gpurun_out/workdir_10g_zc2.err && echo WD_OK && cat gpurun_out/workdir_10g_zc2.json
