set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_runtime.py -q -x > gpurun_out/pytest_async3.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 900 python bench/bench_async.py --gb 100 > gpurun_out/async100c.log 2>&1 && echo A100_OK
