set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -q -x -k "async or checkpointer" > gpurun_out/pytest_async.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 600 python bench/bench_async.py --gb 32 > gpurun_out/async32.log 2>&1 && echo A32_OK &&
timeout -k 10 900 python bench/bench_async.py --gb 100 > gpurun_out/async100.log 2>&1 && echo A100_OK
