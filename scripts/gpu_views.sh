# Non-contiguous view paths: GPU tests, then strided pack/unpack throughput.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_views.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 300 python bench/bench_strided.py > gpurun_out/strided2.log 2>&1 && echo STRIDED_OK &&
timeout -k 10 300 python bench/bench_kernels.py --gb 8 > gpurun_out/kernels_views.log 2>&1 && echo KERNELS_OK
