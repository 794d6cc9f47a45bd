set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_async2.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 900 python bench/bench_async.py --gb 100 > gpurun_out/async100b.log 2>&1 && echo A100_OK &&
timeout -k 10 900 python bench.py > gpurun_out/bench_h.log 2>&1 && echo BENCH_OK
