# Round 1 GPU pass 4: TPZ1 codec -- kernel tests, codec throughput, 100 GB bench with/without.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -q -x > gpurun_out/pytest_codec.log 2>&1 && echo PYTEST_KERNELS_OK &&
timeout -k 10 300 python bench/bench_kernels.py --gb 8 > gpurun_out/kernels_d.log 2>&1 && echo KERNELS_OK &&
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_tpz1.log 2>&1 && echo BENCH_TPZ1_OK &&
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --codec none --no-latency > gpurun_out/bench_raw.log 2>&1 && echo BENCH_RAW_OK &&
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_ALL_OK
