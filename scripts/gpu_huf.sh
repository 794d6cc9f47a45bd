# HUF codec mode on MI355X: GPU suite, kernel bench, smoke, default headline bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "tpz or codec" > gpurun_out/pytest_huf_codec.log 2>&1 && echo CODEC_TESTS_OK &&
timeout -k 10 300 python bench/bench_kernels.py --gb 8 --iters 5 > gpurun_out/kernels_huf.json 2> gpurun_out/kernels_huf.err && echo KERNELS_OK &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_huf.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_huf.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 900 python bench.py > gpurun_out/bench_huf.log 2>&1 && echo BENCH_OK
