set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "tpz or codec" > gpurun_out/pytest_codec_p.log 2>&1 && echo CODEC_TESTS_OK &&
timeout -k 10 300 python bench/bench_kernels.py --gb 8 --iters 5 > gpurun_out/kernels_p.json 2> gpurun_out/kernels_p.err && echo KERNELS_OK && cat gpurun_out/kernels_p.json
