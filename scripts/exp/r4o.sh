# Round 4: tile metadata straight in host memory (meta_view) vs per-chunk copies
# (TPI_DIRECT_META=0), alternating on one box; the GPU kernel tests first.
set -o pipefail
mkdir -p gpurun_out/r4o
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_runtime.py > gpurun_out/r4o/tests.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 400 python bench.py --steps 5 --no-latency --broadcast-gb 0 --no-async \
    > gpurun_out/r4o/direct_$i.json 2> gpurun_out/r4o/direct_$i.err || exit $?
  TPI_DIRECT_META=0 timeout -k 10 400 python bench.py --steps 5 --no-latency --broadcast-gb 0 \
    --no-async > gpurun_out/r4o/copies_$i.json 2> gpurun_out/r4o/copies_$i.err || exit $?
done
