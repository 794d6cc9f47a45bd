# Round 4: restore H2D on its own SDMA engine (TPI_MATERIALIZE_H2D=sdma) vs HIP's engine,
# materializing 170 GB successor, standalone pair, alternating; GPU tests of the new path first.
set -o pipefail
mkdir -p gpurun_out/r4y
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py -k "own_sdma_engine or restore_streams or materialize" \
  > gpurun_out/r4y/tests.log 2>&1 || exit $?
TPI_MATERIALIZE_H2D=sdma timeout -k 10 300 python -u -m pytest -x -v --timeout 120 \
  --timeout-method thread tests/test_gpu_kernels.py -k "materialize" \
  > gpurun_out/r4y/tests_sdma.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 240 python scripts/exp/bigstate_pair.py --mode materialize \
    --successor-env TPI_MATERIALIZE_H2D=sdma > gpurun_out/r4y/sdma_$i.json \
    2> gpurun_out/r4y/sdma_$i.log || exit $?
  timeout -k 10 240 python scripts/exp/bigstate_pair.py --mode materialize \
    > gpurun_out/r4y/hip_$i.json 2> gpurun_out/r4y/hip_$i.log || exit $?
done
