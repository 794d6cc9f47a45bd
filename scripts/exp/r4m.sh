# Round 4: is the successor's restore stalled behind the driver's clearing of freed HBM on
# SDMA engine 0?  HSA_ENABLE_SDMA=0 moves every HIP copy of both ranks to blit kernels.
set -o pipefail
mkdir -p gpurun_out/r4m
HSA_ENABLE_SDMA=0 timeout -k 10 300 python bench/bench_preempt.py --gb 170 --hot --materialize \
  > gpurun_out/r4m/m170_blit.json 2> gpurun_out/r4m/m170_blit.log || exit $?
HSA_ENABLE_SDMA=0 timeout -k 10 300 python bench/bench_preempt.py --gb 170 --hot \
  > gpurun_out/r4m/b170_blit.json 2> gpurun_out/r4m/b170_blit.log || exit $?
