# Round 4: hardware queues per rank process (HIP default 4 vs 8, as bench.py sets for itself)
# for the two-process streamed hand-off, 100 GB, host route (TPI_HBM_HANDOFF=0), alternating.
set -o pipefail
mkdir -p gpurun_out/r4r
for i in 1 2; do
  TPI_HBM_HANDOFF=0 timeout -k 10 300 python bench/bench_preempt.py --gb 100 --hot \
    > gpurun_out/r4r/q4_$i.json 2> gpurun_out/r4r/q4_$i.log || exit $?
  GPU_MAX_HW_QUEUES=8 TPI_HBM_HANDOFF=0 timeout -k 10 300 python bench/bench_preempt.py --gb 100 \
    --hot > gpurun_out/r4r/q8_$i.json 2> gpurun_out/r4r/q8_$i.log || exit $?
done
