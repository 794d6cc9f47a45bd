# Streamed restore with its H2D legs on host-driven SDMA engines (no HIP stream markers in the
# hardware queues the save's kernels use) vs HIP copy streams: kernel tests, then the
# overlapped bench A/B alternating, then config 4's streamed route
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/kern_tests_r3ax.log 2>&1 || exit $?
for i in 1 2; do
  for m in hip sdma; do
    TPI_RESTORE_H2D=$m timeout -k 10 400 python bench.py --steps 5 --no-latency --broadcast-gb 0 --no-async > gpurun_out/bench_h2d${m}_${i}_r3ax.json 2> gpurun_out/bench_h2d${m}_${i}_r3ax.err || exit $?
  done
done
TPI_HBM_HANDOFF=0 timeout -k 10 600 python bench/bench_preempt.py --gb 100 --hot > gpurun_out/preempt_stream_r3ax.json 2> gpurun_out/preempt_stream_r3ax.err
