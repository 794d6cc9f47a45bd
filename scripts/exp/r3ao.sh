# HW queue count A/B, alternating on one box (3 x 4 queues, 3 x 8 queues)
mkdir -p gpurun_out
for i in 1 2 3; do
  for q in 4 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 400 python bench.py --steps 5 --no-latency --broadcast-gb 0 --no-async > gpurun_out/bench_q${q}_${i}_r3ao.json 2> gpurun_out/bench_q${q}_${i}_r3ao.err || exit $?
  done
done
