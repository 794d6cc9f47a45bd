# Does the save's D2H idle because its kernels share a hardware queue with the restore's?
# (HIP maps a process's streams onto GPU_MAX_HW_QUEUES queues, 4 by default)
mkdir -p gpurun_out
for q in 4 8 16 4; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 400 python bench.py --steps 5 --no-latency --broadcast-gb 0 --no-async > gpurun_out/bench_q${q}_r3an.json 2> gpurun_out/bench_q${q}_r3an.err || exit $?
done
