# GPU_MAX_HW_QUEUES and a training loop next to a background spill (save_async), then the
# driver's default bench with bench.py's own queue default
mkdir -p gpurun_out
for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python scripts/exp/async_interference.py 32 8192 256 > gpurun_out/interf_q${q}_r3ap.log 2>&1 || exit $?
done
timeout -k 10 600 python bench.py > gpurun_out/bench_default_r3ap.json 2> gpurun_out/bench_default_r3ap.err
