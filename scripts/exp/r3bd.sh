# The driver's command (20 timed steps after 5 warmups), twice on one box
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver_${i}_r3bd.json 2> gpurun_out/bench_driver_${i}_r3bd.err || exit $?
done
