# Variance of the driver's default bench and the effect of the first-log probe before the
# timed region (A/B/A/B on one box)
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 400 python bench.py --steps 5 > gpurun_out/bench_default_${i}_r3am.json 2> gpurun_out/bench_default_${i}_r3am.err || exit $?
  timeout -k 10 400 python bench.py --steps 5 --no-latency > gpurun_out/bench_nolat_${i}_r3am.json 2> gpurun_out/bench_nolat_${i}_r3am.err || exit $?
done
