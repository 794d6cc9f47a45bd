# Pipeline granularity of the overlapped step after the run-ahead bound: chunk size and ring
# depth (100 GB, 3 timed steps each, two passes)
mkdir -p gpurun_out
for pass in 1 2; do
  for cfg in "256 3" "128 3" "512 3" "256 4"; do
    set -- $cfg
    timeout -k 10 400 python bench.py --steps 3 --no-latency --broadcast-gb 0 --no-async --chunk-mb $1 --nbuf $2 > gpurun_out/bench_c$1_n$2_p${pass}_r3be.json 2> gpurun_out/bench_c$1_n$2_p${pass}_r3be.err || exit $?
  done
done
