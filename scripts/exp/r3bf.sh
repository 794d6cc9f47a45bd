# Ring depth 3 vs 4 staging buffers, alternating, three passes (100 GB, 5 timed steps)
mkdir -p gpurun_out
for pass in 1 2 3; do
  for nb in 3 4; do
    timeout -k 10 400 python bench.py --steps 5 --no-latency --broadcast-gb 0 --no-async --nbuf $nb > gpurun_out/bench_n${nb}_p${pass}_r3bf.json 2> gpurun_out/bench_n${nb}_p${pass}_r3bf.err || exit $?
  done
done
