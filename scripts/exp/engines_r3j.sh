mkdir -p gpurun_out
for e in sdma1 sdma2 sdma3; do
  TPI_D2H_ENGINE=$e timeout -k 10 200 python bench.py --total-gb 32 --steps 3 --warmup 1 --no-latency --broadcast-gb 0 --no-async > gpurun_out/eng_${e}_r3j.json 2> gpurun_out/eng_${e}_r3j.err || exit $?
done
timeout -k 10 300 python bench/bench_preempt.py --gb 100 --hot > gpurun_out/preempt_hot_r3j.json 2> gpurun_out/preempt_hot_r3j.err
