# Round 4: materialize allocation lookahead 3 (default) vs 8 groups, bench_preempt 170 GB,
# alternating on one box.
set -o pipefail
mkdir -p gpurun_out/r4w
for i in 1 2; do
  timeout -k 10 400 python bench/bench_preempt.py --gb 170 --hot --materialize \
    > gpurun_out/r4w/l3_$i.json 2> gpurun_out/r4w/l3_$i.log || exit $?
  TPI_ALLOC_LOOKAHEAD=8 timeout -k 10 400 python bench/bench_preempt.py --gb 170 --hot \
    --materialize > gpurun_out/r4w/l8_$i.json 2> gpurun_out/r4w/l8_$i.log || exit $?
done
