# Round 4: materialize with allocations gated on free memory, standalone pair and bench_preempt.
set -o pipefail
mkdir -p gpurun_out/r4v
for i in 1 2; do
  timeout -k 10 240 python scripts/exp/bigstate_pair.py --mode materialize \
    > gpurun_out/r4v/pair_m$i.json 2> gpurun_out/r4v/pair_m$i.log || exit $?
done
timeout -k 10 240 python scripts/exp/bigstate_pair.py --mode upfront \
  > gpurun_out/r4v/pair_u1.json 2> gpurun_out/r4v/pair_u1.log || exit $?
for i in 1 2; do
  timeout -k 10 400 python bench/bench_preempt.py --gb 170 --hot --materialize \
    > gpurun_out/r4v/bench_m$i.json 2> gpurun_out/r4v/bench_m$i.log || exit $?
done
timeout -k 10 400 python bench/bench_preempt.py --gb 170 --hot \
  > gpurun_out/r4v/bench_u1.json 2> gpurun_out/r4v/bench_u1.log || exit $?
