# Round 4: 170 GB big-state recovery, up-front allocation vs Checkpointer.materialize(),
# alternating on one box, plus the 100 GB streamed host hand-off (two processes, duplex).
set -o pipefail
mkdir -p gpurun_out/r4i
for i in 1 2; do
  timeout -k 10 300 python bench/bench_preempt.py --gb 170 --hot --materialize \
    > gpurun_out/r4i/m170_$i.json 2> gpurun_out/r4i/m170_$i.log || exit $?
  timeout -k 10 300 python bench/bench_preempt.py --gb 170 --hot \
    > gpurun_out/r4i/b170_$i.json 2> gpurun_out/r4i/b170_$i.log || exit $?
done
TPI_HBM_HANDOFF=0 timeout -k 10 300 python bench/bench_preempt.py --gb 100 --hot \
  > gpurun_out/r4i/s100.json 2> gpurun_out/r4i/s100.log || exit $?
