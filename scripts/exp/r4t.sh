# Round 4: big-state hand-off with the successor's spill fully pinned first (a hot standby's
# steady state), both successor modes alternating; then the supervisor-driven bench_preempt.
set -o pipefail
mkdir -p gpurun_out/r4t
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_runtime.py -k "preempt_resume_training" > gpurun_out/r4t/tests.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 240 python scripts/exp/bigstate_pair.py --mode materialize \
    > gpurun_out/r4t/pair_m$i.json 2> gpurun_out/r4t/pair_m$i.log || exit $?
  timeout -k 10 240 python scripts/exp/bigstate_pair.py --mode upfront \
    > gpurun_out/r4t/pair_u$i.json 2> gpurun_out/r4t/pair_u$i.log || exit $?
done
timeout -k 10 400 python bench/bench_preempt.py --gb 170 --hot --materialize \
  > gpurun_out/r4t/bench_m.json 2> gpurun_out/r4t/bench_m.log || exit $?
timeout -k 10 400 python bench/bench_preempt.py --gb 170 --hot \
  > gpurun_out/r4t/bench_u.json 2> gpurun_out/r4t/bench_u.log || exit $?
