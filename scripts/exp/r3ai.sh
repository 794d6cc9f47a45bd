# After bounding the streamed restore's run-ahead: the driver's default bench, a copy timeline
# of the overlapped 100 GB step, and config 4's streamed route (HBM hand-off off)
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_default_r3ai.json 2> gpurun_out/bench_default_r3ai.err || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/prof_r3ai_100 -o prof -- python3 bench.py --total-gb 100 --steps 1 --warmup 1 --no-latency --broadcast-gb 0 --no-async > gpurun_out/bench100_r3ai.json 2> gpurun_out/bench100_r3ai.err || exit $?
TPI_HBM_HANDOFF=0 timeout -k 10 400 python bench/bench_preempt.py --gb 100 --hot > gpurun_out/preempt_stream_r3ai.json 2> gpurun_out/preempt_stream_r3ai.err
