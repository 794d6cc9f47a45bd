# Copy timeline of the overlapped 100 GB step with 8 HW queues (bench.py's default now)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/prof_r3aw_100 -o prof -- python3 bench.py --total-gb 100 --steps 1 --warmup 1 --no-latency --broadcast-gb 0 --no-async > gpurun_out/bench100_r3aw.json 2> gpurun_out/bench100_r3aw.err || exit $?
python3 scripts/exp/copy_timeline.py $(find gpurun_out/prof_r3aw_100 -name 'prof_results.db' | head -1) > gpurun_out/timeline_r3aw.md 2>&1
