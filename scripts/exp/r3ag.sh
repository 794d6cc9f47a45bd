# Copy timeline of the overlapped step at 100 GB vs 32 GB (why the restore lags more at 100 GB)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for gb in 32 100; do
  timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/prof_r3ag_$gb -o prof -- python3 bench.py --total-gb $gb --steps 1 --warmup 1 --no-latency --broadcast-gb 0 --no-async > gpurun_out/bench${gb}_r3ag.json 2> gpurun_out/bench${gb}_r3ag.err || exit $?
  python3 scripts/exp/copy_timeline.py $(find gpurun_out/prof_r3ag_$gb -name 'prof_results.db' | head -1) > gpurun_out/timeline_r3ag_$gb.md 2>&1 || exit $?
done
