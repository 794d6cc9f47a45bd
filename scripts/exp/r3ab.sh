mkdir -p gpurun_out
for c in 256 1024; do timeout -k 10 300 python scripts/exp/async_interference.py 32 8192 $c >> gpurun_out/interf_r3ab.log 2>&1 || exit $?; done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3ab -o prof -- python3 bench.py --total-gb 16 --steps 2 --warmup 1 --no-latency --broadcast-gb 0 --no-async --chunk-mb 1024 > gpurun_out/bench16_c1024_r3ab.json 2> gpurun_out/bench16_c1024_r3ab.err
