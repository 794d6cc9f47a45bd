mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/kern_tests_r3w.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --total-gb 32 --steps 3 --warmup 1 --no-latency --broadcast-gb 0 --no-async > gpurun_out/bench32_r3w.json 2> gpurun_out/bench32_r3w.err || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/prof_r3w -o prof -- python3 bench.py --total-gb 16 --steps 2 --warmup 1 --no-latency --broadcast-gb 0 --no-async > gpurun_out/bench16_r3w.json 2> gpurun_out/bench16_r3w.err
