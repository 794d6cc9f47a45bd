mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/kern_tests_r3u.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --total-gb 32 --steps 3 --warmup 1 --no-latency --broadcast-gb 0 --no-async > gpurun_out/bench32_r3u.json 2> gpurun_out/bench32_r3u.err || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_default_r3u.json 2> gpurun_out/bench_default_r3u.err
