# Kernel microbenchmarks + rocprofv3 kernel-trace/stats of the data-plane kernels.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 300 python bench/bench_kernels.py --gb 8 > gpurun_out/kernels.log 2>&1 && echo KERNELS_OK &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_kernels -o run -- python3 bench/bench_kernels.py --gb 4 --iters 3 > gpurun_out/prof_kernels.log 2>&1 && echo PROF_OK &&
timeout -k 10 300 python bench.py --total-gb 8 --steps 3 --warmup 1 --no-latency --mode direct > gpurun_out/bench_8g_direct.log 2>&1 && echo B8D_OK &&
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/gpurun_out/prof_bench -o run -- python3 bench.py --total-gb 16 --steps 2 --warmup 1 --no-latency > gpurun_out/prof_bench.log 2>&1 && echo PROFB_OK
