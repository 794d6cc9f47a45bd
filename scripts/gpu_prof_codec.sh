# rocprofv3 of the TPZ1 checkpoint path: kernels + copies + roctx ranges, then LDS counters.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --marker-trace --stats -d $R/gpurun_out/prof_codec -o run -- python3 bench.py --total-gb 16 --steps 2 --warmup 1 --no-latency > gpurun_out/prof_codec.log 2>&1 && echo PROF_CODEC_OK &&
timeout -k 10 300 rocprofv3 --list-avail > gpurun_out/counters_avail.txt 2>&1 && echo LIST_OK &&
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES --kernel-trace --stats -d $R/gpurun_out/pmc_codec -o run -- python3 bench/bench_kernels.py --gb 2 --iters 2 > gpurun_out/pmc_codec.log 2>&1 && echo PMC_OK
