# Kernel-level profile of the current data-plane kernels + LDS counters incl. k_transpose.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_k2 -o run -- python3 bench/bench_kernels.py --gb 4 --iters 3 > gpurun_out/prof_k2.log 2>&1 && echo PROF_OK &&
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES --kernel-trace --stats -d $R/gpurun_out/pmc_views -o run -- python3 bench/bench_strided.py > gpurun_out/pmc_views.log 2>&1 && echo PMC_OK
