# Strided-view paths: throughput + rocprofv3 kernel trace (k_transpose vs pack/unpack).
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -q -x > gpurun_out/pytest_views2.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 300 python bench/bench_strided.py > gpurun_out/strided3.log 2>&1 && echo STRIDED_OK &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_views -o run -- python3 bench/bench_strided.py > gpurun_out/prof_views.log 2>&1 && echo PROF_OK
