# rocprofv3 of the TPZ1 (HUF) checkpoint path: kernels + copies.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/gpurun_out/prof_huf -o run -- python3 bench.py --total-gb 16 --steps 2 --warmup 1 --no-latency --no-async > gpurun_out/prof_huf.log 2>&1 && echo PROF_OK &&
python3 scripts/rocpd_summary.py $(ls $R/gpurun_out/prof_huf/*/run_results.db 2>/dev/null | head -1 || ls $R/gpurun_out/prof_huf/run_results.db) > gpurun_out/prof_huf_summary.md 2>&1; ls -R gpurun_out/prof_huf | head -20
