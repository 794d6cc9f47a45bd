# Non-temporal stores in the scatter path (unpack / hand-off copy): kernel tests, in-process
# hand-off copy + verify at 32 GB with a kernel trace
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/kern_tests_r3al.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3al -o prof -- python3 scripts/exp/handoff_kernels.py 32 > gpurun_out/handoff_kernels_prof_r3al.log 2>&1 || exit $?
python3 scripts/rocpd_summary.py $(find gpurun_out/prof_r3al -name 'prof_results.db' | head -1) > gpurun_out/handoff_kernels_prof_r3al.md 2>&1 || exit $?
timeout -k 10 300 python bench/bench_kernels.py > gpurun_out/kernels_r3al.json 2> gpurun_out/kernels_r3al.err
