# Hand-off digest: XXH64-class stream hash vs CRC32C tiles (kernel tests, in-process copy +
# verify at 32 GB with a kernel trace, then config 4 end to end on the HBM route)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/kern_tests_r3ak.log 2>&1 || exit $?
for h in xxh crc32c; do
  TPI_HANDOFF_HASH=$h timeout -k 10 300 python scripts/exp/handoff_kernels.py 32 > gpurun_out/handoff_kernels_${h}_r3ak.log 2>&1 || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3ak -o prof -- python3 scripts/exp/handoff_kernels.py 32 > gpurun_out/handoff_kernels_prof_r3ak.log 2>&1 || exit $?
python3 scripts/rocpd_summary.py $(find gpurun_out/prof_r3ak -name 'prof_results.db' | head -1) > gpurun_out/handoff_kernels_prof_r3ak.md 2>&1 || exit $?
timeout -k 10 600 python bench/bench_preempt.py --gb 100 --hot > gpurun_out/preempt_hot_r3ak.json 2> gpurun_out/preempt_hot_r3ak.err
