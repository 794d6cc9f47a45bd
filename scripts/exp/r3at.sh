# (1) streamed saves copy each chunk's CRCs behind its pack kernel instead of a synchronous
#     hipMemcpy per published chunk: kernel tests, then the overlapped bench A/B, alternating
# (2) config 2 with the push on the GPU's NUMA node vs the caller's cores, alternating
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/kern_tests_r3at.log 2>&1 || exit $?
for i in 1 2; do
  for m in sync async; do
    TPI_SAVE_CRC_COPY=$m timeout -k 10 400 python bench.py --steps 5 --no-latency --broadcast-gb 0 --no-async > gpurun_out/bench_crc${m}_${i}_r3at.json 2> gpurun_out/bench_crc${m}_${i}_r3at.err || exit $?
  done
done
for i in 1 2; do
  for n in 0 1; do
    TPI_PUSH_NUMA=$n timeout -k 10 300 python bench/bench_workdir.py --gb 10 > gpurun_out/config2_numa${n}_${i}_r3at.json 2> gpurun_out/config2_numa${n}_${i}_r3at.err || exit $?
  done
done
