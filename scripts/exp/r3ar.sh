# Background spill next to a GEMM loop: TPZ1 codec vs no codec (training time lost per
# periodic checkpoint), and config 2 alone
mkdir -p gpurun_out
for c in tpz1 none; do
  timeout -k 10 300 python scripts/exp/async_interference.py 32 8192 256 $c > gpurun_out/interf_${c}_r3ar.log 2>&1 || exit $?
done
timeout -k 10 300 python bench/bench_workdir.py --gb 10 > gpurun_out/config2_r3ar.json 2> gpurun_out/config2_r3ar.err
