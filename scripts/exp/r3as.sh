# Config 2: workdir push from the GPU's NUMA node (TPI_PUSH_NUMA=1, default) vs the caller's
# cores, alternating on one box
mkdir -p gpurun_out
for i in 1 2; do
  for n in 0 1; do
    TPI_PUSH_NUMA=$n timeout -k 10 300 python bench/bench_workdir.py --gb 10 > gpurun_out/config2_numa${n}_${i}_r3as.json 2> gpurun_out/config2_numa${n}_${i}_r3as.err || exit $?
  done
done
