# Round 4: config 2 (10 GB workdir) with the push as hard links (TPI_PUSH_LINK=1) vs copies.
set -o pipefail
mkdir -p gpurun_out/r4z
for i in 1 2; do
  timeout -k 10 400 python bench/bench_workdir.py --gb 10 > gpurun_out/r4z/copy_$i.json \
    2> gpurun_out/r4z/copy_$i.log || exit $?
  TPI_PUSH_LINK=1 timeout -k 10 400 python bench/bench_workdir.py --gb 10 \
    > gpurun_out/r4z/link_$i.json 2> gpurun_out/r4z/link_$i.log || exit $?
done
