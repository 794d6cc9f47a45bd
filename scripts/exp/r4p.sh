# Round 4: direct tile metadata on the save side only vs per-chunk copies, alternating.
set -o pipefail
mkdir -p gpurun_out/r4p
for i in 1 2; do
  TPI_DIRECT_META=save timeout -k 10 400 python bench.py --steps 5 --no-latency --broadcast-gb 0 \
    --no-async > gpurun_out/r4p/save_$i.json 2> gpurun_out/r4p/save_$i.err || exit $?
  TPI_DIRECT_META=0 timeout -k 10 400 python bench.py --steps 5 --no-latency --broadcast-gb 0 \
    --no-async > gpurun_out/r4p/copies_$i.json 2> gpurun_out/r4p/copies_$i.err || exit $?
  TPI_DIRECT_META=restore timeout -k 10 400 python bench.py --steps 5 --no-latency \
    --broadcast-gb 0 --no-async > gpurun_out/r4p/restore_$i.json 2> gpurun_out/r4p/restore_$i.err || exit $?
done
