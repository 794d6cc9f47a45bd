# Round 4: chunk size and staging depth with the save's tile metadata stored in place.
set -o pipefail
mkdir -p gpurun_out/r4aa
B="python bench.py --steps 5 --no-latency --broadcast-gb 0 --no-async"
timeout -k 10 400 $B > gpurun_out/r4aa/def_1.json 2> gpurun_out/r4aa/def_1.err || exit $?
timeout -k 10 400 $B --chunk-mb 512 > gpurun_out/r4aa/c512.json 2> gpurun_out/r4aa/c512.err || exit $?
timeout -k 10 400 $B --nbuf 6 > gpurun_out/r4aa/n6.json 2> gpurun_out/r4aa/n6.err || exit $?
timeout -k 10 400 $B --chunk-mb 128 --nbuf 8 > gpurun_out/r4aa/c128n8.json 2> gpurun_out/r4aa/c128n8.err || exit $?
timeout -k 10 400 $B > gpurun_out/r4aa/def_2.json 2> gpurun_out/r4aa/def_2.err || exit $?
