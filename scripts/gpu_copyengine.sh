# Sweep HIP runtime copy-engine knobs for the D2H leg of checkpoint save.
set -o pipefail
mkdir -p gpurun_out
run() { name=$1; shift; echo "== $name" >> gpurun_out/copyengine.log; env "$@" timeout -k 10 200 python bench.py --total-gb 16 --steps 3 --warmup 1 --no-latency >> gpurun_out/copyengine.log 2>&1; }
run default X=1 &&
run blit_type1 GPU_BLIT_ENGINE_TYPE=1 &&
run blit_type2 GPU_BLIT_ENGINE_TYPE=2 &&
run limit_wg16 DEBUG_CLR_LIMIT_BLIT_WG=16 &&
run limit_wg64 DEBUG_CLR_LIMIT_BLIT_WG=64 &&
echo "== direct" >> gpurun_out/copyengine.log; timeout -k 10 200 python bench.py --total-gb 16 --steps 3 --warmup 1 --no-latency --mode direct >> gpurun_out/copyengine.log 2>&1;
echo DONE
