# Round 4: does the successor's host-to-device traffic on SDMA slow its allocations of
# just-freed HBM?  Successor copies on blit kernels (HSA_ENABLE_SDMA=0, successor only) vs
# default, materialize, alternating.
set -o pipefail
mkdir -p gpurun_out/r4x
for i in 1 2; do
  timeout -k 10 240 python scripts/exp/bigstate_pair.py --mode materialize \
    --successor-env HSA_ENABLE_SDMA=0 > gpurun_out/r4x/blit_$i.json 2> gpurun_out/r4x/blit_$i.log || exit $?
  timeout -k 10 240 python scripts/exp/bigstate_pair.py --mode materialize \
    > gpurun_out/r4x/sdma_$i.json 2> gpurun_out/r4x/sdma_$i.log || exit $?
done
timeout -k 10 240 python scripts/exp/bigstate_pair.py --mode upfront \
  --successor-env HSA_ENABLE_SDMA=0 > gpurun_out/r4x/blit_u.json 2> gpurun_out/r4x/blit_u.log || exit $?
