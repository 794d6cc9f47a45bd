# Round 4: which HIP call does the materializing successor block in during its ~2 s stall?
# HIP API + kernel + copy trace of the standalone pair (spill pinned first), one warm-up run.
set -o pipefail
mkdir -p gpurun_out/r4u
timeout -k 10 240 python scripts/exp/bigstate_pair.py --mode materialize \
  > gpurun_out/r4u/warm.json 2> gpurun_out/r4u/warm.log || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv \
  -d gpurun_out/r4u/trace -o run_%pid% -- python3 scripts/exp/bigstate_pair.py --mode materialize \
  > gpurun_out/r4u/traced.json 2> gpurun_out/r4u/traced.log || exit $?
