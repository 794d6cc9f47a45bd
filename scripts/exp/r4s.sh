# Round 4: the big-state hand-off outside the supervisor: traced first (a fresh box's first
# run is the one that showed a ~10 s block), then plain runs of both successor modes.
set -o pipefail
mkdir -p gpurun_out/r4s
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
  -d gpurun_out/r4s/trace -o run_%pid% -- python3 scripts/exp/bigstate_pair.py --mode materialize \
  > gpurun_out/r4s/traced_m.json 2> gpurun_out/r4s/traced_m.log || exit $?
timeout -k 10 240 python scripts/exp/bigstate_pair.py --mode materialize \
  > gpurun_out/r4s/plain_m.json 2> gpurun_out/r4s/plain_m.log || exit $?
timeout -k 10 240 python scripts/exp/bigstate_pair.py --mode upfront \
  > gpurun_out/r4s/plain_u.json 2> gpurun_out/r4s/plain_u.log || exit $?
