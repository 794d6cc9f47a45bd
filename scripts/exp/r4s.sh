# Round 4: the big-state hand-off outside the supervisor (scripts/exp/bigstate_pair.py):
# both successor modes alternating, then one materialize run under a kernel + copy trace.
set -o pipefail
mkdir -p gpurun_out/r4s
for i in 1 2; do
  timeout -k 10 240 python scripts/exp/bigstate_pair.py --mode materialize \
    > gpurun_out/r4s/plain_m$i.json 2> gpurun_out/r4s/plain_m$i.log || exit $?
  timeout -k 10 240 python scripts/exp/bigstate_pair.py --mode upfront \
    > gpurun_out/r4s/plain_u$i.json 2> gpurun_out/r4s/plain_u$i.log || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
  -d gpurun_out/r4s/trace -o run_%pid% -- python3 scripts/exp/bigstate_pair.py --mode materialize \
  > gpurun_out/r4s/traced_m.json 2> gpurun_out/r4s/traced_m.log || exit $?
