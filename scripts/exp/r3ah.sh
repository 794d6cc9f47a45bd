# Streamed restore with lag-driven split H2D (two copy streams): GPU tests, then the 100 GB
# overlapped bench at split leads 2 (default), 1, 4 and off
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest_r3ah.log 2>&1 || exit $?
for lead in 2 1 4 off; do
  TPI_H2D_SPLIT_LEAD=$lead timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-latency --broadcast-gb 0 --no-async > gpurun_out/bench100_lead${lead}_r3ah.json 2> gpurun_out/bench100_lead${lead}_r3ah.err || exit $?
done
