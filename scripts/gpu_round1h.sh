# Round 1 (late) GPU pass: full GPU suite, smoke, default headline bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_h.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_h.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 900 python bench.py > gpurun_out/bench_h.log 2>&1 && echo BENCH_OK && tail -1 gpurun_out/bench_h.log | cut -c1-400
