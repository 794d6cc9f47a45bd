# Round 1 GPU pass: full GPU suite, smoke, default headline bench (100 GB, codec).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu_f.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_f.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 900 python bench.py > gpurun_out/bench_f.log 2>&1 && echo BENCH_OK
