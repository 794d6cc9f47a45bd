# Round 1 GPU pass 5: config 2 (10 GB workdir) after the piece split, full GPU suite, smoke.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python bench/bench_workdir.py --gb 10 --steps 20 > gpurun_out/workdir_10g_e.json 2>gpurun_out/workdir_10g_e.err && echo WD_OK &&
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu_e.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_e.log 2>&1 && echo SMOKE_OK
