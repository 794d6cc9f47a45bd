set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rocm-smi --showtopo > gpurun_out/topo.txt 2>&1 || true
nproc > gpurun_out/sysinfo.txt; free -g >> gpurun_out/sysinfo.txt; cat /sys/kernel/mm/transparent_hugepage/enabled >> gpurun_out/sysinfo.txt 2>&1; df -h /dev/shm >> gpurun_out/sysinfo.txt 2>&1; ulimit -l >> gpurun_out/sysinfo.txt
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 300 python bench.py --total-gb 8 --steps 3 --warmup 1 --no-latency > gpurun_out/bench_8g.log 2>&1 && echo B8_OK &&
timeout -k 10 300 python bench.py --total-gb 8 --steps 3 --warmup 1 --no-latency --mode direct > gpurun_out/bench_8g_direct.log 2>&1 && echo B8D_OK &&
timeout -k 10 900 python bench.py --no-latency > gpurun_out/bench_100g.log 2>&1 && echo B100_OK
