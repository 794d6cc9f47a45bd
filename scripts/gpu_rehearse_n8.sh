# 8 ranks sharing one MI355X (gloo control plane), the full 100 GB split 8 ways: checks the
# N=8 flow, host/HBM memory footprint and teardown.  Not a performance number (one PCIe link).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TPI_BENCH_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29641 bench.py --gpus 8 --steps 2 --warmup 1 --broadcast-gb 0 > gpurun_out/rehearse_n8.log 2>&1 && echo N8_OK; tail -1 gpurun_out/rehearse_n8.log | cut -c1-300
