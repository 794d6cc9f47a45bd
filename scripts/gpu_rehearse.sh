# Multi-rank rehearsal of bench.py on a 1-GPU box (ranks share cuda:0; gloo control plane,
# RCCL cannot put two ranks on one GPU).  Flow check only, not a performance number.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TPI_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29633 bench.py --gpus 2 --total-gb 8 --steps 2 --warmup 1 --broadcast-gb 0 > gpurun_out/rehearse_n2.log 2>&1 && echo N2_OK &&
TPI_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29634 bench.py --gpus 4 --total-gb 8 --steps 2 --warmup 1 --broadcast-gb 0 > gpurun_out/rehearse_n4.log 2>&1 && echo N4_OK &&
timeout -k 10 900 python bench/bench_workdir.py --gb 10 --steps 20 > gpurun_out/workdir_10g_huf.json 2>gpurun_out/workdir_10g_huf.err && echo WD_OK
