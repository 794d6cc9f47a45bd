# Eight ranks on the one-GPU box (gloo control plane, ranks share the GPU): bench.py's N = 8
# path through torch.distributed.run and through its own launcher
mkdir -p gpurun_out
TPI_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29678 bench.py --gpus 8 --total-gb 8 --steps 2 --warmup 1 --broadcast-gb 0 > gpurun_out/rehearse_n8_torchrun_r3av.json 2> gpurun_out/rehearse_n8_torchrun_r3av.err || exit $?
TPI_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 8 --total-gb 8 --steps 2 --warmup 1 --broadcast-gb 0 > gpurun_out/rehearse_n8_self_r3av.json 2> gpurun_out/rehearse_n8_self_r3av.err
