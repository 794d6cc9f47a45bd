# Round 1 GPU pass 3: tests (incl. incremental sync), smoke, kernels, torchrun path.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 300 python bench/bench_kernels.py --gb 8 > gpurun_out/kernels.log 2>&1 && echo KERNELS_OK &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 1 --total-gb 8 --steps 2 --warmup 1 > gpurun_out/torchrun1.log 2>&1 && echo TORCHRUN_OK
