set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python bench.py > gpurun_out/bench_i.log 2>&1 && echo BENCH_OK && tail -1 gpurun_out/bench_i.log | cut -c1-200 &&
TPI_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29636 bench.py --gpus 2 --total-gb 4 --steps 2 --warmup 1 --broadcast-gb 0.5 > gpurun_out/rehearse_bcast2.log 2>&1 && echo BC_OK && tail -1 gpurun_out/rehearse_bcast2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['save_async'], json.dumps(d['workdir_broadcast'])[:300])"
