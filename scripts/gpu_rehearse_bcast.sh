# 2-rank rehearsal incl. the fan-out side measurements (broadcast, scatter+allgather,
# independent H2D) on a 1-GPU box over gloo.  Flow check only.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TPI_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29635 bench.py --gpus 2 --total-gb 4 --steps 2 --warmup 1 --broadcast-gb 1 > gpurun_out/rehearse_bcast.log 2>&1 && echo BC_OK; tail -1 gpurun_out/rehearse_bcast.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d['workdir_broadcast']), d['value'])"
