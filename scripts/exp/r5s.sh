#!/bin/bash
# Round 5: the N=2 bench flow on the 1-GPU box (two ranks share the GPU over gloo: everything
# but RCCL), to check the multi-rank path of bench.py after this round's changes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5s
mkdir -p $O
cd $R
TPI_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 \
  > $O/bench_n2_gloo.json 2> $O/bench_n2_gloo.log
rc=$?
tail -5 $O/bench_n2_gloo.log
grep '^{' $O/bench_n2_gloo.json | tail -1 | cut -c1-1500
exit $rc
