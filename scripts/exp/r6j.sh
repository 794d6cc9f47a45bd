#!/bin/bash
# round 6, call J: the driver's N>1 bench flow rehearsed on one MI355X with the final tree --
# 2 and 4 ranks sharing the GPU over gloo (RCCL needs one GPU per rank), strong scaling, so
# the control flow of the 8-GPU run (rank-0 side measurements, barriers, max over ranks,
# per-rank restore verification) runs on hardware with round 6's gates in place.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6j
mkdir -p $O
cd $R
export TMPDIR=/tmp TPI_BENCH_BACKEND=gloo
for n in 2 4; do
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 2 \
      --warmup 1 > $O/rehearse_n$n.json 2> $O/rehearse_n$n.err
  rc=$?
  tail -c 600 $O/rehearse_n$n.json; echo; echo "n=$n rc $rc"
  [ $rc -eq 0 ] || exit $rc
done
