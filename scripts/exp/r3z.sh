# Multi-rank rehearsal on the one-GPU box: gloo ranks sharing the GPU run bench.py's N>1 path
# (launcher contract, allmax over ranks, per-rank spill regions, fan-out side measurement off).
mkdir -p gpurun_out
for n in 2 4; do
  TPI_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2955$n bench.py --gpus $n --total-gb 16 --steps 2 --warmup 1 > gpurun_out/rehearsal_n${n}_r3z.json 2> gpurun_out/rehearsal_n${n}_r3z.err || exit $?
done
