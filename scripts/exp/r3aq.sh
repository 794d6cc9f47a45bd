# Round-3 final measurements with the current tree: GPU tests + smoke, the driver's default
# bench, config 4 (100 GB HBM hand-off, streamed route, 150 GB), config 2, kernel rates,
# multi-rank rehearsal, config 5 logical slots, and a kernel-trace profile of a 16 GB step
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu.sh tests smoke bench kernels workdir concurrent || exit $?
timeout -k 10 600 python bench/bench_preempt.py --gb 100 --hot > gpurun_out/preempt_hot_r3aq.json 2> gpurun_out/preempt_hot_r3aq.err || exit $?
TPI_HBM_HANDOFF=0 timeout -k 10 600 python bench/bench_preempt.py --gb 100 --hot > gpurun_out/preempt_stream_r3aq.json 2> gpurun_out/preempt_stream_r3aq.err || exit $?
timeout -k 10 600 python bench/bench_preempt.py --gb 150 --hot > gpurun_out/preempt_150_r3aq.json 2> gpurun_out/preempt_150_r3aq.err || exit $?
bash scripts/gpu.sh rehearse prof
