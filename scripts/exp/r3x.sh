mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest_r3x.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_default_r3x.json 2> gpurun_out/bench_default_r3x.err || exit $?
TPI_HBM_HANDOFF=0 timeout -k 10 300 python bench/bench_preempt.py --gb 100 --hot > gpurun_out/preempt_stream_r3x.json 2> gpurun_out/preempt_stream_r3x.err
