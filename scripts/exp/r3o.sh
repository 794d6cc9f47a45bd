mkdir -p gpurun_out
for i in 1 2 3; do timeout -k 10 200 python bench/bench_workdir.py --gb 10 > gpurun_out/config2_r3o_$i.json 2> gpurun_out/config2_r3o_$i.err || exit $?; done
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --durations=10 --timeout 200 --timeout-method thread > gpurun_out/gputest_r3o.log 2>&1
