mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gputest_r3ae.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r3ae.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_default_r3ae.json 2> gpurun_out/bench_default_r3ae.err
