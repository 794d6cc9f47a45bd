mkdir -p gpurun_out
timeout -k 10 200 ./scripts/exp/duplex 4 > gpurun_out/duplex_r3m.log 2>&1 || exit $?
for i in 1 2 3; do timeout -k 10 200 python bench/bench_workdir.py --gb 10 > gpurun_out/config2_r3m_$i.json 2> gpurun_out/config2_r3m_$i.err || exit $?; done
