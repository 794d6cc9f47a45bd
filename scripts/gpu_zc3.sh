set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do timeout -k 10 900 python bench/bench_workdir.py --gb 10 --steps 20 > gpurun_out/workdir_10g_zc3_$i.json 2>gpurun_out/workdir_10g_zc3_$i.err && cat gpurun_out/workdir_10g_zc3_$i.json || exit 1; done
