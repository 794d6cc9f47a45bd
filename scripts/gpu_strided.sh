set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench/bench_strided.py > gpurun_out/strided.log 2>&1 && echo STRIDED_OK
