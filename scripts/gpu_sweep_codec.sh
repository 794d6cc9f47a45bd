# Tile / chunk / ring-depth sweep of the TPZ1 checkpoint pipeline (32 GB, 1 GPU).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/sweep_codec.log
run() {
  echo "== $*" >> gpurun_out/sweep_codec.log
  timeout -k 10 240 python bench.py --total-gb 32 --steps 3 --warmup 1 --no-latency "$@" >> gpurun_out/sweep_codec.log 2>&1
}
run --tile-mb 1 --chunk-mb 256 --nbuf 3 &&
run --tile-mb 0.25 --chunk-mb 256 --nbuf 3 &&
run --tile-mb 4 --chunk-mb 256 --nbuf 3 &&
run --tile-mb 1 --chunk-mb 64 --nbuf 3 &&
run --tile-mb 1 --chunk-mb 128 --nbuf 3 &&
run --tile-mb 1 --chunk-mb 512 --nbuf 3 &&
run --tile-mb 1 --chunk-mb 256 --nbuf 2 &&
run --tile-mb 1 --chunk-mb 256 --nbuf 4 &&
run --tile-mb 1 --chunk-mb 256 --nbuf 3 --codec none &&
echo SWEEP_OK
