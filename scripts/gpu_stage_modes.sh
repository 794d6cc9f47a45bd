set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python scripts/exp/stage_modes.py > gpurun_out/stage_modes.json 2>gpurun_out/stage_modes.err; echo rc=$?; cat gpurun_out/stage_modes.json
DIR=/dev/shm timeout -k 10 300 python scripts/exp/stage_modes.py > gpurun_out/stage_modes_shm.json 2>>gpurun_out/stage_modes.err; echo rc=$?; cat gpurun_out/stage_modes_shm.json
