set -o pipefail; mkdir -p gpurun_out; timeout -k 10 600 python scripts/exp/teardown.py > gpurun_out/exp_teardown.json 2>&1 && echo EXP_OK; cat gpurun_out/exp_teardown.json
