set -o pipefail; mkdir -p gpurun_out; timeout -k 10 300 python scripts/exp/zerocopy_stage.py > gpurun_out/exp_zc.txt 2>&1; echo rc=$?; cat gpurun_out/exp_zc.txt | tail -5
