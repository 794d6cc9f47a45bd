set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_examples.py tests/test_gpu_runtime.py tests/test_task_smoke.py -m gpu -q -x > gpurun_out/pytest_examples.log 2>&1 && echo EX_OK
