#!/bin/bash
# round 6, call A: the GPU suite (new: stuck-import fallback, 2.6 GB staged attach), then the
# HIP IPC runtime matrix -- the matrix only after a clean suite.
set -o pipefail
O=gpurun_out/r6a
mkdir -p $O
export TMPDIR=/tmp
python -c "import torch; print(torch.__version__, torch.version.hip)" > $O/env.txt 2>&1
timeout -k 10 840 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $O/pytest.txt 2>&1
rc=$?
tail -5 $O/pytest.txt
echo "pytest rc $rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u scripts/exp/ipc_runtime.py --out $O/ipc_runtime > $O/ipc_runtime.txt 2>&1
rc=$?
cat $O/ipc_runtime.txt | cut -c1-300
exit $rc
