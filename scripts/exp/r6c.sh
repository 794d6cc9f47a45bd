#!/bin/bash
# round 6, call C: KFD per-process accounting probe, the changed GPU tests (stuck-import
# fallback oracle, preload GPU warm-up by evidence), then the driver's bench command with the
# product gates (GPU settle on orphaned VRAM, hand-off device check) and config 2.
set -o pipefail
O=gpurun_out/r6c
mkdir -p $O
export TMPDIR=/tmp
{
  ls -la /sys/class/kfd/kfd/proc 2>&1 | head -20
  for d in /sys/class/kfd/kfd/proc/*; do echo "$d: $(ls $d 2>&1 | tr '\n' ' ')"; done 2>&1 | head -10
  for n in /sys/class/kfd/kfd/topology/nodes/*; do
    echo "$n gpu_id=$(cat $n/gpu_id 2>&1) $(grep -E 'location_id|domain|gfx_target' $n/properties 2>/dev/null | tr '\n' ' ')"
  done
  python -c "
import sys; sys.path.insert(0, '.')
from terraform_provider_iterative_amd.parallel.placement import discover, kfd_gpu_id, orphaned_vram
for g in discover():
    print(g.to_json(), 'gpu_id', kfd_gpu_id(g.pci), orphaned_vram(g.pci))
"
} > $O/kfd_probe.txt 2>&1
cat $O/kfd_probe.txt | tail -8
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    "tests/test_gpu_kernels.py::test_a_stuck_ipc_import_falls_back_to_the_host_copy_on_hardware" \
    "tests/test_gpu_runtime.py::test_preempted_training_resumes_in_a_preloaded_successor_on_gpu" \
    -s > $O/pytest.txt 2>&1
rc=$?
tail -4 $O/pytest.txt
echo "pytest rc $rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?
tail -12 $O/bench.err
exit $rc
