# Round 1 GPU pass 2: device discovery diagnostics, gpu tests, latency, config 2, headline.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
{ env | grep -E "VISIBLE|ROCR|HIP_|HSA_" ; ls /sys/class/kfd/kfd/topology/nodes; for n in /sys/class/kfd/kfd/topology/nodes/*; do echo "$n $(grep -E 'gfx_target_version|drm_render_minor' $n/properties | tr '\n' ' ')"; done; ls -la /dev/dri; df -h /tmp . ; } > gpurun_out/discovery.txt 2>&1
python -c "from terraform_provider_iterative_amd.parallel.placement import discover; print([g.to_json() for g in discover()])" >> gpurun_out/discovery.txt 2>&1
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 300 python -m terraform_provider_iterative_amd.bench_latency > gpurun_out/latency.json 2>gpurun_out/latency.err && echo LAT_OK &&
timeout -k 10 900 python bench/bench_workdir.py --gb 10 --steps 20 > gpurun_out/workdir_10g.json 2>gpurun_out/workdir_10g.err && echo WD_OK &&
timeout -k 10 900 python bench.py > gpurun_out/bench_default.json 2>gpurun_out/bench_default.err && echo BENCH_OK
