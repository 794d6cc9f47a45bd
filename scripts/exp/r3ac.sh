mkdir -p gpurun_out
python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())" > gpurun_out/interf_r3ac.log 2>&1
for p in low normal high; do TPI_ENGINE_PRIORITY=$p timeout -k 10 300 python scripts/exp/async_interference.py 32 8192 256 >> gpurun_out/interf_r3ac.log 2>&1 || exit $?; done
