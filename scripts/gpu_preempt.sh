# Config 4 end to end on one MI355X: leo preempt -> spill -> respawn -> restore (bench_preempt).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
df -h /dev/shm /tmp > gpurun_out/df.txt 2>&1; free -g >> gpurun_out/df.txt 2>&1; cat gpurun_out/df.txt
SHM_GB=$(df -BG --output=avail /dev/shm | tail -1 | tr -dc 0-9)
GB=100; DIR=/dev/shm
if [ "${SHM_GB:-0}" -lt 120 ]; then DIR=/tmp; GB=16; fi
echo "spill dir $DIR (shm avail ${SHM_GB}G)"
timeout -k 10 300 python bench/bench_preempt.py --gb 8 --spill-dir $DIR > gpurun_out/preempt_8g.json 2> gpurun_out/preempt_8g.err && echo P8_OK && cat gpurun_out/preempt_8g.json &&
timeout -k 10 600 python bench/bench_preempt.py --gb $GB --spill-dir $DIR > gpurun_out/preempt_100g.json 2> gpurun_out/preempt_100g.err && echo P100_OK && cat gpurun_out/preempt_100g.json
