#!/bin/bash
# One runner for every job sent to an MI355X box with gpurun:
#
#   gpurun --timeout 1200 -- 'bash scripts/gpu.sh tests smoke bench'
#
# Jobs run in the order given; each has its own time limit and writes its log under
# gpurun_out/<job>.log (JSON results to gpurun_out/<job>.json).  The chain stops at the first
# job that fails, times out or crashes: nothing more touches the GPU after that.
#
#   tests        pytest -m gpu (one process, per-test timeout)
#   smoke        __graft_entry__.smoke()
#   bench        python bench.py (the driver's headline defaults)
#   bench16      bench.py on a 16 GB checkpoint (quick A/B)
#   prof         rocprofv3 --kernel-trace --stats of bench16 + rocpd summary
#   pmc-codec    PMC pass over the codec kernels alone (one counter block per run)
#   kernels      bench/bench_kernels.py (device kernel GB/s)
#   workdir      bench/bench_workdir.py --gb 10 (config 2: the runtime stages the workdir
#                into HBM before train.py starts; GPU_ARGS_workdir="--stage off" = library path)
#   preempt      bench/bench_preempt.py --gb 100 (config 4 end to end)
#   preempt-standby  the same with a warm standby successor (TPI_WARM_STANDBY=1)
#   preempt-hot  hot standby (started with the rank) restoring behind the streamed spill
#   preempt-170  the hot-standby run with a 170 GB rank (more than half of HBM)
#   preempt-170m the same with the successor materializing its state group by group
#   reclaim      bench/bench_reclaim.py --gb 100 (an on-demand task takes a spot task's GPU)
#   handoff      bench/bench_handoff.py --gb 16 (same-GPU HBM hand-off alone, per copy route)
#   async        bench/bench_async.py --gb 100
#   concurrent   bench/bench_concurrent.py (config 5)
#   rehearse     bench.py at 2 and 4 ranks sharing the one GPU (gloo control plane)
#
# Extra arguments for a job: GPU_ARGS_<job>="..." (e.g. GPU_ARGS_bench="--steps 5").
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"

args() { local v="GPU_ARGS_${1//-/_}"; echo "${!v}"; }

run_job() {
  local job=$1 extra
  extra=$(args "$job")
  case "$job" in
    tests) timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 \
             --timeout-method thread -p no:cacheprovider $extra > "$OUT/tests.log" 2>&1 ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" \
             > "$OUT/smoke.log" 2>&1 ;;
    bench) timeout -k 10 900 python bench.py $extra > "$OUT/bench.json" 2> "$OUT/bench.log" ;;
    bench16) timeout -k 10 600 python bench.py --total-gb 16 --steps 3 --warmup 1 $extra \
               > "$OUT/bench16.json" 2> "$OUT/bench16.log" ;;
    prof) timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- \
            python3 bench.py --total-gb 16 --steps 2 --warmup 1 --no-latency $extra \
            > "$OUT/prof.log" 2>&1 &&
          python3 scripts/rocpd_summary.py "$(find "$OUT/prof" -name 'run_results.db' | head -1)" \
            > "$OUT/prof_summary.md" 2>&1 ;;
    pmc-codec) timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS \
                 SQ_INSTS_FLAT SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU \
                 --kernel-trace --stats -d "$OUT/pmc_codec" -o run -- \
                 python3 scripts/exp/codec_only.py > "$OUT/pmc-codec.log" 2>&1 ;;
    kernels) timeout -k 10 600 python bench/bench_kernels.py $extra \
               > "$OUT/kernels.json" 2> "$OUT/kernels.log" ;;
    workdir) timeout -k 10 900 python bench/bench_workdir.py --gb 10 $extra \
               > "$OUT/workdir.json" 2> "$OUT/workdir.log" ;;
    preempt) timeout -k 10 900 python bench/bench_preempt.py --gb 100 $extra \
               > "$OUT/preempt.json" 2> "$OUT/preempt.log" ;;
    preempt-standby) timeout -k 10 900 python bench/bench_preempt.py --gb 100 --standby $extra \
                       > "$OUT/preempt-standby.json" 2> "$OUT/preempt-standby.log" ;;
    preempt-hot) timeout -k 10 900 python bench/bench_preempt.py --gb 100 --hot $extra \
                   > "$OUT/preempt-hot.json" 2> "$OUT/preempt-hot.log" ;;
    preempt-hot2) timeout -k 10 900 python bench/bench_preempt.py --gb 100 --hot $extra \
                   > "$OUT/preempt-hot2.json" 2> "$OUT/preempt-hot2.log" ;;
    preempt-170) timeout -k 10 900 python bench/bench_preempt.py --gb 170 --hot $extra \
                   > "$OUT/preempt-170.json" 2> "$OUT/preempt-170.log" ;;
    preempt-170m) timeout -k 10 900 python bench/bench_preempt.py --gb 170 --hot --materialize \
                    $extra > "$OUT/preempt-170m.json" 2> "$OUT/preempt-170m.log" ;;
    reclaim) timeout -k 10 900 python bench/bench_reclaim.py --gb 100 $extra \
               > "$OUT/reclaim.json" 2> "$OUT/reclaim.log" ;;
    handoff) timeout -k 10 600 python bench/bench_handoff.py $extra \
               > "$OUT/handoff.json" 2> "$OUT/handoff.log" ;;
    async) timeout -k 10 900 python bench/bench_async.py --gb 100 $extra \
             > "$OUT/async.json" 2> "$OUT/async.log" ;;
    concurrent) timeout -k 10 600 python bench/bench_concurrent.py $extra \
                  > "$OUT/concurrent.json" 2> "$OUT/concurrent.log" ;;
    rehearse)
      for n in 2 4; do
        TPI_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
          --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29630 + n)) bench.py \
          --gpus $n --total-gb 8 --steps 2 --warmup 1 --broadcast-gb 0 $extra \
          > "$OUT/rehearse_n$n.json" 2> "$OUT/rehearse_n$n.log" || return 1
      done ;;
    hostinfo) { for n in /sys/devices/system/node/node*; do
                  echo "$(basename $n) cpus=$(cat $n/cpulist) $(grep -E 'MemTotal|MemFree|FilePages|Shmem:' $n/meminfo | awk '{printf "%s=%s%s ", $3, $4, $5}')"
                done
                grep -E 'MemTotal|MemAvailable|Shmem:|HugePages_Total|Hugepagesize' /proc/meminfo
                echo "shmem THP: $(cat /sys/kernel/mm/transparent_hugepage/shmem_enabled 2>/dev/null)"
                echo "anon THP: $(cat /sys/kernel/mm/transparent_hugepage/enabled 2>/dev/null)"
                df -h /dev/shm /tmp; } > "$OUT/hostinfo.txt" 2>&1 ;;
    *) echo "unknown job: $job" >&2; return 2 ;;
  esac
}

for job in "$@"; do
  start=$(date +%s)
  run_job "$job"
  rc=$?
  echo "job $job rc=$rc $(( $(date +%s) - start ))s"
  [ $rc -eq 0 ] || exit $rc
done
