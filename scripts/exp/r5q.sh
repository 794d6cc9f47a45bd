#!/bin/bash
# Round 5: the HBM copy ceiling (HIP D2D vs the hand-off kernels), and whether a per-rank
# memory cap can be had on this box without a writable cgroup (systemd-run --user --scope).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5q
mkdir -p $O
cd $R
timeout -k 10 200 python -u scripts/exp/d2d_ceiling.py 50 > $O/d2d_ceiling.jsonl 2> $O/d2d_ceiling.log || { tail -20 $O/d2d_ceiling.log; exit 1; }
cat $O/d2d_ceiling.jsonl
{
  echo "== id"; id
  echo "== cgroup"; cat /proc/self/cgroup
  echo "== mount"; grep cgroup /proc/mounts || true
  echo "== cgroup dir writable?"; d=/sys/fs/cgroup$(cut -d: -f3 /proc/self/cgroup | head -1); ls -ld "$d" 2>&1; touch "$d/x" 2>&1 || true
  echo "== systemd-run"; command -v systemd-run || echo none
  timeout 10 systemd-run --user --scope -p MemoryMax=100M true 2>&1 || echo "systemd-run rc=$?"
  echo "== XDG_RUNTIME_DIR=$XDG_RUNTIME_DIR DBUS=$DBUS_SESSION_BUS_ADDRESS"
  echo "== prlimit"; command -v prlimit || echo none
} > $O/memcap_probe.txt 2>&1
cat $O/memcap_probe.txt
