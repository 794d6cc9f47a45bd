#!/bin/bash
# round 6, call T: the workdir push's copy methods on the box's /tmp (CPU only, no GPU use):
# 10 x 1 GB files, copy_file_range pieces vs writes through a shared mapping of the destination.
set -o pipefail
O=gpurun_out/r6t
mkdir -p $O
export TMPDIR=/tmp
B=$(mktemp -d /tmp/tpi-pushexp-XXXX)
mkdir -p $B/src $B/dst
python3 -c "
import os
blk = os.urandom(64 << 20)
for i in range(10):
    with open('$B/src/f%d.bin' % i, 'wb') as f:
        for _ in range(16):
            f.write(blk)
"
nproc > $O/nproc.txt; python3 -c "import os; print(len(os.sched_getaffinity(0)))" >> $O/nproc.txt
df -T /tmp >> $O/nproc.txt
for m in cfr mmap mmap_pop cfr; do
  for t in 10 16 32; do
    for p in 256 64; do
      rm -f $B/dst/*
      timeout -k 5 60 scripts/exp/push_exp $B/src $B/dst 10 $t $p $m >> $O/push.jsonl || { rm -rf $B; exit 1; }
    done
  done
done
cmp $B/src/f9.bin $B/dst/f9.bin && echo "last copy identical" >> $O/push.jsonl
rm -rf $B
cat $O/push.jsonl
