#!/bin/bash
# round 6, call V: the push's copy_file_range piece size and thread count on the box's /tmp
# (CPU only): 10 x 1 GB files, 5 interleaved repetitions of each setting.
set -o pipefail
O=gpurun_out/r6v
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
for r in 1 2 3 4 5; do
  for t in 16 24; do
    for p in 32 64 128 256; do
      rm -f $B/dst/*
      timeout -k 5 60 scripts/exp/push_exp $B/src $B/dst 10 $t $p cfr >> $O/push.jsonl || { rm -rf $B; exit 1; }
    done
  done
done
rm -rf $B
python3 -c "
import json, statistics as st, collections
d = collections.defaultdict(list)
for l in open('$O/push.jsonl'):
    j = json.loads(l); d[(j['threads'], j['piece_mib'])].append(j['GBps'])
for k in sorted(d): print(k, 'median %.1f' % st.median(d[k]), sorted(d[k]))
" | tee $O/summary.txt
