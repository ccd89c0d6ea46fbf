#!/bin/bash
# top-k grid caps A/B (compaction / histogram workgroup counts) on bench_compress.py
set -u
O=gpurun_out/r3tk
mkdir -p $O
for v in "2048 2048" "1024 2048" "512 2048" "256 2048" "2048 1024" "2048 512"; do
  set -- $v
  FEDMI_TK_CBLOCKS=$1 FEDMI_TK_HBLOCKS=$2 timeout -k 10 120 python tools/bench_compress.py > $O/c$1_h$2.log 2>&1; rc=$?
  echo "c=$1 h=$2 rc=$rc $(python3 -c "
import json,sys
for l in open('$O/c$1_h$2.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['payload'], d['topk_us'], end='  ')
")" >> $O/summary.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
done
