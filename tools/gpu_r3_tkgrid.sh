#!/bin/bash
# top-k: tests under each path switch, then A/B on bench_compress.py
set -u
O=gpurun_out/r3tk5
mkdir -p $O
for v in "1 1" "0 1" "1 0"; do
  set -- $v
  FEDMI_TK_SMALL=$1 FEDMI_TK_FUSE_PICK=$2 timeout -k 10 300 python -u -m pytest tests/test_flat_ops_gpu.py -q -x -k "topk" --timeout 200 --timeout-method thread > $O/tests_s$1_fp$2.log 2>&1; rc=$?
  echo "topk tests small=$1 fuse_pick=$2 rc=$rc $(tail -1 $O/tests_s$1_fp$2.log)" >> $O/summary.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
done
for v in "1 1" "0 1" "0 0"; do
  set -- $v
  FEDMI_TK_SMALL=$1 FEDMI_TK_FUSE_PICK=$2 timeout -k 10 120 python tools/bench_compress.py > $O/s$1_fp$2.log 2>&1; rc=$?
  echo "small=$1 fuse_pick=$2 rc=$rc $(python3 -c "
import json
for l in open('$O/s$1_fp$2.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['payload'], d['topk_us'], end='  ')
")" >> $O/summary.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
done
