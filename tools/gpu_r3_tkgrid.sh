#!/bin/bash
# top-k: tests (pick fused into the histogram kernel and not), then A/B on bench_compress.py
set -u
O=gpurun_out/r3tk4
mkdir -p $O
for fp in 1 0; do
  FEDMI_TK_FUSE_PICK=$fp timeout -k 10 300 python -u -m pytest tests/test_flat_ops_gpu.py -q -x -k "topk" --timeout 200 --timeout-method thread > $O/tests_fp$fp.log 2>&1; rc=$?
  echo "topk tests fuse_pick=$fp rc=$rc $(tail -1 $O/tests_fp$fp.log)" >> $O/summary.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
done
for v in "512 1" "512 0" "1024 1"; do
  set -- $v
  FEDMI_TK_CBLOCKS=$1 FEDMI_TK_FUSE_PICK=$2 timeout -k 10 120 python tools/bench_compress.py > $O/c$1_fp$2.log 2>&1; rc=$?
  echo "c=$1 fuse_pick=$2 rc=$rc $(python3 -c "
import json
for l in open('$O/c$1_fp$2.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['payload'], d['topk_us'], end='  ')
")" >> $O/summary.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
done
