#!/bin/bash
# top-k below the 3-level threshold: exact select in the compaction's last workgroup vs its own launch
set -u
O=gpurun_out/r3tk6
mkdir -p $O
for fs in 1 0; do
  FEDMI_TK_FUSE_SELECT=$fs timeout -k 10 300 python -u -m pytest tests/test_flat_ops_gpu.py tests/test_system_gpu.py -q -x -k "topk" --timeout 200 --timeout-method thread > $O/tests_fs$fs.log 2>&1; rc=$?
  echo "topk tests fuse_select=$fs rc=$rc $(tail -1 $O/tests_fs$fs.log)" >> $O/summary.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
done
for fs in 1 0 1 0; do
  FEDMI_TK_FUSE_SELECT=$fs timeout -k 10 120 python tools/bench_compress.py > $O/b_fs$fs.log 2>&1; rc=$?
  echo "fuse_select=$fs rc=$rc $(python3 -c "
import json
for l in open('$O/b_fs$fs.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['payload'], d['topk_us'], end='  ')
")" >> $O/summary.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
done
