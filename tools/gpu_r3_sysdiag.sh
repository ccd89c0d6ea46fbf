#!/bin/bash
set -u
O=gpurun_out/r3sd
mkdir -p $O
for v in "peer Y" "dist Y" "peer N"; do
  set -- $v
  timeout -k 10 150 python tools/diag_system_topk.py $1 $2 > $O/diag_$1_$2.log 2>&1; rc=$?
  echo "== $1 $2 rc=$rc $(grep RESULT $O/diag_$1_$2.log)" >> $O/summary.txt
  grep -E "failed|Exception|flag|Traceback" $O/diag_$1_$2.log | head -8 >> $O/summary.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
echo done >> $O/summary.txt
