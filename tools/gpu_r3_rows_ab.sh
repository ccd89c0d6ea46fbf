#!/bin/bash
# zoo: native-mode GPU tests, then the BN row pass rows-per-lane A/B on the graph-replayed steps
set -u
O=gpurun_out/r3ra
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_native_mode_gpu.py -q -x --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "native_mode tests rc=$rc $(tail -1 $O/tests.log)" >> $O/summary.txt
if [ $rc -ne 0 ]; then exit $rc; fi
BENCH_MODES=fp32 timeout -k 10 300 python tools/bench_hybrid.py densenet_cifar RegNetY_400MF > $O/fp32.jsonl 2>$O/fp32.err || exit $?
for rpl in 16 4 8; do
  FEDMI_ROWS_PER_LANE=$rpl BENCH_MODES=native-graph timeout -k 10 300 python tools/bench_hybrid.py densenet_cifar RegNetY_400MF > $O/rpl$rpl.jsonl 2>$O/rpl$rpl.err; rc=$?
  echo "rows_per_lane=$rpl rc=$rc $(python3 -c "
import json
for l in open('$O/rpl$rpl.jsonl'):
    d=json.loads(l); print(d['model'], d['ms_per_step'], end='  ')
")" >> $O/summary.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
done
cat $O/fp32.jsonl >> $O/summary.txt
