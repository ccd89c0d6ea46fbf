#!/bin/bash
set -u
O=gpurun_out/r3p3
mkdir -p $O
for fz in 1 0; do
  FEDMI_ZOO_FAST=$fz timeout -k 10 200 python -u -m pytest tests/test_native_mode_gpu.py -q -x -k premasked --timeout 120 --timeout-method thread > $O/pm_$fz.log 2>&1; rc=$?
  echo "premasked fast=$fz rc=$rc $(tail -1 $O/pm_$fz.log)" >> $O/summary.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
PYTHONUNBUFFERED=1 FEDMI_DEBUG_STATS=1 DIAG_TAIL=200 timeout -k 10 150 python -u tools/diag_system_topk.py peer Y > $O/diag_probe.log 2>&1; rc=$?
echo "probe rc=$rc" >> $O/summary.txt
