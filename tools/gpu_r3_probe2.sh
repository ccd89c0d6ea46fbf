#!/bin/bash
# stats probes (unbuffered client logs) + densenet fused/unfused diff per parameter under the fast-path switches
set -u
O=gpurun_out/r3p2
mkdir -p $O
PYTHONUNBUFFERED=1 FEDMI_DEBUG_STATS=1 DIAG_TAIL=200 timeout -k 10 150 python -u tools/diag_system_topk.py peer Y > $O/diag_probe.log 2>&1; rc=$?
echo "probe rc=$rc" > $O/summary.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in "1 1" "1 0" "0 0"; do
  set -- $v
  FEDMI_ZOO_FAST=$1 FEDMI_ZOO_FAST_PAD=$2 timeout -k 10 120 python -u tools/diag_fusion_exact.py densenet_cifar > $O/fx_$1$2.log 2>&1; rc=$?
  echo "fast=$1 pad=$2 rc=$rc $(tail -1 $O/fx_$1$2.log)" >> $O/summary.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
done
